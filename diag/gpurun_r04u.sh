#!/bin/bash
# round 4: GELU + Q8_K kernel with its work position advanced incrementally (no 64-bit divide per iteration) against
# HEAD^ q2a_exact.hip (diag/headexact): 64-clip output bit-equality, the quantizer tests, alternating benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
H=diag/headexact/libq2a.so
timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_base.npy || exit 1
Q2A_LIB_PATH=$PWD/$H timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_head.npy || exit 1
python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_head.npy || exit 1
rm -f /tmp/eq_*.npy
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "deferred_gelu or batch_64 or block_batched or quant" > gpurun_out/r04u_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04u_tests.log; [ $rc -eq 0 ] || exit 1
for v in head1=$H new1=$L head2=$H new2=$L head3=$H new3=$L; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r04u_b_$n.json 2> gpurun_out/r04u_b_$n.err || { tail -5 gpurun_out/r04u_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], pk['quant_act']['ms_per_step'], pk['layernorm']['ms_per_step'])" gpurun_out/r04u_b_$n.json
done
