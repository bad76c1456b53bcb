#!/bin/bash
# round 5: (1) the whole GPU suite on the product (8-wave narrow tiles adopted); (2) the fc1 -> fc2 GELU + Q8_K kernel
# on the compact |x| < 10 table with 16 waves per CU (diag/gcomp = q2a_exact.hip -DQ2A_GELU_COMPACT=1): 64-clip output
# bit-equality, the three fc1 paths' codes, then alternating 64-clip benches (quant_act ms per step).
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
Q2A_PARITY_LOG=$PWD/gpurun_out/r05f_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r05f_tests.log
case $rc in 124|137|134|139) exit 1;; esac
timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_base.npy || exit 1
Q2A_LIB_PATH=$PWD/diag/gcomp/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_gc.npy || exit 1
python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_gc.npy || exit 1
rm -f /tmp/eq_*.npy
Q2A_LIB_PATH=$PWD/diag/gcomp/libq2a.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "deferred_gelu" > gpurun_out/r05f_gcomp_tests.log 2>&1 || { tail -5 gpurun_out/r05f_gcomp_tests.log; exit 1; }
tail -1 gpurun_out/r05f_gcomp_tests.log
pk() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in sys.argv[2:]})" "$@"; }
for v in base1=$L gc1=diag/gcomp/libq2a.so base2=$L gc2=diag/gcomp/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05f_q4k64_$n.json 2> gpurun_out/r05f_q4k64_$n.err || { tail -5 gpurun_out/r05f_q4k64_$n.err; exit 1; }
  pk gpurun_out/r05f_q4k64_$n.json quant_act layernorm gemm_fc1 gemm_fc2 attention
done
