#!/bin/bash
# round 5: one-clip GEMMs all on the 64-row narrow tiles (diag/nall = -DQ2A_GEMM_NARROW_ALL=1: QKV 720 tiles, fc1 960
# instead of 360 / 480 128x128 tiles on 256 CUs). Same K order: the linear + batch-invariance tests on the variant,
# then configs[1] (f16x1) and Q4_K one clip alternating
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
Q2A_LIB_PATH=$PWD/diag/nall/libq2a.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "linear_matches or batch_invariant or batch_equals" > gpurun_out/r05o_tests.log 2>&1; rc=$?
echo "nall tests rc=$rc"; tail -2 gpurun_out/r05o_tests.log
[ $rc -eq 0 ] || exit 1
pk() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in sys.argv[2:]})" "$@"; }
for cfg in f16x1 q4kx1; do
  for v in base1=$L nalla=diag/nall/libq2a.so base2=$L nallb=diag/nall/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-legs > gpurun_out/r05o_${cfg}_$n.json 2> gpurun_out/r05o_${cfg}_$n.err || { tail -5 gpurun_out/r05o_${cfg}_$n.err; exit 1; }
    pk gpurun_out/r05o_${cfg}_$n.json gemm_qkv gemm_o gemm_fc1 gemm_fc2 attention layernorm quant_act
  done
done
