#!/bin/bash
# round 5: F32-class attention, five LDS stages for one-workgroup-per-CU grids, iterations force-inlined so the compiler tracks each stage's DMA (plain stage reads)
# waves per SIMD (a single clip). Tests (attention unit, batch invariance: single clip = 16-query waves, batch =
# (a single clip). Tests (attention unit, batch invariance: single clip = 5 stages, batch = 3, bit for bit), then configs[1] / Q4_K one clip / the default workload alternating against the previous
# library (diag/prev = HEAD before the change)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_ggml_backend.py tests/test_gpu_whisper_api.py > gpurun_out/r05s_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05s_tests.log
[ $rc -eq 0 ] || exit 1
pk() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in sys.argv[2:]})" "$@"; }
for cfg in f16x1 q4kx1; do
  for v in preva=diag/prev/libq2a.so newa=$L prevb=diag/prev/libq2a.so newb=$L; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-legs > gpurun_out/r05s_${cfg}_$n.json 2> gpurun_out/r05s_${cfg}_$n.err || { tail -5 gpurun_out/r05s_${cfg}_$n.err; exit 1; }
    pk gpurun_out/r05s_${cfg}_$n.json attention gemm_qkv gemm_fc1
  done
done
for v in preva=diag/prev/libq2a.so newa=$L prevb=diag/prev/libq2a.so newb=$L; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05s_q4k64_$n.json 2> gpurun_out/r05s_q4k64_$n.err || { tail -5 gpurun_out/r05s_q4k64_$n.err; exit 1; }
  pk gpurun_out/r05s_q4k64_$n.json attention gemm_qkv gemm_fc1
done
