#!/bin/bash
# round 3: fused fc1 + GELU + Q8_K epilogue with LDS-staged d / bsum side outputs (diag/fc1f: fc1 path 2 by default)
# vs the product's fc1 PRE_H + separate quantizer: code identity test, then same-box A/B, alternating, two reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "deferred_gelu or block_batched" > gpurun_out/v_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/v_tests.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'fc1', pk['gemm_fc1']['ms_per_step'], 'quant', pk['quant_act']['ms_per_step'])" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in p=$L f=diag/fc1f/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/v_b_$n$i.json 2> gpurun_out/v_b_$n$i.err && s gpurun_out/v_b_$n$i.json || { tail -20 gpurun_out/v_b_$n$i.err; exit 1; }
done
done
