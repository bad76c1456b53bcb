#!/bin/bash
# round 3: attention on 16x16x32 MFMAs (k_attn_t, product) vs k_attn_s (diag/attn_s) vs k_attn_g (diag/attn_g):
# parity subset on the product, then same-box A/B of the default bench workload, alternating, two reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/r_parity_log.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "attention or tiny or full_size" > gpurun_out/r_tests.log 2>&1; echo "tests rc=$?"; tail -4 gpurun_out/r_tests.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'])" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in t=$L s=diag/attn_s/libq2a.so g=diag/attn_g/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r_b_$n$i.json 2> gpurun_out/r_b_$n$i.err && s gpurun_out/r_b_$n$i.json || { tail -20 gpurun_out/r_b_$n$i.err; exit 1; }
done
done
