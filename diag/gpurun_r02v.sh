#!/bin/bash
# k_attn_g with Q2A_ATTN_POLY of every 16 score exponentials on the FMA pipe (exp2_poly): parity per variant, then
# interleaved same-box benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
VS="av_poly4 av_poly8 av_poly12"
for v in $VS; do
  Q2A_PARITY_LOG=$PWD/gpurun_out/v_parity_$v.jsonl Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size_vs" > gpurun_out/v_parity_$v.log 2>&1 || { tail -30 gpurun_out/v_parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/v_parity_$v.log)"
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/v_base.json && s gpurun_out/v_base.json || exit 1
  for v in $VS; do
    Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/v_$v.json && s gpurun_out/v_$v.json || exit 1
  done
done
