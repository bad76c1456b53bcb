#!/bin/bash
# k_attn_g waves per workgroup: 4 (default) vs 6 vs 8 — attention parity under each, then interleaved benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for nw in 6 8; do
  Q2A_ATTN_NW=$nw timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size or batch" > gpurun_out/o_parity_$nw.log 2>&1 || { tail -30 gpurun_out/o_parity_$nw.log; exit 1; }
  tail -1 gpurun_out/o_parity_$nw.log
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  for nw in 4 6 8; do
    Q2A_ATTN_NW=$nw timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/o_nw$nw.json && s gpurun_out/o_nw$nw.json || exit 1
  done
done
