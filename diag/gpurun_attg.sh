#!/bin/bash
# k_attn_g (LDS-DMA K/V, 3 WGs/CU) vs k_attn: parity with Q2A_ATTN_G=1, then interleaved benches
set -e
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_ATTN_G=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "attention or full_size or tiny or batch" > gpurun_out/attg_parity.log 2>&1 || { tail -30 gpurun_out/attg_parity.log; exit 1; }
tail -2 gpurun_out/attg_parity.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/attg_base.json && s gpurun_out/attg_base.json
  Q2A_ATTN_G=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/attg_g.json && s gpurun_out/attg_g.json
done
