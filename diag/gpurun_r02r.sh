#!/bin/bash
# k_attn_g32 (32-key tiles, 118 VGPRs, four workgroups per CU) vs k_attn_g: attention parity under G32, then
# interleaved same-box benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_ATTN_G32=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size_vs or batch" > gpurun_out/r_parity_g32.log 2>&1 || { tail -30 gpurun_out/r_parity_g32.log; exit 1; }
echo "g32 $(tail -1 gpurun_out/r_parity_g32.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  for g in 0 1; do
    Q2A_ATTN_G32=$g timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r_g32_$g.json && s gpurun_out/r_g32_$g.json || exit 1
  done
done
