#!/bin/bash
# k_attn_pp32 (F32-class ping-pong, 32-key tiles): bit-equality with k_attn_g32 on fixed inputs, attention parity
# tests, then interleaved same-box benches against the default k_attn_g
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_ATTN_G32=1 timeout -k 10 200 python3 diag/attn_dump.py gpurun_out/w_g32.npy || exit 1
Q2A_ATTN_PP32=1 timeout -k 10 200 python3 diag/attn_dump.py gpurun_out/w_pp32.npy || exit 1
python3 -c "
import numpy as np
a=np.load('gpurun_out/w_g32.npy'); b=np.load('gpurun_out/w_pp32.npy')
print('pp32 == g32 bitwise:', np.array_equal(a,b), 'max abs diff', float(np.abs(a-b).max()), 'finite', bool(np.isfinite(b).all()))"
Q2A_ATTN_PP32=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size_vs or batch" > gpurun_out/w_parity.log 2>&1 || { tail -30 gpurun_out/w_parity.log; exit 1; }
echo "pp32 $(tail -1 gpurun_out/w_parity.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  for g in 0 1; do
    Q2A_ATTN_PP32=$g timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/w_pp32_$g.json && s gpurun_out/w_pp32_$g.json || exit 1
  done
done
