#!/bin/bash
# k_attn_g packed-f32 softmax arithmetic (Q2A_ATTN_PK=1, the built library) vs the scalar forms (diag/av_pk0):
# parity of the built library, then interleaved same-box benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size_vs or batch" > gpurun_out/z_parity.log 2>&1 || { tail -30 gpurun_out/z_parity.log; exit 1; }
echo "pk parity: $(tail -1 gpurun_out/z_parity.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  Q2A_LIB_PATH=diag/av_pk0/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/z_pk0.json && s gpurun_out/z_pk0.json || exit 1
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/z_pk1.json && s gpurun_out/z_pk1.json || exit 1
done
