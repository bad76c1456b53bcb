#!/bin/bash
# k_attn_g with the two 32-key QK^T chains interleaved per 16-deep step (Q2A_ATTN_KPF=1, 136 VGPRs) vs default:
# attention parity under the variant, then interleaved same-box benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_LIB_PATH=diag/av_kpf/libq2a.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or full_size_vs" > gpurun_out/ae_parity.log 2>&1 || { tail -30 gpurun_out/ae_parity.log; exit 1; }
echo "kpf parity: $(tail -1 gpurun_out/ae_parity.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ae_base.json && s gpurun_out/ae_base.json || exit 1
  Q2A_LIB_PATH=diag/av_kpf/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ae_kpf.json && s gpurun_out/ae_kpf.json || exit 1
done
