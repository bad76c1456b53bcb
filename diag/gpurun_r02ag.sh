#!/bin/bash
# k_attn_g lazy re-basing of the softmax max (Q2A_ATTN_LAZY=1, tau 5): full parity suite under the variant (the F16
# full-size bar is the tight one), then interleaved same-box benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/ag_parity.jsonl Q2A_LIB_PATH=diag/av_lazy/libq2a.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/ag_parity.log 2>&1 || { tail -30 gpurun_out/ag_parity.log; exit 1; }
echo "lazy parity: $(tail -1 gpurun_out/ag_parity.log)"
grep -h "full" gpurun_out/ag_parity.jsonl | head -6
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ag_base.json && s gpurun_out/ag_base.json || exit 1
  Q2A_LIB_PATH=diag/av_lazy/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ag_lazy.json && s gpurun_out/ag_lazy.json || exit 1
done
