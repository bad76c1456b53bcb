#!/bin/bash
# small-tile Q4_K back to one block-start copy (248 registers): parity + batch invariance, single-clip Q4_K, default bench
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ggml_backend.py > gpurun_out/ai_tests.log 2>&1 || { tail -30 gpurun_out/ai_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ai_tests.log)"
for c in q4kx1 q4kx1; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/ai_bench_$c.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/ai_bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['per_kernel']['gemm_qkv']['ms_per_step'])"
done
timeout -k 10 400 python3 -u bench.py > gpurun_out/ai_bench_q4k64.json 2>/dev/null || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/ai_bench_q4k64.json').read().strip().splitlines()[-1]); print('q4k64', d['value'], d['ms_per_step'], d['roofline']['frac'])"
