#!/bin/bash
# round 4: fp8 QK^T correction terms — whole GPU suite with every parity number
# logged, the backend tiny variants, the default bench line (conv cost)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/r04l_parity_log.jsonl
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -25 gpurun_out/r04l_tests.log | cut -c1-400
case $rc in 0|1) ;; *) exit 1;; esac
unset Q2A_PARITY_LOG
timeout -k 10 400 python3 diag/backend_tiny_variants.py > gpurun_out/r04l_variants.jsonl 2> gpurun_out/r04l_variants.err || { tail -5 gpurun_out/r04l_variants.err; exit 1; }
cat gpurun_out/r04l_variants.jsonl
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err || { tail -5 gpurun_out/r04l_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04l_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
timeout -k 10 400 python3 bench.py --config f16x1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04l_bench_f16x1.json 2> gpurun_out/r04l_bench_f16x1.err || { tail -5 gpurun_out/r04l_bench_f16x1.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04l_bench_f16x1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
