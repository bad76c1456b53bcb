#!/bin/bash
# round 4 closing check on HEAD (after the GELU+Q8_K position change): whole GPU suite + smoke + the default bench line (per-class MFMA fractions)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r04x_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04x_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r04x_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python3 bench.py > gpurun_out/r04x_bench_q4k64.json 2> gpurun_out/r04x_bench.err || { tail -5 gpurun_out/r04x_bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v.get('mfma_frac') for k, v in d['per_kernel'].items()})" gpurun_out/r04x_bench_q4k64.json
