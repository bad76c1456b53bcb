#!/bin/bash
# round 5 final sanity on HEAD (after the diag-only experiments were moved out of the product tree): whole GPU suite,
# smoke and one default bench line
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05v_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r05v_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05v_smoke.log 2>&1 || { tail -5 gpurun_out/r05v_smoke.log; exit 1; }
tail -1 gpurun_out/r05v_smoke.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/r05v_bench_q4k64.json 2> gpurun_out/r05v_bench.err || { tail -5 gpurun_out/r05v_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r05v_bench_q4k64.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
