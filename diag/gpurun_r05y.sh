#!/bin/bash
# round 5, second session: rebuilt tree (container re-created) — whole GPU suite + smoke + default bench line
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/r05y_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 gpurun_out/r05y_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05y_smoke.log 2>&1 || { tail -5 gpurun_out/r05y_smoke.log; exit 1; }
tail -2 gpurun_out/r05y_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/r05y_bench_q4k64.json 2> gpurun_out/r05y_bench.err || { tail -5 gpurun_out/r05y_bench.err; exit 1; }
tail -c 600 gpurun_out/r05y_bench_q4k64.json
