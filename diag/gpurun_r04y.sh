#!/bin/bash
# round 4 final tree (+ mel atomics): persistent fc1 + staggered 8-phase GEMMs + exact conv: whole GPU suite + smoke, the default bench line (with the
# CPU baseline), rocprofv3 kernel stats + PMC traffic, SQ counters (profiles/collect*.sh, tag r04y)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/r04y_parity_log.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04y_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 gpurun_out/r04y_tests.log
case $rc in 124|137|134|139) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r04y_smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/r04y_bench_q4k64.json 2> gpurun_out/r04y_bench.err || { tail -5 gpurun_out/r04y_bench.err; exit 1; }
tail -c 1500 gpurun_out/r04y_bench_q4k64.json
timeout -k 10 900 bash profiles/collect.sh r04y q4k64 > gpurun_out/r04y_collect.log 2>&1 || { tail -5 gpurun_out/r04y_collect.log; exit 1; }
timeout -k 10 600 bash profiles/collect_sq.sh r04y q4k64 > gpurun_out/r04y_collect_sq.log 2>&1 || { tail -5 gpurun_out/r04y_collect_sq.log; exit 1; }
echo done
bash diag/gpurun_r04y_configs.sh
