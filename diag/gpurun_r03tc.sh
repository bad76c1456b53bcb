#!/bin/bash
# round 3 closing set after the fc2 tail split: full GPU suite (incl. the RCCL world-size-1 bring-up), smoke,
# profile set r03zt (rocprofv3 kernel stats, PMC traffic, SQ counters) and the default bench line with the CPU baseline
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/tc_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/tc_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tc_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash profiles/collect.sh r03zt q4k64 || exit 1
bash profiles/collect_sq.sh r03zt q4k64 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/tc_bench.json 2> gpurun_out/tc_bench.err || { tail -20 gpurun_out/tc_bench.err; exit 1; }
tail -c 600 gpurun_out/tc_bench.json
