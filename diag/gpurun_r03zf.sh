#!/bin/bash
# round 3 closing set: full GPU suite (parity log), smoke, profile set r03z (rocprofv3 kernel stats, PMC traffic,
# SQ counters) and the default bench line with the CPU baseline
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/zf_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/zf_tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/zf_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash profiles/collect.sh r03z q4k64 || exit 1
bash profiles/collect_sq.sh r03z q4k64 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/zf_bench.json 2> gpurun_out/zf_bench.err || { tail -20 gpurun_out/zf_bench.err; exit 1; }
tail -c 400 gpurun_out/zf_bench.json
