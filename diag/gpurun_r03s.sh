#!/bin/bash
# round 3: full GPU suite (k_attn_t) with parity log, smoke, default bench line (fresh container rebuild)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/s_parity_log.jsonl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1 || { tail -30 gpurun_out/s_tests.log; exit 1; }
tail -3 gpurun_out/s_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || { tail -20 gpurun_out/s_bench.err; exit 1; }
tail -c 1200 gpurun_out/s_bench.json
