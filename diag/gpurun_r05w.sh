#!/bin/bash
# round 5 closing set (second session): whole GPU suite + smoke, the default bench line (with the CPU baseline at both ISA levels),
# rocprofv3 kernel stats + PMC traffic, SQ counters (profiles/collect*.sh, tag r05w)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/r05w_parity_log.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 gpurun_out/r05w_tests.log
case $rc in 124|137|134|139) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05w_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r05w_smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/r05w_bench_q4k64.json 2> gpurun_out/r05w_bench.err || { tail -5 gpurun_out/r05w_bench.err; exit 1; }
tail -c 1500 gpurun_out/r05w_bench_q4k64.json
timeout -k 10 900 bash profiles/collect.sh r05w q4k64 > gpurun_out/r05w_collect.log 2>&1 || { tail -5 gpurun_out/r05w_collect.log; exit 1; }
timeout -k 10 600 bash profiles/collect_sq.sh r05w q4k64 > gpurun_out/r05w_collect_sq.log 2>&1 || { tail -5 gpurun_out/r05w_collect_sq.log; exit 1; }
echo done

