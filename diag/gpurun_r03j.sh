#!/bin/bash
# round 3: exact three-part mel operand for conv1 (engine and ggml backend): front-end divergence vs the reference
# builds, then the whole GPU suite with the parity log
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python3 diag/frontend_diag.py diag/_fe.npz > gpurun_out/j_fe.jsonl 2> gpurun_out/j_fe.err || { tail -5 gpurun_out/j_fe.err; exit 1; }
cat gpurun_out/j_fe.jsonl
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$PWD/gpurun_out/j_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/j_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/j_tests.log)"
grep -E "^FAILED|^ERROR" gpurun_out/j_tests.log | head -20
grep -E "^E   +AssertionError: \(" gpurun_out/j_tests.log | head -20
