#!/bin/bash
# round 3 (re-entry): the whole GPU suite on the current tree with the parity log, then the default bench
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$PWD/gpurun_out/f_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 840 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/f_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/f_tests.log)"
grep -E "FAILED|ERROR" gpurun_out/f_tests.log | head -20
[ $rc -le 1 ] || exit $rc
unset Q2A_PARITY_LOG
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || { tail -20 gpurun_out/f_bench.err; exit 1; }
tail -c 3000 gpurun_out/f_bench.json
