#!/bin/bash
# round 2p: full GPU test suite at HEAD (parity log), then the default bench (configs[2]) and configs[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export Q2A_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -3 gpurun_out/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python -u bench.py --config f16x1 --no-cpu-baseline > gpurun_out/bench_f16x1.json 2> gpurun_out/bench_f16x1.err
