#!/bin/bash
# round-2 closing profile set r02x at HEAD: bench lines for every config, rocprofv3 kernel stats + PMC traffic
# (collect.sh) and SQ MFMA-busy passes (collect_sq.sh) for configs[2] (q4k64)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 400 python3 -u bench.py > gpurun_out/x_bench_q4k64.json 2> gpurun_out/x_bench.err || exit 1
for c in f16x1 q4kx1 f16x64 q80bf16x64; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/x_bench_$c.json 2> gpurun_out/x_bench_$c.err || exit 1
done
bash profiles/collect.sh r02x q4k64 || exit 1
cd $GRAFT_REPO_ROOT
bash profiles/collect_sq.sh r02x q4k64 || exit 1
