#!/bin/bash
# round 6 closing set, part D (tag r06ad): SQ counters of the other configs (the bench line's step-level mfma_util)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in f16x1 q4kx1 f16x64 q80bf16x64; do
  timeout -k 10 600 bash profiles/collect_sq.sh r06ad $c > gpurun_out/r06ad_collect_sq_$c.log 2>&1 || { tail -5 gpurun_out/r06ad_collect_sq_$c.log; exit 1; }
  echo "sq $c"
done
echo done
