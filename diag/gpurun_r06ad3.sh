#!/bin/bash
# round 6 closing set, part C (tag r06ad): rocprofv3 kernel stats + PMC traffic for the 64-clip configs and the SQ
# counters of the default workload, on the same tree as parts A and B
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in q4k64 f16x64 q80bf16x64; do
  timeout -k 10 900 bash profiles/collect.sh r06ad $c > gpurun_out/r06ad_collect_$c.log 2>&1 || { tail -5 gpurun_out/r06ad_collect_$c.log; exit 1; }
  echo "collected $c"
done
timeout -k 10 600 bash profiles/collect_sq.sh r06ad q4k64 > gpurun_out/r06ad_collect_sq.log 2>&1 || { tail -5 gpurun_out/r06ad_collect_sq.log; exit 1; }
echo done
