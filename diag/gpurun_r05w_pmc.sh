#!/bin/bash
# round 5 closing set, the other configs' counter passes (the q4k64 set is in diag/gpurun_r05w.sh): rocprofv3 kernel
# stats + PMC traffic (profiles/collect.sh) and SQ counters (profiles/collect_sq.sh) for f16x1, f16x64, q80bf16x64
cd /root/repo
mkdir -p gpurun_out
for cfg in f16x1 f16x64 q80bf16x64; do
  timeout -k 10 600 bash profiles/collect.sh r05w $cfg > gpurun_out/r05w_collect_$cfg.log 2>&1 || { tail -5 gpurun_out/r05w_collect_$cfg.log; exit 1; }
  timeout -k 10 600 bash profiles/collect_sq.sh r05w $cfg > gpurun_out/r05w_collect_sq_$cfg.log 2>&1 || { tail -5 gpurun_out/r05w_collect_sq_$cfg.log; exit 1; }
  echo "$cfg done"
done
