#!/bin/bash
# round 4: PMC traffic + SQ counters for the other 64-clip configs (F16, configs[4] Q8_0 + bf16) and configs[1]
# (one F16 clip), so each config's bench line can cite its own fc1 traffic / MFMA busy (tag r04v)
cd /root/repo
for c in f16x64 q80bf16x64 f16x1; do
  timeout -k 10 1000 bash profiles/collect.sh r04v $c > gpurun_out/r04v_collect_$c.log 2>&1 || { echo "collect $c failed"; tail -5 gpurun_out/r04v_collect_$c.log; exit 1; }
  timeout -k 10 700 bash profiles/collect_sq.sh r04v $c > gpurun_out/r04v_collect_sq_$c.log 2>&1 || { echo "sq $c failed"; tail -5 gpurun_out/r04v_collect_sq_$c.log; exit 1; }
  echo "$c done"
done
