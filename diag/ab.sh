#!/bin/bash
# A/B timing of diagnostic library variants: bench per-kernel ms for each variant and config
cd /root/repo
export Q2A_BENCH_DIR=/tmp/q2ab
for cfg in "$@"; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_base_$cfg.json 2>>gpurun_out/ab_err.txt || exit 1
  for v in ${VARIANTS:-noglds noepi both}; do
    Q2A_DIAG_BUILD=1 Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${v}_$cfg.json 2>>gpurun_out/ab_err.txt || exit 1
  done
done
