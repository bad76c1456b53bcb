#!/bin/bash
# isolated-linear A/B: base, diagnostic variants, base again (same box)
set -e
export Q2A_BENCH_DIR=/tmp/q2ab
for v in base ${VARIANTS:-norescale nominterm noepi} base; do
  if [ $v = base ]; then timeout -k 10 300 python3 diag/linear_bench.py ${WT:-q4_k}; else Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 diag/linear_bench.py ${WT:-q4_k}; fi
done
