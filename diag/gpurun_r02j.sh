#!/bin/bash
# round-2 profile refresh: kernel-trace stats + PMC traffic for q4k64, bench lines for q4k64 / f16x1 / q80bf16x64
set -e
R=$(pwd)
bash profiles/collect.sh r02b q4k64
cd $R
timeout -k 10 300 python3 bench.py --config f16x1 --no-cpu-baseline > gpurun_out/r02b_f16x1.json
timeout -k 10 300 python3 bench.py --config q80bf16x64 --no-cpu-baseline > gpurun_out/r02b_q80bf16x64.json
