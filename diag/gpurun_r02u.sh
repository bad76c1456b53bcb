#!/bin/bash
# attention cost decomposition (diagnostic builds, wrong values on purpose): k_attn_g as built, without the softmax
# VALU, without the P.V MFMAs, without both — per-kernel attention ms, interleaved
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/u_base.json && s gpurun_out/u_base.json || exit 1
  for v in av_nosm av_noexp; do
    Q2A_DIAG_BUILD=1 Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/u_$v.json && s gpurun_out/u_$v.json || exit 1
  done
done
