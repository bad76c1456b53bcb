#!/bin/bash
# round 6: grouped rasterisation of the one-clip 64-row tiles (O / fc2): six stages for the F16 64-row tiles (diag/ns6), GROUP_M 12 for the 128-row tiles (diag/g128), both
# (diag/both), alternating one-clip benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in f16x1 q4kx1; do
  for i in 1 2; do
    for v in base ns6 g128 both; do
      if [ $v = base ]; then unset Q2A_LIB_PATH; else export Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r06q_${c}_${v}_$i.json 2> gpurun_out/r06q_err.log || { tail -5 gpurun_out/r06q_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06q_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('gemm_fc2', 'gemm_o', 'gemm_qkv', 'gemm_fc1')})"
    done
  done
done
echo done
