#!/bin/bash
# desync experiment: first-round phase offsets for CU groups (Q2A_GEMM_STAGGER_NS / _G)
cd /root/repo
export Q2A_BENCH_DIR=/tmp/q2ab
CFG=${CFG:-f16x64}
for v in ${STAGGER_LIST:-"0 2" "20000 2" "40000 2" "40000 4" "60000 4"}; do
  set -- ${v/_/ }
  Q2A_GEMM_STAGGER_NS=$1 Q2A_GEMM_STAGGER_G=$2 timeout -k 10 300 python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/st_${CFG}_$1_$2.json 2>>gpurun_out/st_err.txt || exit 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/st_${CFG}_$1_$2.json').read().strip().splitlines()[-1])
print('$1 $2', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['per_kernel'].items() if 'gemm' in k})"
done
