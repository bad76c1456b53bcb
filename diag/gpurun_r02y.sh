#!/bin/bash
# single-clip GEMM regime: the deep-pipeline 64x128 tiles for every small-M GEMM (Q2A_GEMM_NARROW_ALL=1) vs the
# default (64x128 only when 128x128 tiles leave CUs idle): parity of the single-clip paths, then interleaved benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_GEMM_NARROW_ALL=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    > gpurun_out/y_parity.log 2>&1 || { tail -30 gpurun_out/y_parity.log; exit 1; }
echo "narrow_all parity: $(tail -1 gpurun_out/y_parity.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], ' '.join('%s=%.3f'%(k[:8],v['ms_per_step']) for k,v in pk.items() if v['ms_per_step']>0.3))" $1; }
for i in 1 2; do
  for c in q4kx1 f16x1; do
    for n in 0 1; do
      Q2A_GEMM_NARROW_ALL=$n timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/y_${c}_$n.json && s gpurun_out/y_${c}_$n.json || exit 1
    done
  done
done
