#!/bin/bash
# same-box A/B of the working tree against diag/prev (build_rev_lib.sh HEAD prev): GPU tests given in $TESTS first,
# then interleaved benches over $CFGS (default q4k64), $REPS rounds
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for t in ${TESTS:-tests/test_gpu_parity.py}; do
  n=$(basename $t .py)
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $t > gpurun_out/ab_$n.log 2>&1 || { tail -30 gpurun_out/ab_$n.log; exit 1; }
  echo "$t: $(tail -1 gpurun_out/ab_$n.log)"
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], ' '.join('%s=%.2f'%(k[:8],v['ms_per_step']) for k,v in pk.items() if v['ms_per_step']>5))" $1; }
for i in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-q4k64}; do
    Q2A_DIAG_BUILD=1 Q2A_LIB_PATH=diag/prev/libq2a.so timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_prev_$cfg.json && s gpurun_out/ab_prev_$cfg.json || exit 1
    timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_new_$cfg.json && s gpurun_out/ab_new_$cfg.json || exit 1
  done
done
