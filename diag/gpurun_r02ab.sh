#!/bin/bash
# narrow Q4_K tiles with five stages (block scales two blocks ahead) after the single-buffer 128-row change: parity,
# tests, then single-clip and batched benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for t in tests/test_gpu_parity.py tests/test_gpu_ggml_backend.py; do
  n=$(basename $t .py)
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $t > gpurun_out/aa_$n.log 2>&1 || { tail -30 gpurun_out/aa_$n.log; exit 1; }
  echo "$t: $(tail -1 gpurun_out/aa_$n.log)"
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], ' '.join('%s=%.3f'%(k[:8],v['ms_per_step']) for k,v in pk.items() if v['ms_per_step']>0.3))" $1; }
for c in q4kx1 q4kx1; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/aa_$c.json && s gpurun_out/aa_$c.json || exit 1
done
