#!/bin/bash
# Q4_K block 0 without the rescale products (acc = 0: only the min term): bit-equality with the HEAD build (20 clips:
# 8-phase kernels; 1 clip: small tiles), parity tests, then same-box A/B
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for n in 20 1; do
  Q2A_LIB_PATH=diag/prev/libq2a.so timeout -k 10 300 python3 diag/encode_dump.py q4_k $n gpurun_out/af_prev_$n.npy || exit 1
  timeout -k 10 300 python3 diag/encode_dump.py q4_k $n gpurun_out/af_new_$n.npy || exit 1
  python3 -c "
import numpy as np
a=np.load('gpurun_out/af_prev_$n.npy'); b=np.load('gpurun_out/af_new_$n.npy')
print('clips=$n bit-identical:', np.array_equal(a,b), float(np.abs(a-b).max()))"
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/af_parity.log 2>&1 || { tail -30 gpurun_out/af_parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/af_parity.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], ' '.join('%s=%.2f'%(k[:8],v['ms_per_step']) for k,v in pk.items() if k.startswith('gemm')))" $1; }
for i in 1 2 3; do
  Q2A_LIB_PATH=diag/prev/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/af_prev.json && s gpurun_out/af_prev.json || exit 1
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/af_new.json && s gpurun_out/af_new.json || exit 1
done
