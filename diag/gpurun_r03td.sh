#!/bin/bash
# round 3: tail on the 64x128 deep-pipeline tiles at every K (diag/tail3: O, fc1 and fc2) vs the product (128x128 tail,
# fc2 only): linear/batch-invariance parity subset of the variant, then a same-box A/B, alternating, three reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_LIB_PATH=$PWD/diag/tail3/libq2a.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "invariant or linear" > gpurun_out/td_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/td_tests.log; [ $rc = 0 ] || exit 1
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('gemm_qkv', 'gemm_o', 'gemm_fc1', 'gemm_fc2', 'attention')})" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2 3; do
for v in new=$L t3=diag/tail3/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/td_b_$n$i.json 2> gpurun_out/td_b_$n$i.err && s gpurun_out/td_b_$n$i.json || { tail -20 gpurun_out/td_b_$n$i.err; exit 1; }
done
done
