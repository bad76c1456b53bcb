#!/bin/bash
# round 6: the attention kernel with 16 queries per wave for grids that would leave CUs idle (one clip) and the lazy
# re-base decided per 16-query block: attention + batch-invariance tests, then alternating A/B against the previous
# attention object (diag/attnbase) at one clip (F16, Q4_K) and 64 clips Q4_K
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "attention or batch" > gpurun_out/r06k_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r06k_tests.log | tail -20
case $rc in 0) ;; *) exit 1;; esac
for c in f16x1 q4kx1 q4k64; do
  for i in 1 2; do
    for v in base new; do
      if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/attnbase/libq2a.so; else unset Q2A_LIB_PATH; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06k_${c}_${v}_$i.json 2> gpurun_out/r06k_err.log || { tail -5 gpurun_out/r06k_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06k_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('attention', 'gemm_qkv', 'gemm_fc1')})"
    done
  done
done
echo done
