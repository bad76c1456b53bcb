#!/bin/bash
# round 6: persistent Q4_K residual GEMMs (O-projection, fc2's whole rounds): GPU suite, then A/B against the previous
# tree (diag/pbase), alternating, q4k64
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r06g_tests.log
case $rc in 0) ;; *) exit 1;; esac
for c in q4k64; do
  for i in 1 2 3; do
    for v in base new; do
      if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/pbase/libq2a.so; else unset Q2A_LIB_PATH; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06g_${c}_${v}_$i.json 2> gpurun_out/r06g_err.log || { tail -5 gpurun_out/r06g_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06g_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k.startswith('gemm') or k.startswith('att')})"
    done
  done
done
