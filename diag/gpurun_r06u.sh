#!/bin/bash
# round 6: the one-clip residual GEMMs normalise the rows they complete (LN2 after O, the next layer's LN1 after fc2:
# sc1 stores, a per-64-row-block counter, the LayerNorm kernel's arithmetic on sc1 loads): the whole GPU suite, then
# alternating one-clip benches against the previous library (diag/lnbase)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06u_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06u_tests.log
case $rc in 0) ;; *) exit 1;; esac
for c in f16x1 q4kx1; do
  for i in 1 2 3; do
    for v in base new; do
      if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/lnbase/libq2a.so; else unset Q2A_LIB_PATH; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r06u_${c}_${v}_$i.json 2> gpurun_out/r06u_err.log || { tail -5 gpurun_out/r06u_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06u_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm', 'gemm_o', 'gemm_fc2')})"
    done
  done
done
echo done
