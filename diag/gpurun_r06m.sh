#!/bin/bash
# round 6: fc2's partial-round tail on other tile shapes (diag/tail1: 128x256, diag/tail2: 64x128 on 8 waves; product:
# 128x128; diag/tail3: 128x256 and the tail for K >= 1024 too, i.e. O and F16 fc1) — 64-clip batch invariance with each, then alternating q4k64 / f16x64 benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for v in tail1 tail2 tail3; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "batch_64_is_batch_invariant" > gpurun_out/r06m_tests_$v.log 2>&1 || { echo "$v tests failed"; tail -15 gpurun_out/r06m_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06m_tests_$v.log)"
done
for c in q4k64 f16x64; do
  for i in 1 2; do
    for v in base tail1 tail2 tail3; do
      if [ $v = base ]; then unset Q2A_LIB_PATH; else export Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06m_${c}_${v}_$i.json 2> gpurun_out/r06m_err.log || { tail -5 gpurun_out/r06m_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06m_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('gemm_fc2', 'gemm_o')})"
    done
  done
done
echo done
