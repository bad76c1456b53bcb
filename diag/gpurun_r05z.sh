#!/bin/bash
# round 5: residual GEMMs' partial last round on a side stream beside the next LayerNorm (run_block tail overlap).
# Parity first (batch invariance, block, linear, full-size encodes), then alternating same-box bench pairs:
# A = Q2A_NO_TAIL_OVERLAP=1 (one launch per GEMM), B = default; q4k64 and f16x64
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05z_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r05z_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export Q2A_NO_TAIL_OVERLAP=1; else unset Q2A_NO_TAIL_OVERLAP; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05z_q4k64_${v}$i.json 2> gpurun_out/r05z_err.log || { tail -5 gpurun_out/r05z_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05z_q4k64_${v}$i.json'));print('q4k64 $v$i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm','gemm_o','gemm_fc2')})"
  done
done
for v in A B; do
  if [ $v = A ]; then export Q2A_NO_TAIL_OVERLAP=1; else unset Q2A_NO_TAIL_OVERLAP; fi
  timeout -k 10 300 python3 bench.py --config f16x64 --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05z_f16x64_$v.json 2> gpurun_out/r05z_err.log || { tail -5 gpurun_out/r05z_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05z_f16x64_$v.json'));print('f16x64 $v', d['ms_per_step'])"
done
