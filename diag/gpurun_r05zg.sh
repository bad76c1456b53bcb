#!/bin/bash
# round 5: a single clip's fp16 QKV / fc1 on 128x256 tiles with three LDS stages (one workgroup per CU, one round)
# instead of two-stage 128x128 tiles (Q2A_NO_SMALL_WIDE=1). Parity first (batch invariance F16: the clip alone takes
# the new tiles, inside the 64-clip batch the 8-phase kernel), then alternating same-box f16x1 bench pairs
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_isolated.py tests/test_gpu_whisper_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05zg_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r05zg_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export Q2A_NO_SMALL_WIDE=1; else unset Q2A_NO_SMALL_WIDE; fi
    timeout -k 10 300 python3 bench.py --config f16x1 --steps 20 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05zg_f16x1_${v}$i.json 2> gpurun_out/r05zg_err.log || { tail -5 gpurun_out/r05zg_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05zg_f16x1_${v}$i.json'));print('f16x1 $v$i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('gemm_qkv','gemm_fc1','gemm_o','gemm_fc2','attention')})"
  done
done
