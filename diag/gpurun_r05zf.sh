#!/bin/bash
# round 5: GELU + Q8_K quantizer with its input two iterations ahead (k_gelu_quant_q8k_h16<2>: two LDS stages per wave,
# the workgroup's whole 160 KiB) against one iteration ahead (<1>, Q2A_GELU_ONE_STAGE=1). Parity first (the three fc1
# paths' codes identical, batch invariance incl. the ragged single clip), then alternating same-box bench pairs
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05zf_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r05zf_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export Q2A_GELU_ONE_STAGE=1; else unset Q2A_GELU_ONE_STAGE; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05zf_q4k64_${v}$i.json 2> gpurun_out/r05zf_err.log || { tail -5 gpurun_out/r05zf_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05zf_q4k64_${v}$i.json'));print('q4k64 $v$i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('quant_act','gemm_fc1','gemm_fc2')})"
  done
done
