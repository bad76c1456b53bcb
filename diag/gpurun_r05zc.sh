#!/bin/bash
# round 5: attention workgroups of four heads writing the O-projection's Q8_K operand (k_attn_t<4>) instead of the
# separate quantizer pass. Parity first (64-clip batch invariance: clip alone = separate quantizer, in the batch =
# fused; block, dist, golden encodes), then alternating same-box bench pairs: A = Q2A_NO_ATTN_Q8K=1, B = fused
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_group.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05zc_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r05zc_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export Q2A_NO_ATTN_Q8K=1; else unset Q2A_NO_ATTN_Q8K; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05zc_q4k64_${v}$i.json 2> gpurun_out/r05zc_err.log || { tail -5 gpurun_out/r05zc_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05zc_q4k64_${v}$i.json'));print('q4k64 $v$i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('attention','quant_act','gemm_o')})"
  done
done
