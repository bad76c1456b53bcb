#!/bin/bash
# round 5: why four-head attention workgroups are slower — the HG = 4 binary with single-head workgroups only
# (Q2A_ATTN_DIAG_SMALL4 with the fusion off) against the HG = 1 kernel (off) and the mixed grid (default)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for i in 1 2; do
  for v in A B C; do
    unset Q2A_NO_ATTN_Q8K Q2A_ATTN_DIAG_SMALL4
    case $v in A) export Q2A_NO_ATTN_Q8K=1;; C) export Q2A_NO_ATTN_Q8K=1 Q2A_ATTN_DIAG_SMALL4=1;; esac
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05ze_q4k64_${v}$i.json 2> gpurun_out/r05ze_err.log || { tail -5 gpurun_out/r05ze_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05ze_q4k64_${v}$i.json'));print('q4k64 $v$i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('attention','quant_act','gemm_o')})"
  done
done
