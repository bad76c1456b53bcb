#!/bin/bash
# round 5: the residual GEMMs' partial last round beside the next LayerNorm, three schedules (Q2A_TAIL_MODE):
# 0 one launch per GEMM (round-4 schedule), 1 partial round on a top-priority side stream, 2 the LayerNorm's first rows
# on a CU-masked side stream. Parity of modes 1 and 2 (batch invariance, block, linear, dist), then alternating
# same-box bench triples (q4k64) and one f16x64 triple
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for m in 1 2; do
  Q2A_TAIL_MODE=$m timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05za_tests_m$m.log 2>&1; rc=$?
  echo "mode $m gpu tests rc=$rc"; tail -2 gpurun_out/r05za_tests_m$m.log
  case $rc in 0) ;; *) exit 1;; esac
done
for i in 1 2; do
  for m in 0 1 2; do
    Q2A_TAIL_MODE=$m timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05za_q4k64_m${m}_$i.json 2> gpurun_out/r05za_err.log || { tail -5 gpurun_out/r05za_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05za_q4k64_m${m}_$i.json'));print('q4k64 mode $m rep $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm','gemm_o','gemm_fc2')})"
  done
done
for m in 0 1 2; do
  Q2A_TAIL_MODE=$m timeout -k 10 300 python3 bench.py --config f16x64 --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05za_f16x64_m$m.json 2> gpurun_out/r05za_err.log || { tail -5 gpurun_out/r05za_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05za_f16x64_m$m.json'));print('f16x64 mode $m', d['ms_per_step'])"
done
