#!/bin/bash
# round 5: the persistent fc1's partial last round beside the GELU + Q8_K quantizer (Q2A_TAIL_MODE=1 with
# Q2A_TAIL_FC1 on / off) against the one-launch schedule (mode 0, default). Parity of mode 1 with fc1 split first
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_TAIL_MODE=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05zb_tests.log 2>&1; rc=$?
echo "mode 1 + fc1 gpu tests rc=$rc"; tail -2 gpurun_out/r05zb_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2; do
  for v in m0 m1 m1nofc1; do
    case $v in m0) export Q2A_TAIL_MODE=0 Q2A_TAIL_FC1=1;; m1) export Q2A_TAIL_MODE=1 Q2A_TAIL_FC1=1;; m1nofc1) export Q2A_TAIL_MODE=1 Q2A_TAIL_FC1=0;; esac
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-legs > gpurun_out/r05zb_q4k64_${v}_$i.json 2> gpurun_out/r05zb_err.log || { tail -5 gpurun_out/r05zb_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05zb_q4k64_${v}_$i.json'));print('q4k64 $v rep $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm','quant_act','gemm_o','gemm_fc1','gemm_fc2')})"
  done
done
