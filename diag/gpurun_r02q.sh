#!/bin/bash
# k_attn_g: v_permlane32_swap max exchange and s_setprio around the MFMA clusters — attention parity under each
# variant, then interleaved same-box benches (per-kernel attention ms)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
VS="av_base av_p32 av_p32pr1 av_p32pr2"
for v in $VS; do
  Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "attention or (full_size_vs and f16)" > gpurun_out/q_parity_$v.log 2>&1 || { tail -30 gpurun_out/q_parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/q_parity_$v.log)"
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2; do
  for v in $VS; do
    Q2A_LIB_PATH=diag/$v/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/q_$v.json && s gpurun_out/q_$v.json || exit 1
  done
done
