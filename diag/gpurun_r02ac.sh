#!/bin/bash
# ggml backend: K|Q grouped launch for Q4_K weights too — backend tests (golden, fusion/graph bit-equality), engine
# parity, then whisper_full timing
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for t in tests/test_gpu_ggml_backend.py tests/test_gpu_parity.py; do
  n=$(basename $t .py)
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $t > gpurun_out/ac_$n.log 2>&1 || { tail -30 gpurun_out/ac_$n.log; exit 1; }
  echo "$t: $(tail -1 gpurun_out/ac_$n.log)"
done
timeout -k 10 600 bash diag/ggml_backend_timing.sh > gpurun_out/ac_gb.log 2>&1 || { tail -20 gpurun_out/ac_gb.log; exit 1; }
grep "graph {" gpurun_out/ac_gb.log | cut -c1-400
