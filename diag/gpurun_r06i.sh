#!/bin/bash
# round 6: ggml backend with the fused Q|K|V route writing row-major V (k_attn_t<true>): the backend suite, then the
# reference's whisper_full timing on the backend (diag/ggml_backend_timing.sh) next to the engine's one-clip lines
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ggml_backend.py tests/test_gpu_whisper_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r06i_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 600 bash diag/ggml_backend_timing.sh > gpurun_out/r06i_backend.log 2>&1 || { tail -5 gpurun_out/r06i_backend.log; exit 1; }
cat gpurun_out/r06i_backend.log
