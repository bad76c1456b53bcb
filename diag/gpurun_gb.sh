#!/bin/bash
# ggml-backend: upload-time repack check (tests) + whisper_full timing (first call vs best)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ggml_backend.py \
  > gpurun_out/gb_tests.log 2>&1 || { tail -30 gpurun_out/gb_tests.log; exit 1; }
tail -3 gpurun_out/gb_tests.log
bash diag/ggml_backend_timing.sh
