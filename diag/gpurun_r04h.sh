#!/bin/bash
# round 4: does the conv's own summation error explain the ggml-backend F16 excess? tiny F16 clip-averaged distances
# of the backend variants (diag/backend_tiny_variants.py, incl. the f64-summed conv), then the backend's F16 parity
# tests with the f64 conv, every comparison logged (Q2A_PARITY_LOG)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python3 diag/backend_tiny_variants.py > gpurun_out/r04h_variants.jsonl 2> gpurun_out/r04h_variants.err || { tail -5 gpurun_out/r04h_variants.err; exit 1; }
cat gpurun_out/r04h_variants.jsonl
GGML_Q2A_CONV_F64=1 Q2A_PARITY_LOG=$PWD/gpurun_out/r04h_convf64_parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ggml_backend.py -m gpu -q -k "f16" --timeout 300 --timeout-method thread > gpurun_out/r04h_convf64_tests.log 2>&1; echo "conv_f64 backend tests rc=$?"
tail -5 gpurun_out/r04h_convf64_tests.log
cat gpurun_out/r04h_convf64_parity.jsonl
