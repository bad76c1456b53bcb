#!/bin/bash
# round 3: where the ggml backend's tiny-F16 rounding departs from the engine's (diag/backend_tiny_variants.py)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python3 -u diag/backend_tiny_variants.py > gpurun_out/t_variants.log 2>&1; echo rc=$?; tail -8 gpurun_out/t_variants.log
