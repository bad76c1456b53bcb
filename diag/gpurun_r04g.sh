#!/bin/bash
# round 4: layer-0 node trace of the ggml-backend drop-in path and of the engine (tiny F16) against the reference CPU
# builds (diag/backend_l0_trace.py); then PMC traffic + SQ counters of the persistent-fc1 product (profiles/collect*.sh)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python3 diag/backend_l0_trace.py gpu diag/_l0ref.npz > gpurun_out/r04g_backend_l0.jsonl 2> gpurun_out/r04g_backend_l0.err || { tail -5 gpurun_out/r04g_backend_l0.err; exit 1; }
cat gpurun_out/r04g_backend_l0.jsonl | cut -c1-330
bash profiles/collect.sh r04g q4k64 > gpurun_out/r04g_collect.log 2>&1 || { tail -20 gpurun_out/r04g_collect.log; exit 1; }
bash profiles/collect_sq.sh r04g q4k64 > gpurun_out/r04g_collect_sq.log 2>&1 || { tail -20 gpurun_out/r04g_collect_sq.log; exit 1; }
echo collected
