#!/bin/bash
# round 3: front-end divergence diagnostic (GPU mel vs oracle, layer-0 input vs every reference build)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python3 diag/frontend_diag.py diag/_fe.npz > gpurun_out/i_fe.jsonl 2> gpurun_out/i_fe.err || { tail -5 gpurun_out/i_fe.err; exit 1; }
cat gpurun_out/i_fe.jsonl
