#!/bin/bash
# round 6: configs[1] with a NULL stream vs an explicit stream (diag/null_stream_ab.py), F16 and Q4_K one clip
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in f16x1 q4kx1; do
  timeout -k 10 300 python3 diag/null_stream_ab.py $c >> gpurun_out/r06d_null_stream.jsonl 2> gpurun_out/r06d_err.log || { tail -5 gpurun_out/r06d_err.log; exit 1; }
done
cat gpurun_out/r06d_null_stream.jsonl
