#!/bin/bash
# round 5: (1) LDS read-burst attribution in the 8-phase loop — timing-only builds (wrong results, fixed inputs) that
# skip phase 1's 8 A-fragment reads (its 12-read burst becomes 4: diag/skipra1) or phase 3's 8 (diag/skipra3);
# (2) the reference's whisper_full on the ggml backend after the 8-wave narrow tiles (drop-in route timing).
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for r in 1 2; do
  for v in base=$L skipra1=diag/skipra1/libq2a.so skipra3=diag/skipra3/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 diag/linear_bench.py f16 > gpurun_out/r05g_lin_${n}_$r.json || exit 1
    echo "$n $(cat gpurun_out/r05g_lin_${n}_$r.json)"
  done
done
timeout -k 10 900 bash diag/ggml_backend_timing.sh > gpurun_out/r05g_gb.log 2>&1; rc=$?
echo "backend timing rc=$rc"; grep -E "graph|nograph" gpurun_out/r05g_gb.log | cut -c1-400
