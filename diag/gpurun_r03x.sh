#!/bin/bash
# round 3: where k_attn_t's energy goes — diagnostic builds (wrong values on purpose) without the K lo / V^T lo
# fragment reads or without the exponentials, against the product, same box, alternating, two reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'])" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in t=$L nokl=diag/attn_NOKL/libq2a.so novl=diag/attn_NOVL/libq2a.so noexp=diag/attn_NOEXP/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/x_b_$n$i.json 2> gpurun_out/x_b_$n$i.err && s gpurun_out/x_b_$n$i.json || { tail -20 gpurun_out/x_b_$n$i.err; exit 1; }
done
done
