#!/bin/bash
# round 3: attention occupancy A/B: cur (3 WG/CU, 168-VGPR budget, 2 spilled outside the loop) vs occ2 (2 WG/CU,
# 175 VGPRs, no spill), two alternating reps each
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'])" $1; }
for i in 1 2; do
for v in cur=$L occ2=diag/occ2/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/n_b_$n$i.json 2> gpurun_out/n_b_$n$i.err && s gpurun_out/n_b_$n$i.json || { tail -20 gpurun_out/n_b_$n$i.err; exit 1; }
done
done
