#!/bin/bash
# round 4: what an fp8 (block-scaled 16x16x128) form of the QK^T correction terms would cost — timing-only build
# diag/f8time (-DQ2A_ATTN_DIAG_F8TIME, wrong values) against the product, alternating on one box
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('attention', 'gemm_qkv', 'gemm_fc1')})" $1; }
for i in 1 2; do
for v in base=$L f8time=diag/f8time/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04k_b_$n$i.json 2> gpurun_out/r04k_b_$n$i.err && s gpurun_out/r04k_b_$n$i.json || { tail -20 gpurun_out/r04k_b_$n$i.err; exit 1; }
done
done
