#!/bin/bash
# round 4: tile / stage A/B of the exact-accumulation conv GEMMs (Q2A_GEMM_EXACT_TILE / _NS; bit-identical outputs)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 3) for k in ('conv1', 'conv2')})" $1; }
for v in base=$L exns4=diag/exns4/libq2a.so ext128=diag/ext128/libq2a.so ext128n3=diag/ext128n3/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04m_b_$n.json 2> gpurun_out/r04m_b_$n.err && s gpurun_out/r04m_b_$n.json || { tail -20 gpurun_out/r04m_b_$n.err; exit 1; }
done
