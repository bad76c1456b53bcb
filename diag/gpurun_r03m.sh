#!/bin/bash
# round 3: QK^T term variants end to end (pv_parity) and their attention time: cur = 3 terms, qk21 = K as fp16,
# qk22 = Q as fp16
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 600 python3 -u diag/pv_parity.py gpurun_out/m_pv.jsonl cur=$L qk21=diag/qk21/libq2a.so qk22=diag/qk22/libq2a.so \
    > gpurun_out/m_pv.log 2>&1 || { tail -30 gpurun_out/m_pv.log; exit 1; }
cat gpurun_out/m_pv.jsonl
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'], 'qkv', pk['gemm_qkv']['ms_per_step'])" $1; }
for v in cur=$L qk21=diag/qk21/libq2a.so qk22=diag/qk22/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/m_b_$n.json 2> gpurun_out/m_b_$n.err && s gpurun_out/m_b_$n.json || { tail -20 gpurun_out/m_b_$n.err; exit 1; }
done
