#!/bin/bash
# round 3: k_attn_t with the softmax split over both MFMA regions (exponentials of tile t+1 among the P.V MFMAs of
# tile t, the P split of tile t among the QK^T MFMAs of tile t+1) — parity subset on the product, then same-box A/B
# against the previous k_attn_t (diag/attn_t0) and its energy probes (wrong values on purpose: no K lo reads, no V^T lo
# reads, no exponentials), alternating, two reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/y_parity_log.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "attention or tiny or full_size" > gpurun_out/y_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/y_tests.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'])" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in new=$L t0=diag/attn_t0/libq2a.so nokl=diag/attn_NOKL/libq2a.so novl=diag/attn_NOVL/libq2a.so noexp=diag/attn_NOEXP/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/y_b_$n$i.json 2> gpurun_out/y_b_$n$i.err && s gpurun_out/y_b_$n$i.json || { tail -20 gpurun_out/y_b_$n$i.err; exit 1; }
done
done
