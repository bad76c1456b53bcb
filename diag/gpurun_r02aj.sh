#!/bin/bash
# k_attn_g<KPAD>: whole-tile K loads without the clamp on the engine's workspace (kpad): bit-equality with the HEAD
# build (20 clips), parity + attention variant tests, then same-box A/B
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_LIB_PATH=qwen2-audio-whisper-ggml_amd/lib/libq2a.so timeout -k 10 300 python3 diag/encode_dump.py q4_k 20 gpurun_out/aj_prev.npy || exit 1
Q2A_LIB_PATH=diag/kpad/libq2a.so timeout -k 10 300 python3 diag/encode_dump.py q4_k 20 gpurun_out/aj_new.npy || exit 1
python3 -c "
import numpy as np
a=np.load('gpurun_out/aj_prev.npy'); b=np.load('gpurun_out/aj_new.npy')
print('bit-identical:', np.array_equal(a,b), float(np.abs(a-b).max()))"
Q2A_LIB_PATH=diag/kpad/libq2a.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_attention_variants.py > gpurun_out/aj_tests.log 2>&1 || { tail -30 gpurun_out/aj_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/aj_tests.log)"
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1 2 3; do
  Q2A_LIB_PATH=qwen2-audio-whisper-ggml_amd/lib/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/aj_prev.json && s gpurun_out/aj_prev.json || exit 1
  Q2A_LIB_PATH=diag/kpad/libq2a.so timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/aj_new.json && s gpurun_out/aj_new.json || exit 1
done
