#!/bin/bash
# round 2n: ggml backend upload-time repack (tests + whisper_full timing), k_attn_g V^T b128 reads + saddr DMA:
# attention parity, then same-box A/B against diag/prev (HEAD build)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
: timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ggml_backend.py \
  > gpurun_out/n_gb_tests.log 2>&1 || { tail -30 gpurun_out/n_gb_tests.log; exit 1; }
tail -2 gpurun_out/n_gb_tests.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  > gpurun_out/n_parity.log 2>&1 || { tail -30 gpurun_out/n_parity.log; exit 1; }
tail -2 gpurun_out/n_parity.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16_act.py \
  > gpurun_out/n_bf16.log 2>&1 || { tail -30 gpurun_out/n_bf16.log; exit 1; }
tail -2 gpurun_out/n_bf16.log
for cfg in q4k64 q80bf16x64 q4k64 q80bf16x64; do
  Q2A_DIAG_BUILD=1 Q2A_LIB_PATH=diag/prev/libq2a.so timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/n_prev_$cfg.json && s gpurun_out/n_prev_$cfg.json || exit 1
  timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/n_new_$cfg.json && s gpurun_out/n_new_$cfg.json || exit 1
done
: bash diag/ggml_backend_timing.sh
