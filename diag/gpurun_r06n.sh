#!/bin/bash
# round 6: the backend's conv MUL_MAT over the hi part alone when every activation is an fp16 value (conv2), else the
# three-part GEMM (device-side choice between two launches): the ggml-backend tests, then whisper_full with the
# previous libraries (diag/convbase) and the new ones — encode times and embd_enc compared bit for bit
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ggml_backend.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06n_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r06n_tests.log | tail -30
case $rc in 0) ;; *) exit 1;; esac
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null && $T quantize $W/full-f16.bin $W/full-q4_k.bin q4_k 16 > /dev/null && $T synth-clip $W/clip0.f32 480000 0 > /dev/null || exit 1
for m in f16 q4_k; do
  for i in 1 2; do
    LD_LIBRARY_PATH=$PWD/diag/convbase timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/base_$m.f32 8 > gpurun_out/r06n_base_${m}_$i.json || exit 1
    timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/new_$m.f32 8 > gpurun_out/r06n_new_${m}_$i.json || exit 1
    python3 -c "import json;b=json.load(open('gpurun_out/r06n_base_${m}_$i.json'));n=json.load(open('gpurun_out/r06n_new_${m}_$i.json'));print('$m $i encode base', b['best_encode_s'], 'new', n['best_encode_s'])"
  done
  cmp $W/base_$m.f32 $W/new_$m.f32 && echo "$m: embd_enc identical (bitwise)"
done
echo done
