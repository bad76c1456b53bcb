#!/bin/bash
# round 6: the ggml backend's encoder head (transpose + positional rows) and tail (pool between permutes) folded:
# the backend suite (fused vs per-node
# bit-identity included), then whisper_full encode times and a kernel trace
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ggml_backend.py tests/test_gpu_whisper_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06t_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06t_tests.log
case $rc in 0) ;; *) exit 1;; esac
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null && $T quantize $W/full-f16.bin $W/full-q4_k.bin q4_k 16 > /dev/null && $T synth-clip $W/clip0.f32 480000 0 > /dev/null || exit 1
for m in f16 q4_k; do
  for i in 1 2 3; do
    timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/new_$m.f32 8 > gpurun_out/r06t_${m}_$i.json || exit 1
    python3 -c "import json;n=json.load(open('gpurun_out/r06t_${m}_$i.json'));print('$m $i encode', n['best_encode_s'], 'fused', n['fused'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06t_prof -o gb --output-format csv -- oracle/_ref/ggml_harness encode $W/full-f16.bin $W/clip0.f32 $W/o.f32 8 > gpurun_out/r06t_prof.json 2> gpurun_out/r06t_prof.err || { tail -5 gpurun_out/r06t_prof.err; exit 1; }
echo done
