#!/bin/bash
# the reference's own whisper_full (oracle/_ref/ggml_harness: unmodified src/qwen2-whisper.cpp + ggml, GPU branch
# pointed at libggml-q2a.so) on one full-size 30 s clip, next to the engine's single-clip encode of the same file
set -e
cd /root/repo
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
[ -f $W/full-f16.bin ] || $T gen-model $W/full-f16.bin full f16 0x51A2 16
[ -f $W/full-q4_k.bin ] || $T quantize $W/full-f16.bin $W/full-q4_k.bin q4_k 16
$T synth-clip $W/clip0.f32 480000 0
for m in f16 q4_k; do
  timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_$m.f32 8 > gpurun_out/gb_$m.json
  echo "$m graph $(cat gpurun_out/gb_$m.json)"
  GGML_Q2A_NO_GRAPH=1 timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_${m}_ng.f32 8 \
    > gpurun_out/gb_${m}_nograph.json
  echo "$m nograph $(cat gpurun_out/gb_${m}_nograph.json)"
  cmp $W/out_$m.f32 $W/out_${m}_ng.f32 && echo "$m graph == nograph (bitwise)"
done
if [ -n "$GB_PROF" ]; then   # kernel traces: GPU time per whisper_full vs the wall clock
  for m in f16 q4_k; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gb_prof_$m -o gb --output-format csv -- \
      oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_prof.f32 8 > gpurun_out/gb_prof_$m.json
  done
fi
