#!/bin/bash
# round 5: where the fused Q|K|V route departs from the separate projections (F16): harness variants, bitwise cmp
cd /root/repo
mkdir -p gpurun_out
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
H=oracle/_ref/ggml_harness
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null
$T gen-model $W/tiny-f16.bin tiny f16 0x51A2 16 > /dev/null
$T synth-clip $W/clip0.f32 480000 0 > /dev/null
for m in tiny full; do
  for v in fused sep nofuse; do
    case $v in fused) E="";; sep) E="GGML_Q2A_NO_FUSED_QKV=1";; nofuse) E="GGML_Q2A_NO_FUSE=1";; esac
    env $E timeout -k 10 120 $H encode $W/$m-f16.bin $W/clip0.f32 $W/o_${m}_$v.f32 1 > gpurun_out/r05k_${m}_$v.json || exit 1
  done
  cmp -s $W/o_${m}_fused.f32 $W/o_${m}_sep.f32 && echo "$m fused == sep" || echo "$m fused != sep"
  cmp -s $W/o_${m}_sep.f32 $W/o_${m}_nofuse.f32 && echo "$m sep == nofuse" || echo "$m sep != nofuse"
  cmp -s $W/o_${m}_fused.f32 $W/o_${m}_nofuse.f32 && echo "$m fused == nofuse" || echo "$m fused != nofuse"
done
