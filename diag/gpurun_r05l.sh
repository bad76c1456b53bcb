#!/bin/bash
# round 5: fused Q|K|V vs separate projections (full F16) with the 4-wave narrow tiles (diag/nw2: NARROW_WM=2)
cd /root/repo
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
H=oracle/_ref/ggml_harness
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null
$T synth-clip $W/clip0.f32 480000 0 > /dev/null
for lib in base nw2; do
  [ $lib = nw2 ] && export LD_LIBRARY_PATH=$PWD/diag/nw2
  for v in fused sep; do
    case $v in fused) E="";; sep) E="GGML_Q2A_NO_FUSED_QKV=1";; esac
    env $E timeout -k 10 120 $H encode $W/full-f16.bin $W/clip0.f32 $W/o_${lib}_$v.f32 1 > /dev/null || exit 1
  done
  cmp -s $W/o_${lib}_fused.f32 $W/o_${lib}_sep.f32 && echo "$lib fused == sep" || echo "$lib fused != sep"
done
cmp -s $W/o_base_sep.f32 $W/o_nw2_sep.f32 && echo "sep: base == nw2" || echo "sep: base != nw2"
cmp -s $W/o_base_fused.f32 $W/o_nw2_fused.f32 && echo "fused: base == nw2" || echo "fused: base != nw2"
