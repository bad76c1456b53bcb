#!/bin/bash
# round 3: which stage differs between the small-tile (1 clip) and 8-phase (30 clips) regimes, per library
cd /root/repo
mkdir -p gpurun_out /tmp/q2ac
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model /tmp/q2ac/tiny-f16.bin tiny f16 0x51A2 16 > /dev/null && $T gen-model /tmp/q2ac/full-f16.bin full f16 0x51A2 16 > /dev/null || exit 1
for v in cur=qwen2-audio-whisper-ggml_amd/lib/libq2a.so stg0=diag/stg0/libq2a.so fp16pv=diag/pv_fp16/libq2a.so r02=diag/pv_r02/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  for m in tiny full; do
    echo "== $n $m"
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 diag/regime_diff.py /tmp/q2ac/$m-f16.bin 0 || exit 1
  done
done
