#!/bin/bash
# round 6: the reference's unmodified whisper_full on the ggml backend after the LayerNorm load fix, the GELU-lookup
# fix and the conv transpose's batched loads (diag/bkbase = libggml-q2a.so + libq2a.so of 63563f3, before them):
# backend suite, then alternating encodes with output bits compared
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ggml_backend.py tests/test_gpu_whisper_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06ab_tests.log
case $rc in 0) ;; *) exit 1;; esac
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null && $T quantize $W/full-f16.bin $W/full-q4_k.bin q4_k 16 > /dev/null && $T synth-clip $W/clip0.f32 480000 0 > /dev/null || exit 1
for m in f16 q4_k; do
  for i in 1 2 3; do
    for v in base new; do
      if [ $v = base ]; then export LD_LIBRARY_PATH=$PWD/diag/bkbase; else unset LD_LIBRARY_PATH; fi
      timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/${v}_$m.f32 8 > gpurun_out/r06ab_${m}_${v}_$i.json || exit 1
      python3 -c "import json;n=json.load(open('gpurun_out/r06ab_${m}_${v}_$i.json'));print('$m $v $i encode', n['best_encode_s'], 'fused', n['fused'])"
    done
    cmp $W/base_$m.f32 $W/new_$m.f32 && echo "$m outputs identical"
  done
done
unset LD_LIBRARY_PATH
echo done
