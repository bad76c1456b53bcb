#!/bin/bash
# build a diagnostic variant of libq2a.so into diag/<name>/libq2a.so with ONE source file recompiled with extra -D flags
# (A/B timing only): bash diag/build_variant_src.sh <q2a_gemm|q2a_attn|q2a_exact|q2a_engine> <name> [flags...]
set -e
SRC=$1; NAME=$2; shift 2
R=/root/repo/qwen2-audio-whisper-ggml_amd
O=/root/repo/diag/$NAME
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -munsafe-fp-atomics -w"
case $SRC in
  q2a_exact) F="$F -ffp-contract=off";;
  q2a_attn) F="$F -fno-honor-nans";;
esac
/opt/rocm/bin/hipcc $F $* -c $R/csrc/$SRC.hip -o $O/$SRC.o
OBJS=""
for o in q2a_gemm q2a_attn q2a_engine q2a_exact q2a_format q2a_whisper q2a_wav q2a_group; do
  if [ $o = $SRC ]; then OBJS="$OBJS $O/$o.o"; else OBJS="$OBJS $R/build/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libq2a.so $OBJS -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lpthread
rm -f $O/$SRC.o
echo built $O/libq2a.so
