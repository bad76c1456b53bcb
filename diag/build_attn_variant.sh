#!/bin/bash
# build a diagnostic attention variant of libq2a.so into diag/<name>/libq2a.so: diag/attn_variants.hip (the product
# q2a_attn.hip plus the schedules not adopted) under extra -D flags, e.g.
#   diag/build_attn_variant.sh attnv_g32 -DQ2A_ATTN_VARIANT=2        diag/build_attn_variant.sh attn_phl -DQ2A_ATTN_PHL=1
# linked with the product's other objects (make -C qwen2-audio-whisper-ggml_amd first). Never the shipped library.
set -e
NAME=$1; shift
D=$(cd "$(dirname "$0")" && pwd)
R=$D/../qwen2-audio-whisper-ggml_amd
O=$D/$NAME
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -munsafe-fp-atomics -fno-honor-nans -w $*"
/opt/rocm/bin/hipcc $F -c $D/attn_variants.hip -o $O/q2a_attn.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libq2a.so $R/build/q2a_gemm.o $O/q2a_attn.o $R/build/q2a_engine.o $R/build/q2a_exact.o $R/build/q2a_format.o $R/build/q2a_whisper.o $R/build/q2a_wav.o $R/build/q2a_group.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lpthread
echo built $O/libq2a.so
