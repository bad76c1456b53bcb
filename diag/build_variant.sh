#!/bin/bash
# build a diagnostic variant of libq2a.so into diag/<name>/libq2a.so with extra -D flags (A/B timing only; the
# experiment knobs of rounds 1-5 need diag/experiment_knobs_r05.patch applied first, the Q2A_DIAG_NO_STORE / STAMPS
# timing builds work on the product source)
set -e
NAME=$1; shift
R=/root/repo/qwen2-audio-whisper-ggml_amd
O=/root/repo/diag/$NAME
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/../include -I$R/csrc -munsafe-fp-atomics -w $*"
/opt/rocm/bin/hipcc $F -c $R/csrc/q2a_gemm.hip -o $O/q2a_gemm.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libq2a.so $O/q2a_gemm.o $R/build/q2a_attn.o $R/build/q2a_engine.o $R/build/q2a_exact.o $R/build/q2a_format.o $R/build/q2a_whisper.o $R/build/q2a_wav.o $R/build/q2a_group.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lpthread
echo built $O/libq2a.so
