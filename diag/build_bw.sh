#!/bin/bash
# bwbench variants: diag/bw_<name> linked against a q2a_exact.o built with extra -D flags (timing only)
set -e
R=/root/repo/qwen2-audio-whisper-ggml_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/include -I$R/csrc -c /root/repo/diag/bwbench.hip -o /tmp/bwbench.o
for v in "base"; do
  set -- $v
  n=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include -I$R/csrc -munsafe-fp-atomics -w -ffp-contract=off "$@" -c $R/csrc/q2a_exact.hip -o /tmp/ex_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/bwbench.o /tmp/ex_$n.o -o /root/repo/diag/bw_$n
done
