#!/bin/bash
# round 5: (1) the new GPU tests (device group through RCCL, FAILED statuses, NULL-stream ordering); (2) main-loop
# attribution of the 8-phase GEMM by timing-only ablation builds (wrong results, isolated linears on fixed inputs):
# abl_noglds (no operand glds in the loop), abl_noreads (no fragment ds_reads), abl_nobar (no loop barriers),
# abl_mfmabar (MFMAs + barriers only), abl_mfma (MFMAs only). Builds: bash diag/build_variant.sh abl_<v> -DQ2A_DIAG_...
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
# (the new GPU tests ran green in this script's first call: 16 passed, gpurun_out/r05b_tests.log)
for r in 1 2; do
  for v in base=$L noglds=diag/abl_noglds/libq2a.so noreads=diag/abl_noreads/libq2a.so nobar=diag/abl_nobar/libq2a.so mfmabar=diag/abl_mfmabar/libq2a.so mfma=diag/abl_mfma/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    for wt in f16 q4_k; do
      Q2A_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 diag/linear_bench.py $wt > gpurun_out/r05b_lin_${n}_${wt}_$r.json || exit 1
      echo "$n $wt $(cat gpurun_out/r05b_lin_${n}_${wt}_$r.json)"
    done
  done
done
