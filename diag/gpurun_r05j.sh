#!/bin/bash
# round 5: the ggml backend's fused Q|K|V route (one GEMM writing the attention operands): backend tests, then the
# reference's whisper_full timing (one full-size clip, F16 and Q4_K) with and without the route, and a kernel trace
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ggml_backend.py \
  > gpurun_out/r05j_tests.log 2>&1; rc=$?
echo "backend tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05j_tests.log | tail -25
[ $rc = 0 ] || exit 1
timeout -k 10 300 bash diag/ggml_backend_timing.sh > gpurun_out/r05j_gb.log 2>&1 || { tail -5 gpurun_out/r05j_gb.log; exit 1; }
grep -E "graph|bitwise" gpurun_out/r05j_gb.log | grep -v nograph
W=/tmp/q2a_gb
for m in f16 q4_k; do
  GGML_Q2A_NO_FUSED_QKV=1 timeout -k 10 300 oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_${m}_sep.f32 8 > gpurun_out/r05j_sep_$m.json || exit 1
  echo "$m sep $(cat gpurun_out/r05j_sep_$m.json)"
  cmp $W/out_$m.f32 $W/out_${m}_sep.f32 && echo "$m fused == separate (bitwise)"
done
for m in f16 q4_k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05j_prof_$m -o gb --output-format csv -- \
    oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_prof.f32 8 > /dev/null || exit 1
done
find gpurun_out/r05j_prof_* -name "*kernel_stats.csv" | head
