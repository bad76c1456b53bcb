#!/bin/bash
# round 5: ggml backend fused routes (Q|K|V GEMM, fc1 -> fc2 operand, fused LayerNorm operand, fp16 attention output):
# the QKV epilogue: backend tests + whisper_full timing + kernel trace, then the whole GPU suite
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ggml_backend.py \
  > gpurun_out/r05n_tests.log 2>&1; rc=$?
echo "backend tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05n_tests.log | tail -5
[ $rc = 0 ] || exit 1
timeout -k 10 300 bash diag/ggml_backend_timing.sh > gpurun_out/r05n_gb.log 2>&1 || { tail -5 gpurun_out/r05n_gb.log; exit 1; }
grep -E "graph|bitwise" gpurun_out/r05n_gb.log | grep -v nograph
W=/tmp/q2a_gb
for m in f16 q4_k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n_prof_$m -o gb --output-format csv -- \
    oracle/_ref/ggml_harness encode $W/full-$m.bin $W/clip0.f32 $W/out_prof.f32 8 > /dev/null || exit 1
done
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r05n_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r05n_suite.log
