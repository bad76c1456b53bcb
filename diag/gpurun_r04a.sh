#!/bin/bash
# round 4: (1) the round's new / changed parity tests on the product library; (2) the 8-phase wave stagger (waves 4-7
# one barrier behind; diag/wstag) and the 64x128 deep-pipeline tail at every K (diag/tail3): parity subset of each
# variant, isolated linears, then whole-step A/B alternating against the product
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$PWD/gpurun_out/r04a_parity_log.jsonl
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "compact or nan or attention_matches or full_size_bench or invariant or block_batched or device_blob" > gpurun_out/r04a_tests_base.log 2>&1; rc=$?; echo "tests base rc=$rc"; tail -3 gpurun_out/r04a_tests_base.log; [ $rc = 0 ] || exit 1
unset Q2A_PARITY_LOG
for v in wstag; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "invariant or linear" > gpurun_out/r04a_tests_$v.log 2>&1; rc=$?; echo "tests $v rc=$rc"; tail -2 gpurun_out/r04a_tests_$v.log; [ $rc = 0 ] || exit 1
done
for i in 1 2; do
  for v in base=$L wstag=diag/wstag/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 diag/linear_bench.py q4_k > gpurun_out/r04a_lin_$n$i.json 2>gpurun_out/r04a_lin_$n$i.err || { tail -5 gpurun_out/r04a_lin_$n$i.err; exit 1; }
    cat gpurun_out/r04a_lin_$n$i.json
  done
done
for v in base=$L wstag=diag/wstag/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 diag/linear_bench.py f16 > gpurun_out/r04a_linf16_$n.json 2>/dev/null || exit 1
  cat gpurun_out/r04a_linf16_$n.json
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('gemm_qkv', 'gemm_o', 'gemm_fc1', 'gemm_fc2', 'attention')}, d['setup_s'])" $1; }
for i in 1 2; do
for v in base=$L wstag=diag/wstag/libq2a.so t3=diag/tail3/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04a_b_$n$i.json 2> gpurun_out/r04a_b_$n$i.err && s gpurun_out/r04a_b_$n$i.json || { tail -20 gpurun_out/r04a_b_$n$i.err; exit 1; }
done
done
Q2A_LIB_PATH=$PWD/diag/tail3/libq2a.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "invariant or full_size_bench" > gpurun_out/r04a_tests_tail3.log 2>&1; rc=$?; echo "tests tail3 rc=$rc"; tail -2 gpurun_out/r04a_tests_tail3.log
