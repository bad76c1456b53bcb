#!/bin/bash
# round 4: where the 8-phase tile's time goes (s_memtime stamps: fc1 lockstep / staggered, O+fc2), then the isolated
# linears and the whole-step A/B of the wave stagger (diag/wstag) and the 64x128 tail at every K (diag/tail3)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
# the whole GPU suite on the product library first (round-4 tests included); a failure is recorded, not fatal
Q2A_PARITY_LOG=$PWD/gpurun_out/r04b_parity_log.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/r04b_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -15 gpurun_out/r04b_tests.log
case $rc in 124|137|134|139) exit 1;; esac
for v in stamps7 stamps7w stamps1; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 300 python3 diag/tile_stamps.py $v > gpurun_out/r04b_$v.json 2> gpurun_out/r04b_$v.err || { tail -5 gpurun_out/r04b_$v.err; exit 1; }
  cat gpurun_out/r04b_$v.json
done
for i in 1 2; do
  for v in base=$L wstag=diag/wstag/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 diag/linear_bench.py q4_k > gpurun_out/r04b_lin_$n$i.json 2>gpurun_out/r04b_lin_$n$i.err || { tail -5 gpurun_out/r04b_lin_$n$i.err; exit 1; }
    cat gpurun_out/r04b_lin_$n$i.json
  done
done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('gemm_qkv', 'gemm_o', 'gemm_fc1', 'gemm_fc2', 'attention')}, d['setup_s'])" $1; }
for i in 1 2; do
for v in base=$L wstag=diag/wstag/libq2a.so t3=diag/tail3/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04b_b_$n$i.json 2> gpurun_out/r04b_b_$n$i.err && s gpurun_out/r04b_b_$n$i.json || { tail -20 gpurun_out/r04b_b_$n$i.err; exit 1; }
done
done
