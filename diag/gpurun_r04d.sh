#!/bin/bash
# round 4: the persistent fc1 kernel (diag/pers: Q2A_GEMM_PERSIST=1) — GPU suite on it, then the whole-step A/B against
# the product library (alternating, same box); then the closing per-config measurements (diag/gpurun_r04_configs.sh)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
Q2A_LIB_PATH=$PWD/diag/pers/libq2a.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04d_pers_tests.log 2>&1; rc=$?
echo "pers gpu tests rc=$rc"; tail -15 gpurun_out/r04d_pers_tests.log
case $rc in 0) ;; *) exit 1;; esac
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('gemm_qkv', 'gemm_o', 'gemm_fc1', 'gemm_fc2', 'attention')})" $1; }
for i in 1 2; do
for v in base=$L pers=diag/pers/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04d_b_$n$i.json 2> gpurun_out/r04d_b_$n$i.err && s gpurun_out/r04d_b_$n$i.json || { tail -20 gpurun_out/r04d_b_$n$i.err; exit 1; }
done
done
( cd /tmp && export TMPDIR=/tmp && Q2A_LIB_PATH=/root/repo/diag/pers/libq2a.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r04d_pers_prof -o run --output-format csv -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > /root/repo/gpurun_out/r04d_pers_prof.json 2> /root/repo/gpurun_out/r04d_pers_prof.err ) || { tail -5 gpurun_out/r04d_pers_prof.err; exit 1; }
grep -h "k_gemm" gpurun_out/r04d_pers_prof/run_kernel_stats.csv | cut -d, -f1-4
bash diag/gpurun_r04_configs.sh
