#!/bin/bash
# round 5 closing measurements on the final tree: bench lines + rocprofv3 kernel stats for every config
# (configs[1] f16x1, Q4_K one clip, F16 x64, configs[4] q80bf16x64) and the reference's whisper_full on the ggml
# backend; outputs under gpurun_out/r05w_*
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for cfg in f16x1 q4kx1 f16x64 q80bf16x64; do
  timeout -k 10 400 python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05w_bench_$cfg.json 2> gpurun_out/r05w_bench_$cfg.err || { tail -5 gpurun_out/r05w_bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r05w_bench_$cfg.json
  O=$PWD/gpurun_out/r05w_prof_$cfg; mkdir -p $O
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 /root/repo/bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > $O/bench_traced.json 2> $O/trace.err ) || { tail -5 $O/trace.err; exit 1; }
done
timeout -k 10 600 bash diag/ggml_backend_timing.sh > gpurun_out/r05w_ggml_backend.txt 2>&1; echo "ggml backend rc=$?"; tail -8 gpurun_out/r05w_ggml_backend.txt
