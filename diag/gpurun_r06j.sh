#!/bin/bash
# round 6: the other configs' bench lines on the current tree (F16 x64, configs[4] per rank q80bf16x64), and the
# configs[1] rocprofv3 kernel stats (profiles/collect.sh r06j f16x1)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in f16x64 q80bf16x64; do
  timeout -k 10 500 python3 bench.py --config $c --no-cpu-baseline --no-c-group > gpurun_out/r06j_bench_$c.json 2> gpurun_out/r06j_err.log || { tail -5 gpurun_out/r06j_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06j_bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
done
timeout -k 10 600 bash profiles/collect.sh r06j f16x1 > gpurun_out/r06j_collect.log 2>&1 || { tail -5 gpurun_out/r06j_collect.log; exit 1; }
echo done
