#!/bin/bash
# round 6 closing set, part B (tag r06ad): rocprofv3 kernel stats + PMC traffic for the Q4_K one-clip config, then the
# bench lines of the other configs
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 bash profiles/collect.sh r06ad q4kx1 > gpurun_out/r06ad_collect2.log 2>&1 || { tail -5 gpurun_out/r06ad_collect2.log; exit 1; }
for c in f16x1 q4kx1 f16x64 q80bf16x64; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline --no-c-group > gpurun_out/r06ad_bench_$c.json 2> gpurun_out/r06ad_err.log || { tail -5 gpurun_out/r06ad_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06ad_bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['frac'], d['roofline']['traffic_source'])"
done
echo done
