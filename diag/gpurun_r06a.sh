#!/bin/bash
# round 6 start: the round-5 tree's numbers on this round's first box (q4k64 + configs[1] per-kernel breakdown)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for c in q4k64 f16x1 q4k64 f16x1; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06a_$c.json 2> gpurun_out/r06a_err.log || { tail -5 gpurun_out/r06a_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06a_$c.json'));print('$c', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
done
