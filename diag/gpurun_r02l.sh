#!/bin/bash
# batched LUT reads + LDS-DMA GELU quantizer: full GPU suite, then benches (default, fused-Q8K opt-in, F16 64 / 1)
set -e
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02l_gpu.log 2>&1 || { tail -30 gpurun_out/r02l_gpu.log; exit 1; }
tail -2 gpurun_out/r02l_gpu.log
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['per_kernel'].items()})" $1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02l_q4k64.json && s gpurun_out/r02l_q4k64.json
Q2A_FUSE_Q8K=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02l_q4k64_fuse.json && s gpurun_out/r02l_q4k64_fuse.json
timeout -k 10 300 python3 bench.py --config f16x64 --no-cpu-baseline > gpurun_out/r02l_f16x64.json && s gpurun_out/r02l_f16x64.json
timeout -k 10 300 python3 bench.py --config f16x1 --no-cpu-baseline > gpurun_out/r02l_f16x1.json && s gpurun_out/r02l_f16x1.json
