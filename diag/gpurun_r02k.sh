#!/bin/bash
# residual epilogue: parity (block / full-size / batch invariance) then bench q4k64 + f16x64
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02k_parity.log 2>&1
tail -3 gpurun_out/r02k_parity.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02k_q4k64.json
timeout -k 10 300 python3 bench.py --config f16x64 --no-cpu-baseline > gpurun_out/r02k_f16x64.json
python3 -c "
import json
for f in ['q4k64','f16x64']:
    d=json.loads(open('gpurun_out/r02k_'+f+'.json').read().strip().splitlines()[-1])
    print(f, d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['per_kernel'].items()})
"
