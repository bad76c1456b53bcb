#!/bin/bash
# round 5: what the GEMM epilogues' global stores cost per class (timing diagnostic, WRONG results downstream: the
# stores predicated off — every epilogue: diag/nostore; only the QKV V^T scatter: diag/novt), against the product
# library; per-class times from the bench's event pass (the next lever in DESIGN.md §7: the QKV epilogue)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for i in 1 2; do
  for v in base nostore novt; do
    if [ $v = base ]; then unset Q2A_LIB_PATH; else export Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so; fi
    timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05zh_q4k64_${v}_$i.json 2> gpurun_out/r05zh_err.log || { tail -5 gpurun_out/r05zh_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r05zh_q4k64_${v}_$i.json'));print('q4k64 $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k.startswith('gemm')})"
  done
done
