#!/bin/bash
# round 6: whole GPU suite on the hygiene tree + whole-line fc1 stores, then fc1-store A/B against the previous
# epilogue (diag/fc1base: HEAD's q2a_gemm.hip) alternating on one box, then one default bench line (c_group leg)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r06c_tests.log
case $rc in 0) ;; *) exit 1;; esac
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/fc1base/libq2a.so; else unset Q2A_LIB_PATH; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06c_${v}_$i.json 2> gpurun_out/r06c_err.log || { tail -5 gpurun_out/r06c_err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06c_${v}_$i.json'));print('$v $i', d['ms_per_step'], d['roofline_gemm_fc1']['avg_launch_ms'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k.startswith('gemm')})"
  done
done
unset Q2A_LIB_PATH
timeout -k 10 500 python3 bench.py --no-cpu-baseline > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || { tail -5 gpurun_out/r06c_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06c_bench.json'));print(d['ms_per_step'], json.dumps(d['roofline']), json.dumps(d['c_group']))"
