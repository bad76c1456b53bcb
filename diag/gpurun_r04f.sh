#!/bin/bash
# round 4: persistent fc1 as the product — whole GPU suite + smoke, the default bench line; then the layer-0 node
# trace of the ggml-backend drop-in path (diag/backend_l0_trace.py)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/r04f_parity_log.jsonl
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -15 gpurun_out/r04f_tests.log
case $rc in 0|1) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 || { tail -20 gpurun_out/r04f_smoke.log; exit 1; }
echo "smoke ok"; tail -2 gpurun_out/r04f_smoke.log
timeout -k 10 300 python3 diag/backend_l0_trace.py gpu diag/_l0ref.npz > gpurun_out/r04f_backend_l0.jsonl 2> gpurun_out/r04f_backend_l0.err || { tail -5 gpurun_out/r04f_backend_l0.err; exit 1; }
cat gpurun_out/r04f_backend_l0.jsonl
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -5 gpurun_out/r04f_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04f_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline']['all_weight_gemms_tflops'])"
