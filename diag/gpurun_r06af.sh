#!/bin/bash
# round 6 closing check on the final tree (after the r06ad set and the reverted two-rows experiment): whole GPU
# suite, smoke, the default bench line
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/r06af_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06af_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06af_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06af_smoke.log 2>&1 || { tail -5 gpurun_out/r06af_smoke.log; exit 1; }
tail -1 gpurun_out/r06af_smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/r06af_bench_q4k64.json 2> gpurun_out/r06af_bench.err || { tail -5 gpurun_out/r06af_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06af_bench_q4k64.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gemm_fc1']['frac'], d['cpu_baseline']['value'], d['mfma_util']['value'])"
echo done
