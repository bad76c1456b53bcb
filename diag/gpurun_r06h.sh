#!/bin/bash
# round 6 profile set (tag r06h) on the current tree: GPU suite + smoke, the default bench line (CPU baseline at both
# ISA levels, c_group leg), rocprofv3 kernel stats + PMC traffic (profiles/collect.sh) and SQ counters
# (profiles/collect_sq.sh) for q4k64, then the configs[1] / Q4_K one-clip bench lines
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/r06h_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06h_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06h_smoke.log 2>&1 || { tail -5 gpurun_out/r06h_smoke.log; exit 1; }
tail -1 gpurun_out/r06h_smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/r06h_bench_q4k64.json 2> gpurun_out/r06h_bench.err || { tail -5 gpurun_out/r06h_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06h_bench_q4k64.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gemm_fc1']['frac'], d['cpu_baseline']['value'], d['c_group'])"
timeout -k 10 900 bash profiles/collect.sh r06h q4k64 > gpurun_out/r06h_collect.log 2>&1 || { tail -5 gpurun_out/r06h_collect.log; exit 1; }
timeout -k 10 600 bash profiles/collect_sq.sh r06h q4k64 > gpurun_out/r06h_collect_sq.log 2>&1 || { tail -5 gpurun_out/r06h_collect_sq.log; exit 1; }
for c in f16x1 q4kx1; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r06h_bench_$c.json 2> gpurun_out/r06h_err.log || { tail -5 gpurun_out/r06h_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06h_bench_$c.json'));print('$c', d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['avg_launch_source'][:40])"
done
echo done
