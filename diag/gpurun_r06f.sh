#!/bin/bash
# round 6: GPU suite after the NULL-stream change (calls with stream = NULL run on the legacy stream itself), then
# NULL vs explicit stream again and the bench lines of configs[1], Q4_K one clip and configs[2]
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r06f_tests.log
case $rc in 0) ;; *) exit 1;; esac
rm -f gpurun_out/r06f_null_stream.jsonl
for c in f16x1 q4kx1; do
  timeout -k 10 300 python3 diag/null_stream_ab.py $c >> gpurun_out/r06f_null_stream.jsonl 2> gpurun_out/r06f_err.log || { tail -5 gpurun_out/r06f_err.log; exit 1; }
done
cat gpurun_out/r06f_null_stream.jsonl
for c in f16x1 q4kx1 q4k64; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r06f_$c.json 2> gpurun_out/r06f_err.log || { tail -5 gpurun_out/r06f_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06f_$c.json'));print('$c', d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['frac'], d['roofline_gemm_fc1']['avg_launch_ms'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
done
