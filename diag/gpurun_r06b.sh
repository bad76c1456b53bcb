#!/bin/bash
# round 6: group over an open engine (q2a_group_open_with), whisper / backend suites, the bench line's new roofline
# objects and c_group leg
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_whisper_api.py tests/test_gpu_ggml_backend.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r06b_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err || { tail -5 gpurun_out/r06b_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06b_bench.json'));print(d['ms_per_step'], json.dumps(d['roofline']), json.dumps(d['roofline_gemm_fc1']), json.dumps(d['c_group']))"
