#!/bin/bash
# round 4: mel kernel with one clip-maximum atomic per workgroup (q2a_exact.hip k_mel_frames) — GPU suite + bench
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/r04p_parity_log.jsonl
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -8 gpurun_out/r04p_tests.log | cut -c1-300
case $rc in 0|1) ;; *) exit 1;; esac
unset Q2A_PARITY_LOG
for i in 1 2; do
timeout -k 10 400 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r04p_bench$i.json 2> gpurun_out/r04p_bench$i.err || { tail -5 gpurun_out/r04p_bench$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04p_bench$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items()})"
done
