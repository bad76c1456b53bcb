#!/bin/bash
# round 3: fc2 tail split (Q2A_GEMM_TAIL, K >= 4096 only) — full GPU suite + smoke on the product library, then a
# same-box A/B: product (128x128 tail) vs diag/tail2 (128x256 two-stage tail) vs diag/notail, alternating, two reps
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
Q2A_PARITY_LOG=$PWD/gpurun_out/tb_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/tb_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tb_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], {k: round(pk[k]['ms_per_step'], 2) for k in ('gemm_qkv', 'gemm_o', 'gemm_fc1', 'gemm_fc2', 'attention')})" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in new=$L t2=diag/tail2/libq2a.so nt=diag/notail/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/tb_b_$n$i.json 2> gpurun_out/tb_b_$n$i.err && s gpurun_out/tb_b_$n$i.json || { tail -20 gpurun_out/tb_b_$n$i.err; exit 1; }
done
done
