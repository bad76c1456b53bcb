#!/bin/bash
# round-2 end validation (after the attention lazy re-basing, interleaved QK chains, Q4_K block-0 start, grouped Q4_K backend launch): the whole GPU suite, smoke(), the default bench and the single-clip / exact-Q8_0 configs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/z_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/z_gputest.log 2>&1 || { tail -30 gpurun_out/z_gputest.log; exit 1; }
tail -1 gpurun_out/z_gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 || { tail -20 gpurun_out/z_smoke.log; exit 1; }
echo "smoke ok: $(tail -1 gpurun_out/z_smoke.log)"
timeout -k 10 400 python3 -u bench.py > gpurun_out/z_bench_q4k64.json 2> gpurun_out/z_bench.err || exit 1
for c in q4kx1 f16x1 q80bf16x64 f16x64; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/z_bench_$c.json 2> gpurun_out/z_bench_$c.err || exit 1
done
for c in q4k64 q4kx1 f16x1 q80bf16x64 f16x64; do python3 -c "
import json,sys
d=json.loads(open('gpurun_out/z_bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
