set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export Q2A_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_attn.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16_act.py -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_pp.json 2>/dev/null &&
Q2A_ATTN_V1=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_v1.json 2>/dev/null &&
timeout -k 10 300 python -u bench.py --config q80bf16x64 --no-cpu-baseline --steps 5 > gpurun_out/bench_bf16_pp.json 2>/dev/null
exit $rc
