set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 500 python -u diag/layer_trace.py --wt q4_k --out gpurun_out/layer_trace_q4_k.json > gpurun_out/trace.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
