set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./diag/mfma_q4k_ceiling > gpurun_out/mfma_ceiling.json 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python -u bench.py --config f16x1 --no-cpu-baseline > gpurun_out/bench_f16x1.json 2> gpurun_out/bench_f16x1.err
