set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export Q2A_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_terms.jsonl
rm -f $Q2A_PARITY_LOG
for t in 2 1; do
  echo "terms=$t" >> $Q2A_PARITY_LOG
  Q2A_ATTN_TERMS=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "full_size_vs_reference or attention_matches" > gpurun_out/terms$t.log 2>&1
  Q2A_ATTN_TERMS=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_terms$t.json 2>/dev/null || exit 1
done
