#!/bin/bash
# (this container, after gpurun merged gpurun_out/) copy one closing set's artifacts into profiles/ under the TAG:
# rocprofv3 kernel stats, the bench line under rocprofv3, the PMC traffic summary and the SQ summary of each config
# found, and the default bench line / parity log of part A.      bash profiles/store_set.sh TAG SCRIPT
set -e
TAG=$1; SCRIPT=${2:-diag/gpurun_$1.sh}
cd /root/repo
for d in gpurun_out/prof_${TAG}_*; do
  [ -d "$d" ] || continue
  CFG=${d#gpurun_out/prof_${TAG}_}
  cp $d/trace/run_kernel_stats.csv profiles/${TAG}_${CFG}_rocprof_kernel_stats.csv
  cp $d/bench_traced.json profiles/${TAG}_${CFG}_bench_under_rocprof.json
  python3 profiles/pmc_summary.py $d/fetch/run_counter_collection.csv $d/write/run_counter_collection.csv \
    profiles/${TAG}_${CFG}_pmc_traffic.json \
    "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --config $CFG --steps 1 --warmup 0 (profiles/collect.sh $TAG $CFG)"
  echo "stored $CFG"
done
for d in gpurun_out/sq_${TAG}_*; do
  [ -d "$d" ] || continue
  CFG=${d#gpurun_out/sq_${TAG}_}
  python3 profiles/sq_summary.py $d/sq2/run_counter_collection.csv $d/sq/run_counter_collection.csv \
    profiles/${TAG}_${CFG}_sq_mfma.json "rocprofv3 --pmc SQ passes (profiles/collect_sq.sh $TAG $CFG, $SCRIPT)"
  echo "stored SQ $CFG"
done
for f in gpurun_out/${TAG}_bench_*.json gpurun_out/${TAG}_parity_log.jsonl; do
  [ -f "$f" ] && cp $f profiles/ && echo "stored $(basename $f)"
done
exit 0
