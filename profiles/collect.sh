#!/bin/bash
# Round profile collection on the GPU box (run from the repo root through gpurun):
#   bash profiles/collect.sh TAG CONFIG
# 1) rocprofv3 --kernel-trace --stats over a 5-step bench run; 2) two separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# over a 1-step run, summarised by profiles/pmc_summary.py. Outputs land in gpurun_out/prof_TAG/.
set -e
TAG=${1:-r01}; CFG=${2:-q4k64}
R=$(pwd)
O=$R/gpurun_out/prof_${TAG}_${CFG}
mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-host-legs > $O/bench_traced.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gemm|k_attn" -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gemm|k_attn" -d $O/write -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/write.err
find $O -name "*.csv" | head -20
