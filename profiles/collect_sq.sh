#!/bin/bash
# SQ counter passes (each its own rocprofv3 --pmc run, kernel-trace only, within the gfx950 per-pass slot limits:
# <= 8 SQ, 2 GRBM) over a 1-step bench: MFMA busy cycles, issue/wait breakdown, LDS use of the GEMM and attention
# kernels. Summarised by profiles/sq_summary.py.    bash profiles/collect_sq.sh TAG CONFIG
set -e
TAG=${1:-r02}; CFG=${2:-q4k64}
R=$(pwd)
O=$R/gpurun_out/sq_${TAG}_${CFG}
mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 400 python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_gemm|k_attn" -d $O/sq2 -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/sq2.err
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_gemm|k_attn|k_rownorm|k_quant|k_gelu" -d $O/sq -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/sq.err
find $O -name "*.csv"
