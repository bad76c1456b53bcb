#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc pass, kernel-trace only) over a 1-step bench: issue/wait breakdown of the
# GEMM and attention kernels.   bash profiles/collect_sq.sh TAG CONFIG
set -e
TAG=${1:-r01}; CFG=${2:-q4k64}
R=$(pwd)
O=$R/gpurun_out/sq_${TAG}_${CFG}
mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_gemm|k_attn|k_rownorm|k_quant" -d $O/sq -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/sq.err
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex "k_gemm|k_attn" -d $O/sq2 -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/sq2.err
find $O -name "*.csv"
