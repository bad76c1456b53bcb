#!/bin/bash
# attention stall evidence: counter list, then SQ passes (each its own rocprofv3 --pmc run) on k_attn_g
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq_attn
mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1
timeout -k 10 400 python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err || exit 1
run() { n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_attn" -d $O/$n -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/$n.err; echo "$n rc=$?"; }
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC
run b SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES
run c SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP GRBM_GUI_ACTIVE GRBM_COUNT
run d SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAIT_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
find $O -name "*.csv"
grep -i "^SQ_\|^ *SQ_" $O/counters_list.txt | head -3
