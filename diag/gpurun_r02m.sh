#!/bin/bash
# PMC passes over the bandwidth kernels (GELU+Q8_K quantizer, LayerNorm+Q8_K, attention-output quantizer)
set -e
R=$(pwd)
O=$R/gpurun_out/bw
mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
K="k_gelu|k_rownorm|k_quant"
timeout -k 10 300 python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err
run() { n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d $O/$n -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/$n.err; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
run sq2 SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE
run tcc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum
run ta TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum
cd $R && python3 diag/pmc_kernels.py $(find $O -name "*counter_collection.csv") > $O/summary.txt && cat $O/summary.txt
