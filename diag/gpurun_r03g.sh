#!/bin/bash
# round 3: profile set of the current tree (F32-class attention): rocprofv3 kernel stats + PMC traffic, SQ counters,
# plus an attention co-execution / LDS / transcendental pass
cd /root/repo
bash profiles/collect.sh r03g q4k64 || exit 1
bash profiles/collect_sq.sh r03g q4k64 || exit 1
O=$PWD/gpurun_out/sq_r03g_q4k64
cd /tmp && export TMPDIR=/tmp Q2A_BENCH_DIR=/tmp/q2ab
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --kernel-include-regex "k_attn|k_gemm" -d $O/sq3 -o run --output-format csv -- python3 /root/repo/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/sq3.err
find $O -name "*counter_collection.csv"
