#!/bin/bash
# round 3: profile set of the current tree (rocprofv3 kernel stats + PMC traffic with --no-host-legs, SQ counters,
# attention co-execution pass), then the default bench line with the CPU baseline
cd /root/repo
bash profiles/collect.sh r03l q4k64 || exit 1
bash profiles/collect_sq.sh r03l q4k64 || exit 1
O=$PWD/gpurun_out/sq_r03l_q4k64
( cd /tmp && export TMPDIR=/tmp Q2A_BENCH_DIR=/tmp/q2ab && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --kernel-include-regex "k_attn|k_gemm" -d $O/sq3 -o run --output-format csv -- python3 /root/repo/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/sq3.err ) || exit 1
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 bench.py > gpurun_out/l_bench.json 2> gpurun_out/l_bench.err || { tail -20 gpurun_out/l_bench.err; exit 1; }
tail -c 1500 gpurun_out/l_bench.json
