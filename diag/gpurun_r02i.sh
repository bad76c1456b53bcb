set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd); O=$R/gpurun_out/sq_attn; mkdir -p $O
export Q2A_BENCH_DIR=/tmp/q2ab
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err
for v in 0 1; do
Q2A_ATTN_V1=$v timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "k_attn" -d $O/m$v -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/m$v.err || exit 1
Q2A_ATTN_V1=$v timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_attn" -d $O/w$v -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/w$v.err || exit 1
done
