set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -iE "MFMA|SQ_BUSY|GRBM_GUI|LDS_BANK|SQ_INSTS_VALU\b|SQ_WAIT" gpurun_out/counters_list.txt | head -80 > gpurun_out/counters_grep.txt || true
