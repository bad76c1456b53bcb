#!/bin/bash
# round 5: locate the q4_k 64-clip batch-invariance failure of the ALT schedule: ALT with and without the persistent
# fc1 kernel (diag/altnp = -DQ2A_GEMM_ALT=1 -DQ2A_GEMM_PERSIST=0), batch-64 and one-block tests
cd /root/repo
mkdir -p gpurun_out
for v in altnp alt; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "batch_64 or block_batched" > gpurun_out/r05i_$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -E "passed|failed|^FAILED" gpurun_out/r05i_$v.log
  case $rc in 0|1) ;; *) exit 1;; esac
done
