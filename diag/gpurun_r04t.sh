#!/bin/bash
# round 4: Q / K tiles of the Q4_K QKV GEMM on persistent tiles (diag/pqkv = -DQ2A_GEMM_PERSIST_QKV=1, V's tiles a
# second launch) against the product and against HEAD's GEMM source (diag/headgemm: the n_base / n_end launch fields
# must cost nothing): 64-clip output bit-equality, the 64-clip batch-invariance test on the variant, alternating
# benches (per-kernel ms per step). Builds: git apply diag/qkv_persistent.patch && bash diag/build_variant.sh pqkv
# -DQ2A_GEMM_PERSIST_QKV=1 (then revert); diag/headgemm = libq2a.so with the pre-patch q2a_gemm.hip
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_base.npy || exit 1
for v in pqkv headgemm; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 64 /tmp/eq_$v.npy || exit 1
  python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_$v.npy || exit 1
done
rm -f /tmp/eq_*.npy
Q2A_LIB_PATH=$PWD/diag/pqkv/libq2a.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "batch_64 or batch_invariant or block_batched" > gpurun_out/r04t_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04t_tests.log; [ $rc -eq 0 ] || exit 1
for v in head1=diag/headgemm/libq2a.so base1=$L pq1=diag/pqkv/libq2a.so head2=diag/headgemm/libq2a.so base2=$L pq2=diag/pqkv/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r04t_b_$n.json 2> gpurun_out/r04t_b_$n.err || { tail -5 gpurun_out/r04t_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in ('gemm_qkv','gemm_o','gemm_fc1','gemm_fc2','attention')})" gpurun_out/r04t_b_$n.json
done
