#!/bin/bash
# round 5: small-batch GEMM tiles with 8 waves (diag/nw8: the 64x128 narrow tiles of a single clip's O / fc2 as 4x2
# waves of 16 rows; diag/nw8s: also the 128x128 tiles of its QKV / fc1 as 4x2 waves of 32 rows) — the glds issue of a
# tile's K-step spread over twice the waves, two per SIMD. Same K order per output: the linear tests and the 64-clip
# batch-invariance tests (single clip = these tiles, batch = the 8-phase kernel, bit for bit) on each variant; then
# configs[1] / Q4_K one clip alternating; then the ggml-backend whisper_full kernel profile (drop-in route overhead).
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for v in nw8 nw8s; do
  Q2A_LIB_PATH=$PWD/diag/$v/libq2a.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "linear_matches or batch_invariant or block" > gpurun_out/r05e_tests_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -2 gpurun_out/r05e_tests_$v.log
  [ $rc -eq 0 ] || exit 1
done
pk() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in sys.argv[2:]})" "$@"; }
for cfg in f16x1 q4kx1; do
  for v in base1=$L nw8a=diag/nw8/libq2a.so nw8sa=diag/nw8s/libq2a.so base2=$L nw8b=diag/nw8/libq2a.so nw8sb=diag/nw8s/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-legs > gpurun_out/r05e_${cfg}_$n.json 2> gpurun_out/r05e_${cfg}_$n.err || { tail -5 gpurun_out/r05e_${cfg}_$n.err; exit 1; }
    pk gpurun_out/r05e_${cfg}_$n.json gemm_qkv gemm_o gemm_fc1 gemm_fc2 attention layernorm
  done
done
GB_PROF=1 timeout -k 10 900 bash diag/ggml_backend_timing.sh > gpurun_out/r05e_gb.log 2>&1; rc=$?
echo "backend timing rc=$rc"; grep -v "^$" gpurun_out/r05e_gb.log | tail -8
