#!/bin/bash
# round 5: Q4_K 8-phase GEMM with the B fragments of a block's first phase read before its block start (diag/bsr =
# 64-clip output bit-equality (Q4_K and F16: same K order, so identical bits), isolated linears alternating, then
# alternating whole-step benches (per-kernel ms per step). Build: bash diag/build_variant.sh bsr -DQ2A_GEMM_BSR=1
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
# the GEMM parity tests through the variant (linears at every tile regime + the 64-clip batch invariance)
Q2A_LIB_PATH=$PWD/diag/bsr/libq2a.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "linear or batch or encoder_full or block_batched" > gpurun_out/r05r_tests.log 2>&1; rc=$?
echo "bsr tests rc=$rc"; tail -3 gpurun_out/r05r_tests.log
[ $rc = 0 ] || exit 1
for wt in q4_k f16; do
  timeout -k 10 300 python3 diag/lib_equal.py encode $wt 64 /tmp/eq_base.npy || exit 1
  Q2A_LIB_PATH=$PWD/diag/bsr/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode $wt 64 /tmp/eq_bsr.npy || exit 1
  python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_bsr.npy || exit 1
done
rm -f /tmp/eq_*.npy
for r in 1 2; do
  for v in base=$L bsr=diag/bsr/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    for wt in q4_k f16; do
      Q2A_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 diag/linear_bench.py $wt > gpurun_out/r05r_lin_${n}_${wt}_$r.json || exit 1
      echo "$n $wt $(cat gpurun_out/r05r_lin_${n}_${wt}_$r.json)"
    done
  done
done
for v in base1=$L bsra=diag/bsr/libq2a.so base2=$L bsrb=diag/bsr/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05r_b_$n.json 2> gpurun_out/r05r_b_$n.err || { tail -5 gpurun_out/r05r_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'], {k: pk[k]['ms_per_step'] for k in ('gemm_qkv','gemm_o','gemm_fc1','gemm_fc2','attention')})" gpurun_out/r05r_b_$n.json
done
