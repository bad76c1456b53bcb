#!/bin/bash
# round 5: the 8-phase GEMM with glds issued inside the MFMA segments (diag/gldsc = -DQ2A_GEMM_GLDS_C=1) against the product:
# 64-clip output bit-equality (Q4_K and F16: same K order, so identical bits), isolated linears alternating, then
# alternating whole-step benches (per-kernel ms per step). Build: bash diag/build_variant.sh gldsc -DQ2A_GEMM_GLDS_C=1
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for wt in q4_k f16; do
  timeout -k 10 300 python3 diag/lib_equal.py encode $wt 64 /tmp/eq_base.npy || exit 1
  Q2A_LIB_PATH=$PWD/diag/gldsc/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode $wt 64 /tmp/eq_gldsc.npy || exit 1
  python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_gldsc.npy || exit 1
done
rm -f /tmp/eq_*.npy
for r in 1 2; do
  for v in base=$L gldsc=diag/gldsc/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    for wt in q4_k f16; do
      Q2A_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 diag/linear_bench.py $wt > gpurun_out/r05c_lin_${n}_${wt}_$r.json || exit 1
      echo "$n $wt $(cat gpurun_out/r05c_lin_${n}_${wt}_$r.json)"
    done
  done
done
for v in base1=$L gldsca=diag/gldsc/libq2a.so base2=$L gldscb=diag/gldsc/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05c_b_$n.json 2> gpurun_out/r05c_b_$n.err || { tail -5 gpurun_out/r05c_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'], {k: pk[k]['ms_per_step'] for k in ('gemm_qkv','gemm_o','gemm_fc1','gemm_fc2','attention')})" gpurun_out/r05c_b_$n.json
done
