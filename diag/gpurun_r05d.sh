#!/bin/bash
# round 5: (1) small-batch weight prefetch on a side stream (diag/pf4 = q2a_engine.hip -DQ2A_PREFETCH_MAX_B=4) against
# the product on configs[1] (F16, one clip) and Q4_K one clip, alternating; output bit-equality of one clip;
# (2) the GELU+Q8_K kernel's table-lookup bank conflicts as a timing bound (diag/gnoconf = q2a_exact.hip
# -DQ2A_DIAG_GELU_NOCONF: every lane reads entry 0, wrong results) on the default 64-clip bench, per-kernel quant_act.
# Builds: bash diag/build_variant_src.sh q2a_engine pf4 -DQ2A_PREFETCH_MAX_B=4;
#         bash diag/build_variant_src.sh q2a_exact gnoconf -DQ2A_DIAG_GELU_NOCONF
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 300 python3 diag/lib_equal.py encode f16 1 /tmp/eq_base.npy || exit 1
Q2A_LIB_PATH=$PWD/diag/pf4/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode f16 1 /tmp/eq_pf.npy || exit 1
python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_pf.npy || exit 1
pk() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in sys.argv[2:]})" "$@"; }
for cfg in f16x1 q4kx1; do
  for v in base1=$L pf1=diag/pf4/libq2a.so base2=$L pf2=diag/pf4/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-legs > gpurun_out/r05d_${cfg}_$n.json 2> gpurun_out/r05d_${cfg}_$n.err || { tail -5 gpurun_out/r05d_${cfg}_$n.err; exit 1; }
    pk gpurun_out/r05d_${cfg}_$n.json gemm_qkv gemm_o gemm_fc1 gemm_fc2 attention layernorm
  done
done
for v in base1=$L gnc1=diag/gnoconf/libq2a.so base2=$L gnc2=diag/gnoconf/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r05d_q4k64_$n.json 2> gpurun_out/r05d_q4k64_$n.err || { tail -5 gpurun_out/r05d_q4k64_$n.err; exit 1; }
  pk gpurun_out/r05d_q4k64_$n.json quant_act layernorm gemm_fc2 attention
done
