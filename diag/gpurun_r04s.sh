#!/bin/bash
# round 4: LayerNorm + Q8_K with the affine weights held in registers over RPW row groups per workgroup
# (k_ln_q8k_rows, diag/lnrpw2|4 = -DQ2A_LN_RPW) against the product's one group per workgroup: bit-equality of the
# encoder output (16 clips, Q4_K), then alternating benches (layernorm ms per step)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 16 /tmp/eq_base.npy || exit 1
for v in 2 4; do
  Q2A_LIB_PATH=$PWD/diag/lnrpw$v/libq2a.so timeout -k 10 300 python3 diag/lib_equal.py encode q4_k 16 /tmp/eq_$v.npy || exit 1
  python3 diag/lib_equal.py compare /tmp/eq_base.npy /tmp/eq_$v.npy || exit 1
done
for v in base1=$L r4a=diag/lnrpw4/libq2a.so r2a=diag/lnrpw2/libq2a.so base2=$L r4b=diag/lnrpw4/libq2a.so r2b=diag/lnrpw2/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r04s_b_$n.json 2> gpurun_out/r04s_b_$n.err || { tail -5 gpurun_out/r04s_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], pk['layernorm']['ms_per_step'], pk['quant_act']['ms_per_step'])" gpurun_out/r04s_b_$n.json
done
