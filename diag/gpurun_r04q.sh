#!/bin/bash
# round 4: what biased-uint8 activation codes would cost the 8-phase GEMMs — the unpack VALU (4 v_perm_b32 +
# 4 v_pk_add_f16 per 8-code fragment) issued as identity operations (diag/u8unpack, results bit-identical, so the
# operand data and the chip's power state are the product's) against the product, alternating, per-kernel ms/step
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for v in base1=$L u8a=diag/u8unpack/libq2a.so base2=$L u8b=diag/u8unpack/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r04q_b_$n.json 2> gpurun_out/r04q_b_$n.err || { tail -5 gpurun_out/r04q_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']; print(sys.argv[1], d['ms_per_step'], {k: pk[k]['ms_per_step'] for k in ('gemm_qkv','gemm_o','gemm_fc1','gemm_fc2')})" gpurun_out/r04q_b_$n.json
done
