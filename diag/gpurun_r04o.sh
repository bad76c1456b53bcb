#!/bin/bash
# round 4: where k_mel_frames spends its time — timing-only builds without the filterbank loop (diag/melNOFB) or the
# 25-point leaf DFTs (diag/melNODFT) against the product (mel ms per step from the bench's per-kernel events)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for v in base=$L nofft=diag/melNOFFT/libq2a.so flog=diag/melFLOG/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/r04o_b_$n.json 2> gpurun_out/r04o_b_$n.err || { tail -5 gpurun_out/r04o_b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['per_kernel']['mel'])" gpurun_out/r04o_b_$n.json
done
