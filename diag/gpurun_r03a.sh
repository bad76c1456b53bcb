#!/bin/bash
# round 3: attention P.V precision variants — end-to-end parity against the reference golden + the reference's own
# cross-build spread (diag/pv_parity.py), then same-box attention timing of each variant (bench per_kernel)
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
timeout -k 10 900 python3 -u diag/pv_parity.py gpurun_out/a_pv.jsonl r02=diag/pv_r02/libq2a.so rtz_l=$L \
    phl=diag/pv_phl/libq2a.so vhl=diag/pv_vhl/libq2a.so phl_vhl=diag/pv_phl_vhl/libq2a.so > gpurun_out/a_pv.log 2>&1 \
    || { tail -30 gpurun_out/a_pv.log; exit 1; }
echo parity done
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], 'attention', d['per_kernel']['attention']['ms_per_step'])" $1; }
for i in 1; do
  for v in r02=diag/pv_r02/libq2a.so rtz_l=$L phl=diag/pv_phl/libq2a.so vhl=diag/pv_vhl/libq2a.so phl_vhl=diag/pv_phl_vhl/libq2a.so; do
    n=${v%%=*}; lib=${v#*=}
    Q2A_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/a_b_$n.json 2> gpurun_out/a_b_$n.err && s gpurun_out/a_b_$n.json || { tail -20 gpurun_out/a_b_$n.err; exit 1; }
  done
done
