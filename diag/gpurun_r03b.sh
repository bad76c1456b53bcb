#!/bin/bash
# round 3: the whole GPU suite on the F32-class attention + staged fp16 epilogues + pipelined host path, then
# same-box bench A/B: r02 library, this tree with fp16 P.V (diag/pv_fp16), this tree
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$PWD/gpurun_out/b_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/b_tests.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/b_tests.log)"
grep -E "FAILED|ERROR" gpurun_out/b_tests.log | head -20
unset Q2A_PARITY_LOG
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'], 'qkv', pk['gemm_qkv']['ms_per_step'], 'fc1', pk['gemm_fc1']['ms_per_step'], 'o', pk['gemm_o']['ms_per_step'], 'fc2', pk['gemm_fc2']['ms_per_step'], 'quant', pk['quant_act']['ms_per_step'], 'ln', pk['layernorm']['ms_per_step'], 'pcie', d.get('pcie_inclusive_frames_per_s'), 'host', d.get('host_api_frames_per_s'), 'value', d['value'])" $1; }
for v in r02=diag/pv_r02/libq2a.so fp16pv=diag/pv_fp16/libq2a.so cur=qwen2-audio-whisper-ggml_amd/lib/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_b_$n.json 2> gpurun_out/b_b_$n.err && s gpurun_out/b_b_$n.json || { tail -20 gpurun_out/b_b_$n.err; exit 1; }
done
