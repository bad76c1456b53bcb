#!/bin/bash
# round 3: GPU suite on the tree (attention: -m' folded into the QK^T MFMAs, sum-based lazy re-base; QKV V^T hi|lo
# epilogue without the half-workgroup serialisation), tiny layer-0 trace vs the reference, same-box A/B vs HEAD
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
export Q2A_PARITY_LOG=$PWD/gpurun_out/h_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/h_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/h_tests.log)"
grep -E "^FAILED|^ERROR" gpurun_out/h_tests.log | head -20
[ $rc -le 1 ] || exit $rc
unset Q2A_PARITY_LOG
timeout -k 10 200 python3 diag/tiny_l0_trace.py gpu diag/_l0ref.npz > gpurun_out/h_l0.jsonl 2> gpurun_out/h_l0.err || { tail -5 gpurun_out/h_l0.err; exit 1; }
cat gpurun_out/h_l0.jsonl
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'], 'qkv', pk['gemm_qkv']['ms_per_step'], 'fc1', pk['gemm_fc1']['ms_per_step'], 'o', pk['gemm_o']['ms_per_step'], 'fc2', pk['gemm_fc2']['ms_per_step'], 'quant', pk['quant_act']['ms_per_step'], 'ln', pk['layernorm']['ms_per_step'], 'pcie', d.get('pcie_inclusive_frames_per_s'), 'host', d.get('host_api_frames_per_s'), 'value', d['value'])" $1; }
for i in 1 2; do
for v in prev=diag/prev/libq2a.so cur=qwen2-audio-whisper-ggml_amd/lib/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/h_b_$n$i.json 2> gpurun_out/h_b_$n$i.err && s gpurun_out/h_b_$n$i.json || { tail -20 gpurun_out/h_b_$n$i.err; exit 1; }
done
done
