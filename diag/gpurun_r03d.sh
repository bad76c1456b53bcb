#!/bin/bash
# round 3: regime bit-equality after the contraction fix, then the previously failing GPU tests
cd /root/repo
mkdir -p gpurun_out /tmp/q2ac
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model /tmp/q2ac/tiny-f16.bin tiny f16 0x51A2 16 > /dev/null && $T gen-model /tmp/q2ac/full-f16.bin full f16 0x51A2 16 > /dev/null || exit 1
for m in tiny full; do
  timeout -k 10 200 python3 diag/regime_diff.py /tmp/q2ac/$m-f16.bin 0 | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$m', d['what'], d['n_diff'], d['max_abs'])" || exit 1
done
export Q2A_PARITY_LOG=$PWD/gpurun_out/d_parity.jsonl
rm -f $Q2A_PARITY_LOG
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_isolated.py \
    tests/test_bench_launch.py "tests/test_gpu_parity.py::test_encoder_bench_batch_64_is_batch_invariant" \
    "tests/test_gpu_parity.py::test_encoder_full_size_vs_reference_samples" "tests/test_gpu_parity.py::test_encoder_tiny_quantized_vs_reference" \
    "tests/test_gpu_parity.py::test_encoder_tiny_f16_vs_reference" > gpurun_out/d_tests.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/d_tests.log)"
grep -E "^E   .*Error|FAILED" gpurun_out/d_tests.log | head -20
