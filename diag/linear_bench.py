"""Time the engine's batched linears in isolation (diagnostic A/B of GEMM variants on FIXED inputs, so a variant that
computes wrong values cannot change the operand data — and with it the chip's power state — of the timed launches).
q2a_test_linear = activation quantizer + one GEMM (plain f32 store epilogue) for one weight matrix of one layer.
usage: [Q2A_LIB_PATH=diag/<v>/libq2a.so] python diag/linear_bench.py [q4_k|f16] [M]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
import bench  # noqa: E402
import q2a  # noqa: E402

wt = sys.argv[1] if len(sys.argv) > 1 else "q4_k"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 96000
workdir = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
os.makedirs(workdir, exist_ok=True)
eng = q2a.Engine(bench.make_model(wt, workdir, 16), device=0)
D, F = 1280, 5120
st = torch.cuda.Stream()   # a non-default stream: handle 0 would select the engine's own stream
torch.cuda.set_stream(st)
res = {"lib": os.environ.get("Q2A_LIB_PATH", "default"), "wt": wt, "M": M}
g = torch.Generator(device="cuda").manual_seed(1)
for which, name, K, N in [(0, "qkv", D, 3 * D), (1, "o", D, D), (2, "fc1", D, F), (3, "fc2", F, D)]:
    x = torch.randn((M, K), device="cuda", generator=g, dtype=torch.float32) * (0.3 if which == 3 else 1.0)
    y = torch.empty((M, N), device="cuda", dtype=torch.float32)
    for _ in range(3):
        eng.test_linear(1, which, x.data_ptr(), M, y.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        eng.test_linear(1, which, x.data_ptr(), M, y.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res[name] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
print(json.dumps(res))
