"""Diagnostic: run the engine's attention (q2a_test_attention, whichever kernel the Q2A_ATTN_* environment selects) on
fixed random Q/K/V for 3 full-size clips and save the output, so two kernel variants can be compared bit for bit
in separate processes:  python3 diag/attn_dump.py OUT.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
import bench  # noqa: E402


def main():
    import torch
    import q2a
    wd = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
    os.makedirs(wd, exist_ok=True)
    path = bench.make_model("q4_k", wd, 16)
    e = q2a.Engine(path, 0)
    B, T, D = 3, 1500, 1280
    g = torch.Generator(device="cpu").manual_seed(1)
    q = (torch.randn(B * T, D, generator=g) * 0.5).cuda()
    k = (torch.randn(B * T, D, generator=g) * 1.5).cuda()
    v = torch.randn(B * T, D, generator=g).cuda()
    out = torch.empty_like(q)
    e.test_attention(q.data_ptr(), k.data_ptr(), v.data_ptr(), B, out.data_ptr())
    torch.cuda.synchronize()
    np.save(sys.argv[1], out.cpu().numpy())
    e.close()


if __name__ == "__main__":
    main()
