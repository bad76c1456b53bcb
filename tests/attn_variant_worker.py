"""One attention-kernel variant on the GPU (tests/test_gpu_attention_variants.py): the engine's q2a_test_attention on
seeded random Q/K/V, through whichever library Q2A_LIB_PATH names (a diag/ variant build, or the shipped library when
unset). Writes the output to OUT.npy.    python tests/attn_variant_worker.py MODEL OUT.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))

B, T, D = 2, 1500, 256   # the tiny model's attention shape (4 heads of 64)


def inputs():
    rng = np.random.default_rng(7)
    q = (rng.standard_normal((B * T, D)) * 0.5).astype(np.float32)
    k = (rng.standard_normal((B * T, D)) * 1.5).astype(np.float32)
    v = rng.standard_normal((B * T, D)).astype(np.float32)
    return q, k, v


def main():
    import torch
    import q2a
    e = q2a.Engine(sys.argv[1], 0)
    q, k, v = (torch.from_numpy(a).cuda() for a in inputs())
    out = torch.empty_like(q)
    e.test_attention(q.data_ptr(), k.data_ptr(), v.data_ptr(), B, out.data_ptr())
    torch.cuda.synchronize()
    np.save(sys.argv[2], out.cpu().numpy())
    e.close()


if __name__ == "__main__":
    main()
