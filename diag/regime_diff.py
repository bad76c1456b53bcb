"""Where do the small-tile (one clip) and 8-phase (30 clips) regimes diverge? One encoder block through
q2a_test_block_taps on clip 0 alone and on 30 copies of it: compares the four GEMM A operands (LN1 -> QKV,
attention -> O, LN2 -> fc1, GELU -> fc2) and the block output bit for bit (diagnostic; prints JSON lines).
usage: [Q2A_LIB_PATH=...] python diag/regime_diff.py MODEL [layer]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
import q2a  # noqa: E402

model = sys.argv[1]
layer = int(sys.argv[2]) if len(sys.argv) > 2 else 0
e = q2a.Engine(model, device=0)
T, D = e.info.n_audio_ctx, e.info.n_audio_state
F = 4 * D
rng = np.random.default_rng(3)
x0 = (rng.standard_normal((T, D)) * 0.5).astype(np.float32)


def run(B):
    x = torch.from_numpy(np.tile(x0, (B, 1))).cuda()
    taps = [torch.zeros((B * T, D), dtype=torch.float16, device="cuda") for _ in range(3)] + \
           [torch.zeros((B * T, F), dtype=torch.float16, device="cuda")]
    e.test_block_taps(layer, x.data_ptr(), B, [t.data_ptr() for t in taps])
    torch.cuda.synchronize()
    return [t[:T].cpu().numpy() for t in taps] + [x[:T].cpu().numpy()]


a, b = run(1), run(30)
names = ["ln1_op", "attn_op", "ln2_op", "fc2_op", "block_out"]
for n, u, v in zip(names, a, b):
    uu, vv = u.astype(np.float64), v.astype(np.float64)
    ne = int((u != v).sum())
    rows = np.nonzero((u != v).any(axis=1))[0]
    cols = np.nonzero((u != v).any(axis=0))[0]
    print(json.dumps({"lib": os.environ.get("Q2A_LIB_PATH", "default"), "what": n, "n_diff": ne,
                      "max_abs": float(np.abs(uu - vv).max()), "first_rows": rows[:8].tolist(),
                      "first_cols": cols[:8].tolist(), "n_rows": int(len(rows)), "n_cols": int(len(cols))}), flush=True)
e.close()
