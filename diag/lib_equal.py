"""Bit-equality of two libq2a.so builds on the bench's own workload shape (diagnostic A/B of a variant that must not
change results): each invocation encodes N synthetic 30 s clips with the library named by Q2A_LIB_PATH and saves the
embeddings; `compare A.npy B.npy` checks them bit for bit.
usage: [Q2A_LIB_PATH=...] python diag/lib_equal.py encode q4_k N OUT.npy | compare A.npy B.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))

if sys.argv[1] == "compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    print("bit-identical" if same else f"DIFFER: {int((a != b).sum())} of {a.size}")
    sys.exit(0 if same else 1)

import torch  # noqa: E402
import bench  # noqa: E402
import q2a  # noqa: E402

wt, n, out = sys.argv[2], int(sys.argv[3]), sys.argv[4]
workdir = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
os.makedirs(workdir, exist_ok=True)
e = q2a.Engine(bench.make_model(wt, workdir, 16), device=0)
pcm = torch.from_numpy(bench.synth_clips(0, n)).cuda()
y = torch.empty((n,) + e.out_shape, dtype=torch.float32, device="cuda")
st = e.encode_device(pcm.data_ptr(), pcm.shape[1], [pcm.shape[1]] * n, y.data_ptr())
torch.cuda.synchronize()
assert list(st) == [0] * n
np.save(out, y.cpu().numpy())
print("saved", out, y.shape)
