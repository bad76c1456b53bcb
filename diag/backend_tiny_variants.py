"""Tiny F16 model: the reference's whisper_full on the Q2A ggml backend under its test hooks (fused / generic
attention, hi/lo / exact-f32 conv) against the golden build, clip-averaged over the cross-build fixture's clips, and
the engine's own distance, to locate where the backend's rounding departs from the engine's (round 3 diagnostic)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
TOOL = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "bin", "q2a_tool")
H = os.path.join(ROOT, "oracle", "_ref", "ggml_harness")
W = "/tmp/q2a_btv"
os.makedirs(W, exist_ok=True)
g = dict(np.load(os.path.join(ROOT, "tests/golden/golden.npz")))
xc = dict(np.load(os.path.join(ROOT, "tests/golden/xclips.npz")))
rows = g["rows_stride5"]
model = os.path.join(W, "tiny-f16.bin")
if not os.path.exists(model):
    subprocess.check_call([TOOL, "gen-model", model, "tiny", "f16", "0x51A2", "16"])
clips = [0, 101, 102, 103, 104]
pcm = {}
for c in clips:
    p = os.path.join(W, f"clip{c}.f32")
    if not os.path.exists(p):
        subprocess.check_call([TOOL, "synth-clip", p, "480000", str(c)])
    pcm[c] = p


def ref(c):
    return g["tiny_f16_c0"][rows] if c == 0 else xc[f"tiny_f16_c{c}_rows"]


def stats(a, b):
    d = a.astype(np.float64) - b.astype(np.float64)
    return float(np.abs(d).max() / np.abs(b).max()), float(np.linalg.norm(d) / np.linalg.norm(b))


def backend(env):
    out = {}
    for c in clips:
        o = os.path.join(W, f"b{c}.f32")
        e = dict(os.environ, **env)
        r = subprocess.run([H, "encode", model, pcm[c], o, "1"], capture_output=True, text=True, env=e, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        info = json.loads(r.stdout.strip().splitlines()[-1])
        out[c] = np.fromfile(o, dtype=np.float32).reshape(info["ne1"], info["ne0"])
    return out


import q2a  # noqa: E402
eng = q2a.Engine(model, device=0)
eo, _ = eng.encode_host([np.fromfile(pcm[c], dtype=np.float32) for c in clips])
engine = {c: eo[i] for i, c in enumerate(clips)}
res = {"engine": engine}
for name, env in [("fused", {}), ("conv_f64", {"GGML_Q2A_CONV_F64": "1"}), ("no_fused_attn", {"GGML_Q2A_NO_FUSED_ATTN": "1"}),
                  ("no_conv_hilo", {"GGML_Q2A_NO_CONV_HILO": "1"})]:
    res[name] = backend(env)
for name, out in res.items():
    st = [stats(out[c][rows], ref(c)) for c in clips]
    de = [stats(out[c][rows], engine[c][rows]) for c in clips]
    print(json.dumps({"variant": name, "avg_max_rel": np.mean([s[0] for s in st]), "avg_rel_l2": np.mean([s[1] for s in st]),
                      "per_clip_rel_l2": [round(s[1], 9) for s in st], "vs_engine_rel_l2": np.mean([s[1] for s in de])}),
          flush=True)
