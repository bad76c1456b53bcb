"""Parity of attention-precision variants end to end.

    python diag/pv_parity.py OUT.jsonl NAME=LIB [NAME=LIB ...]

Generates the tiny and full-size F16 / Q4_K / Q8_0 model files once (same generator seeds and SHA-256 as
tests/golden), then, for each library in its own process (Q2A_LIB_PATH), encodes clip 0 and writes one JSON line per
(variant, model): max-rel / rel-L2 against the reference's golden samples and, for the full-size files, the ratio to
the WIDEST disagreement between the reference's own builds (tests/golden/crossbuild.json); plus the attention unit
error against float64 torch. A diagnostic: nothing in lib/libq2a.so or the test suite reads it."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd")
TOOL = os.path.join(PKG, "bin", "q2a_tool")
GOLD = os.path.join(ROOT, "tests", "golden")
WORK = os.environ.get("Q2A_PV_WORK", "/tmp/q2a_pv")


def models():
    os.makedirs(WORK, exist_ok=True)
    out = {}
    th = str(min(16, os.cpu_count() or 8))
    for cfg in ("tiny", "full"):
        base = os.path.join(WORK, f"{cfg}-f16.bin")
        if not os.path.exists(base):
            subprocess.check_call([TOOL, "gen-model", base, cfg, "f16", "0x51A2", th])
        out[(cfg, "f16")] = base
        for wt in ("q4_k", "q8_0"):
            p = os.path.join(WORK, f"{cfg}-{wt}.bin")
            if not os.path.exists(p):
                subprocess.check_call([TOOL, "quantize", base, p, wt, th])
            out[(cfg, wt)] = p
    clip = os.path.join(WORK, "clip0.f32")
    if not os.path.exists(clip):
        subprocess.check_call([TOOL, "synth-clip", clip, "480000", "0"])
    return out, clip


def worker(name, res_path):
    sys.path.insert(0, PKG)
    import torch
    import q2a
    ms, clip = models()
    pcm = np.fromfile(clip, dtype=np.float32)
    g = dict(np.load(os.path.join(GOLD, "golden.npz"), allow_pickle=False))
    cb = json.load(open(os.path.join(GOLD, "crossbuild.json")))
    rows = []

    def rel(o, r):
        d = o.astype(np.float64) - r.astype(np.float64)
        return float(np.abs(d).max() / np.abs(r).max()), float(np.linalg.norm(d) / np.linalg.norm(r))

    for (cfg, wt), path in sorted(ms.items()):
        e = q2a.Engine(path, device=0)
        out, st = e.encode_host([pcm])
        e.close()
        o = out[0]
        if cfg == "tiny":
            ref = g["tiny_f16_c0"] if wt == "f16" else None
            if ref is None:
                mx, l2 = rel(o[g["rows_stride5"]], g[f"tiny_{wt}_c0_rows"])
            else:
                mx, l2 = rel(o, ref)
            rows.append({"variant": name, "model": f"tiny-{wt}", "max_rel": mx, "rel_l2": l2})
        else:
            mx, l2 = rel(o.reshape(-1)[g[f"full_{wt}_c0_idx"]], g[f"full_{wt}_c0_val"])
            pairs = cb[wt]["pairs"].values()
            wl2 = max(p["sampled_rel_l2"] for p in pairs)
            wmx = max(p["sampled_max_rel"] for p in pairs)
            rows.append({"variant": name, "model": f"full-{wt}", "max_rel": mx, "rel_l2": l2,
                         "rel_l2_over_widest_pair": l2 / wl2, "max_rel_over_widest_pair": mx / wmx})
    # attention unit error (tests/test_gpu_parity.py::test_attention_matches_fp32_reference inputs)
    e = q2a.Engine(ms[("tiny", "f16")], device=0)
    T, D, H, B = 1500, 256, 4, 2
    gen = torch.Generator(device="cpu").manual_seed(0)
    q = (torch.randn(B * T, D, generator=gen) * 0.5).cuda()
    k = (torch.randn(B * T, D, generator=gen) * 1.5).cuda()
    v = torch.randn(B * T, D, generator=gen).cuda()
    y = torch.empty_like(q)
    e.test_attention(q.data_ptr(), k.data_ptr(), v.data_ptr(), B, y.data_ptr())
    torch.cuda.synchronize()
    e.close()
    qh, kh, vh = (t.view(B, T, H, 64).permute(0, 2, 1, 3).double() for t in (q, k, v))
    ref = (torch.softmax(qh @ kh.transpose(-1, -2), dim=-1) @ vh).permute(0, 2, 1, 3).reshape(B * T, D)
    mx, l2 = rel(y.cpu().numpy(), ref.cpu().numpy())
    rows.append({"variant": name, "model": "attention-unit", "max_rel": mx, "rel_l2": l2})
    with open(res_path, "a") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


def main():
    if sys.argv[1] == "--worker":
        worker(sys.argv[2], sys.argv[3])
        return
    res = sys.argv[1]
    models()
    for spec in sys.argv[2:]:
        name, lib = spec.split("=", 1)
        env = dict(os.environ)
        env["Q2A_LIB_PATH"] = os.path.abspath(lib)
        print(f"[pv_parity] {name}: {lib}", flush=True)
        subprocess.run([sys.executable, "-u", __file__, "--worker", name, res], env=env, check=True, timeout=600)
        with open(res) as f:
            for line in f:
                r = json.loads(line)
                if r["variant"] == name:
                    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
