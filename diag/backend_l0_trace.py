"""Layer-0 node-by-node distance of the ggml-backend drop-in path (tiny F16 model, clip 0) to the reference's CPU
builds, next to the distance between two CPU builds at the same node (diagnostic for VERDICT r03 weak 1).

  python diag/backend_l0_trace.py ref REF.npz   (build container: oracle/_ref, _ref_x86-64, _ref_fma dumps of the
                                                 first 40 encoder nodes, every 5th row kept)
  python diag/backend_l0_trace.py gpu REF.npz   (GPU box: oracle/_ref/ggml_harness with the same dumps, the
                                                 attention chain 9-23 left unobserved so it runs fused)

A node whose backend distance jumps well past the CPU pairs' while its inputs were still inside them is where the
backend's rounding departs from the reference's."""
import glob
import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "bin", "q2a_tool")
BUILDS = {"avx2": "_ref", "x86-64": "_ref_x86-64", "fma": "_ref_fma"}
SKIP = (9, 23)
W = "/tmp/q2a_bl0"


def inputs():
    os.makedirs(W, exist_ok=True)
    model, clip = os.path.join(W, "tiny-f16.bin"), os.path.join(W, "clip0.f32")
    if not os.path.exists(model):
        subprocess.check_call([TOOL, "gen-model", model, "tiny", "f16", "0x51A2", "16"])
    if not os.path.exists(clip):
        subprocess.check_call([TOOL, "synth-clip", clip, "480000", "0"])
    return model, clip


def load(dump):
    out = {}
    for line in open(os.path.join(dump, "index.txt")):
        idx, op, ne0, ne1, ne2, ne3, name = line.split()
        idx = int(idx)
        if SKIP[0] <= idx <= SKIP[1]:
            continue
        a = np.fromfile(os.path.join(dump, name), dtype=np.float32).reshape(int(ne2) * int(ne1), int(ne0))
        out[f"n{idx:03d}_{op}"] = a[::5] if a.shape[0] == 1500 else a
    return out


def stats(a, b):
    d = a.astype(np.float64) - b.astype(np.float64)
    return {"rel_l2": float(np.linalg.norm(d) / np.linalg.norm(b)), "max_rel": float(np.abs(d).max() / np.abs(b).max()),
            "fp16_flips": int((a.astype(np.float16) != b.astype(np.float16)).sum())}


def ref(out):
    model, clip = inputs()
    arrs = {}
    for b, d in BUILDS.items():
        dump = os.path.join(W, f"dump-{b}")
        shutil.rmtree(dump, ignore_errors=True)
        os.makedirs(dump)
        subprocess.run([os.path.join(ROOT, "oracle", d, "ref_harness"), "encode", model, clip, os.path.join(dump, "y.f32"),
                        "8", "1", dump, "40"], check=True, capture_output=True)
        arrs[b] = load(dump)
    save = {k: v for k, v in arrs["avx2"].items()}
    for b in ("x86-64", "fma"):
        for k, v in arrs[b].items():
            save[f"{b}:{k}"] = v
    np.savez_compressed(out, **save)


def engine(model, clip, r):
    """The engine's layer-0 values at the same nodes (test_frontend = block input n003; the fp16 GEMM operands LN1
    n006, attention n024, LN2 n030, GELU n033; the block output n036), against the same AVX2 dumps."""
    sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
    import torch
    import q2a
    e = q2a.Engine(model, device=0)
    T, D = e.info.n_audio_ctx, e.info.n_audio_state
    pcm = torch.from_numpy(np.fromfile(clip, dtype=np.float32)).cuda()
    x = torch.empty((T, D), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    e.test_frontend(pcm.data_ptr(), pcm.numel(), [pcm.numel()], x.data_ptr())
    torch.cuda.synchronize()
    x0 = x.cpu().numpy().copy()
    taps = [torch.zeros((T, D), dtype=torch.float16, device="cuda") for _ in range(3)] + \
           [torch.zeros((T, 4 * D), dtype=torch.float16, device="cuda")]
    e.test_block_taps(0, x.data_ptr(), 1, [t.data_ptr() for t in taps])
    torch.cuda.synchronize()
    vals = {"n003_ADD": x0, "n036_ADD": x.cpu().numpy()}
    for k, t in zip(("n006_ADD", "n024_CONT", "n030_ADD", "n033_GELU"), taps):
        vals[k] = t.cpu().numpy().astype(np.float32)
    e.close()
    for k, v in vals.items():
        v = v[::5]
        st = stats(v, r[k])
        if k not in ("n003_ADD", "n036_ADD"):
            st = {"fp16_flips": st["fp16_flips"]}   # fp16 operands: only code flips are comparable
        print(json.dumps({"node": k, "engine": st}))


def gpu(refnpz):
    r = dict(np.load(refnpz))
    model, clip = inputs()
    h = os.path.join(ROOT, "oracle", "_ref", "ggml_harness")
    for label, env in (("backend", {}), ("backend_conv_f32", {"GGML_Q2A_NO_CONV_HILO": "1"})):
        dump = os.path.join(W, "dump-" + label)
        shutil.rmtree(dump, ignore_errors=True)
        os.makedirs(dump)
        p = subprocess.run([h, "encode", model, clip, os.path.join(dump, "y.f32"), "1", "0", dump, "40",
                            f"{SKIP[0]}-{SKIP[1]}"], capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
        assert p.returncode == 0, p.stderr[-2000:]
        print(p.stdout.strip().splitlines()[-1])
        be = load(dump)
        for k in sorted(be):
            if k not in r:
                continue
            row = {"node": k, label: stats(be[k], r[k])}
            for b in ("x86-64", "fma"):
                if f"{b}:{k}" in r:
                    row[b] = stats(r[f"{b}:{k}"], r[k])
            print(json.dumps(row))
    engine(model, clip, r)


if __name__ == "__main__":
    (ref if sys.argv[1] == "ref" else gpu)(sys.argv[2])
