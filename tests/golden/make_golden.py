"""Generate the golden fixtures under tests/golden/ from the REAL reference CPU path.

Runs only in the build container (needs /root/reference compiled into oracle/_ref/ref_harness via
`make -C oracle ref`). Inputs are produced by our deterministic tooling (bin/q2a_tool: splitmix64 model
generator, synthetic clips, byte-exact quantizer) so the GPU box can regenerate identical bytes; the SHA-256
of every input is recorded so a drift in the generator is caught before any numeric comparison.

Outputs (committed):
  golden.npz   arrays (sampled where the full tensor would be large)
  golden.json  metadata: hashes, shapes, sample seeds, reference timings
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd")
TOOL = os.path.join(PKG, "bin", "q2a_tool")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

CLIPS = {0: 480000, 1: 480000, 2: 116800, 3: 656000}   # 30 s, 30 s, 7.3 s (short), 41 s (long)
FTYPE_ID = {"q4_k": 12, "q8_0": 7, "q4_0": 2}


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def run(*args, **kw):
    return subprocess.run(list(map(str, args)), check=True, capture_output=True, text=True, **kw).stdout


def sample_idx(n, k, seed):
    return np.sort(np.random.default_rng(seed).choice(n, size=min(k, n), replace=False)).astype(np.int64)


def main():
    tmp = tempfile.mkdtemp(prefix="q2a_golden_")
    arrays, meta = {}, {"clips": {}, "models": {}, "outputs": {}}
    nthreads = os.cpu_count() or 8

    for c, n in CLIPS.items():
        p = os.path.join(tmp, f"clip{c}.f32")
        run(TOOL, "synth-clip", p, n, c)
        meta["clips"][str(c)] = {"n_samples": n, "sha256": sha(p)}

    def model(cfg, wt):
        base = os.path.join(tmp, f"{cfg}-f16.bin")
        if not os.path.exists(base):
            run(TOOL, "gen-model", base, cfg, "f16", "0x51A2", nthreads)
        if wt == "f16":
            return base
        mine = os.path.join(tmp, f"{cfg}-{wt}.bin")
        run(TOOL, "quantize", base, mine, wt, nthreads)
        if cfg == "tiny":   # pin our quantizer against the reference quantize flow, byte for byte
            theirs = os.path.join(tmp, f"{cfg}-{wt}.ref.bin")
            run(REF, "quantize-model", base, theirs, FTYPE_ID[wt])
            assert sha(mine) == sha(theirs), f"quantizer mismatch for {wt}"
        return mine

    def encode(mpath, clip, tag, dumpdir=None, reps=1):
        out = os.path.join(tmp, f"{tag}.out")
        args = [REF, "encode", mpath, os.path.join(tmp, f"clip{clip}.f32"), out, nthreads, reps]
        if dumpdir:
            args += [dumpdir, 40]
        info = json.loads(run(*args).strip().splitlines()[-1])
        y = np.fromfile(out, dtype=np.float32).reshape(info["ne1"], info["ne0"])
        return y, info

    # ---- mel (reference log_mel_spectrogram) for 30 s / short / long clips
    tiny = model("tiny", "f16")
    meta["models"]["tiny-f16"] = {"sha256": sha(tiny)}
    for c in (0, 2, 3):
        out = os.path.join(tmp, f"mel{c}.bin")
        run(REF, "mel", tiny, os.path.join(tmp, f"clip{c}.f32"), out, nthreads)
        raw = np.fromfile(out, dtype=np.int32)
        n_mel, n_len = int(raw[0]), int(raw[1])
        mel = raw[2:].view(np.float32).reshape(n_mel, n_len)
        idx = sample_idx(mel.size, 16384, 100 + c)
        arrays[f"mel{c}_idx"] = idx
        arrays[f"mel{c}_val"] = mel.reshape(-1)[idx]
        arrays[f"mel{c}_rowsum"] = mel.astype(np.float64).sum(axis=1)
        meta["outputs"][f"mel{c}"] = {"n_mel": n_mel, "n_len": n_len, "max": float(mel.max()), "min": float(mel.min())}

    # ---- tiny encoder outputs: F16 full + layer-0 intermediates; quantized / short / long sampled rows
    dumpdir = os.path.join(tmp, "dump")
    os.makedirs(dumpdir)
    y, info = encode(tiny, 0, "tiny-f16-c0", dumpdir=dumpdir)
    arrays["tiny_f16_c0"] = y
    names = {3: "conv_out", 6: "ln1", 8: "v", 12: "k", 18: "q", 24: "attn", 27: "x1", 33: "gelu", 36: "x2"}
    for node, nm in names.items():
        f = glob.glob(os.path.join(dumpdir, f"node{node:03d}_*.f32"))[0]
        a = np.fromfile(f, dtype=np.float32)
        idx = sample_idx(a.size, 8192, 200 + node)
        arrays[f"tiny_f16_l0_{nm}_idx"] = idx
        arrays[f"tiny_f16_l0_{nm}_val"] = a[idx]
    rows = np.arange(0, 750, 5)
    for wt in ("q4_k", "q8_0", "q4_0"):
        mp = model("tiny", wt)
        meta["models"][f"tiny-{wt}"] = {"sha256": sha(mp)}
        y, _ = encode(mp, 0, f"tiny-{wt}-c0")
        arrays[f"tiny_{wt}_c0_rows"] = y[rows]
        meta["outputs"][f"tiny_{wt}_c0"] = {"l2": float(np.linalg.norm(y)), "maxabs": float(np.abs(y).max())}
    for c in (1, 2, 3):
        y, _ = encode(tiny, c, f"tiny-f16-c{c}")
        arrays[f"tiny_f16_c{c}_rows"] = y[rows]
        meta["outputs"][f"tiny_f16_c{c}"] = {"l2": float(np.linalg.norm(y)), "maxabs": float(np.abs(y).max())}
    arrays["rows_stride5"] = rows

    # ---- quantizer / activation-quantizer / dot known answers (8 x 1280 gaussian rows)
    rng = np.random.default_rng(7)
    x = rng.standard_normal((8, 1280)).astype(np.float32)
    xp = os.path.join(tmp, "kat_x.f32")
    x.tofile(xp)
    arrays["kat_x"] = x
    for kind in ("q4k", "q80", "act_q8k", "act_q80", "f16"):
        op = os.path.join(tmp, f"kat_{kind}.bin")
        run(REF, "qrow", kind, xp, 1280, op)
        arrays[f"kat_{kind}"] = np.fromfile(op, dtype=np.uint8)
    w = (rng.standard_normal((96, 1280)) * 0.02).astype(np.float32)
    xa = rng.standard_normal((40, 1280)).astype(np.float32)
    wp, xap = os.path.join(tmp, "kat_w.f32"), os.path.join(tmp, "kat_xa.f32")
    w.tofile(wp)
    xa.tofile(xap)
    arrays["kat_w"], arrays["kat_xa"] = w, xa
    for kind in ("f16", "q4k", "q80"):
        op = os.path.join(tmp, f"kat_gemm_{kind}.f32")
        run(REF, "gemm", kind, wp, xap, 1280, op)
        arrays[f"kat_gemm_{kind}"] = np.fromfile(op, dtype=np.float32).reshape(40, 96)

    # ---- full-size model (L=32, D=1280, H=20): sampled outputs + row norms
    if "--no-full" not in sys.argv:
        for wt in ("f16", "q4_k", "q8_0"):
            mp = model("full", wt)
            meta["models"][f"full-{wt}"] = {"sha256": sha(mp)}
            y, info = encode(mp, 0, f"full-{wt}-c0")
            idx = sample_idx(y.size, 8192, 300)
            arrays[f"full_{wt}_c0_idx"] = idx
            arrays[f"full_{wt}_c0_val"] = y.reshape(-1)[idx]
            arrays[f"full_{wt}_c0_rownorm"] = np.linalg.norm(y.astype(np.float64), axis=1)
            meta["outputs"][f"full_{wt}_c0"] = {"l2": float(np.linalg.norm(y)), "maxabs": float(np.abs(y).max()),
                                                 "ref_seconds": info["best_s"], "threads": nthreads}
            print(wt, info, flush=True)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.npz"), flush=True)


if __name__ == "__main__":
    main()
