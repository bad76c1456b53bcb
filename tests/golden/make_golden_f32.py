"""Golden fixtures for ALL-F32 model files (ftype 0: the reference's default `ggml-model-f32.bin`,
examples/main/main.cpp:77, and the only file type its unmodified CPU/CUDA sched runs end to end),
generated from the REAL reference CPU path (oracle/_ref/ref_harness; F32 files need no conv shim).

Runs only in the build container. Inputs come from our deterministic tooling (bin/q2a_tool gen-model ... f32), so
the GPU box regenerates identical bytes; their SHA-256 is recorded.

Outputs (committed): golden_f32.npz, golden_f32.json
  tiny_f32_c0_rows   embd_enc rows 0, 5, 10, ... of the tiny (L=2, D=256) model on clip 0
  tiny_f32_c2_rows   same on the 7.3 s clip 2
  full_f32_c0_{idx,val,rownorm}  8192 sampled outputs + the 750 row L2 norms of the full-size model on clip 0
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
TOOL = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "bin", "q2a_tool")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
CLIPS = {0: 480000, 2: 116800}


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def run(*args):
    return subprocess.run(list(map(str, args)), check=True, capture_output=True, text=True).stdout


def main():
    tmp = tempfile.mkdtemp(prefix="q2a_golden_f32_")
    nthreads = os.cpu_count() or 8
    arrays, meta = {}, {"models": {}, "outputs": {}}
    for c, n in CLIPS.items():
        run(TOOL, "synth-clip", os.path.join(tmp, f"clip{c}.f32"), n, c)

    def encode(mpath, clip, tag):
        out = os.path.join(tmp, f"{tag}.out")
        info = json.loads(run(REF, "encode", mpath, os.path.join(tmp, f"clip{clip}.f32"), out, nthreads, 1).strip().splitlines()[-1])
        return np.fromfile(out, dtype=np.float32).reshape(info["ne1"], info["ne0"]), info

    rows = np.arange(0, 750, 5)
    tiny = os.path.join(tmp, "tiny-f32.bin")
    run(TOOL, "gen-model", tiny, "tiny", "f32", "0x51A2", nthreads)
    meta["models"]["tiny-f32"] = {"sha256": sha(tiny)}
    for c in CLIPS:
        y, _ = encode(tiny, c, f"tiny-f32-c{c}")
        arrays[f"tiny_f32_c{c}_rows"] = y[rows]
        meta["outputs"][f"tiny_f32_c{c}"] = {"l2": float(np.linalg.norm(y)), "maxabs": float(np.abs(y).max())}
    if "--no-full" not in sys.argv:
        full = os.path.join(tmp, "full-f32.bin")
        run(TOOL, "gen-model", full, "full", "f32", "0x51A2", nthreads)
        meta["models"]["full-f32"] = {"sha256": sha(full)}
        y, info = encode(full, 0, "full-f32-c0")
        idx = np.sort(np.random.default_rng(300).choice(y.size, size=8192, replace=False)).astype(np.int64)
        arrays["full_f32_c0_idx"] = idx
        arrays["full_f32_c0_val"] = y.reshape(-1)[idx]
        arrays["full_f32_c0_rownorm"] = np.linalg.norm(y.astype(np.float64), axis=1)
        meta["outputs"]["full_f32_c0"] = {"l2": float(np.linalg.norm(y)), "maxabs": float(np.abs(y).max()),
                                          "ref_seconds": info["best_s"], "threads": nthreads}
    arrays["rows_stride5"] = rows
    np.savez_compressed(os.path.join(HERE, "golden_f32.npz"), **arrays)
    with open(os.path.join(HERE, "golden_f32.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta["outputs"]))


if __name__ == "__main__":
    main()
