"""Per-layer divergence trace: the engine (libq2a.so on the GPU) against the reference CPU path, layer by layer.

For the full-size synthetic model (seed 0x51A2) and clip 0 it runs the reference (oracle/_ref/ref_harness, the
/root/reference sources compiled here; dumps of every layer's block input and the four tensors ggml re-quantizes
before a weight GEMM) and then, for every layer l:

  identical input  X_l taken from the REFERENCE's own dump, one engine block (q2a_test_block_taps), compared with
                   the reference's X_{l+1}; the engine's four GEMM A operands (Q8_K codes for Q4_K) compared code
                   by code with ggml's quantization of the reference's own intermediates -> code flips per point
  chained          the engine's own trajectory from the reference's layer-0 input (block after block), compared
                   with the reference's X_{l+1}: how the per-layer differences grow

The same statistics between two builds of the reference itself (scalar vs AVX2 vs AVX-512) are in
tests/golden/crossbuild.json (tests/golden/make_crossbuild.py): that is the yardstick for the numbers here.
The oracle is test infrastructure: this script only CHECKS the engine with it.

usage (GPU box): python diag/layer_trace.py --wt q4_k --out gpurun_out/layer_trace_q4_k.json
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_crossbuild import CODES, POINTS, relerr  # noqa: E402  (numpy restatements of ggml's conversions)

T, D, F, L = 1500, 1280, 5120, 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wt", default="q4_k")
    ap.add_argument("--out", required=True)
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "q2a_trace"))
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    args = ap.parse_args()
    import torch
    import q2a

    os.makedirs(args.workdir, exist_ok=True)
    t0 = time.time()
    base = os.path.join(args.workdir, "full-f16.bin")
    if not os.path.exists(base):
        subprocess.check_call([q2a.TOOL_PATH, "gen-model", base, "full", "f16", "0x51A2", str(args.threads)])
    model = base if args.wt == "f16" else os.path.join(args.workdir, f"full-{args.wt}.bin")
    if not os.path.exists(model):
        subprocess.check_call([q2a.TOOL_PATH, "quantize", base, model, args.wt, str(args.threads)])
    clip = os.path.join(args.workdir, "clip0.f32")
    subprocess.check_call([q2a.TOOL_PATH, "synth-clip", clip, "480000", "0"])
    dump = os.path.join(args.workdir, f"dump-{args.wt}")
    shutil.rmtree(dump, ignore_errors=True)
    os.makedirs(dump)
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    subprocess.run([ref, "encode", model, clip, os.path.join(args.workdir, "ref.out"), str(args.threads), "1", dump, "-1"],
                   check=True, capture_output=True)
    print(f"reference dumps ready ({time.time() - t0:.0f} s)", flush=True)

    def node(idx):
        f = glob.glob(os.path.join(dump, f"node{idx:03d}_*.f32"))
        assert len(f) == 1, idx
        return np.fromfile(f[0], dtype=np.float32)

    eng = q2a.Engine(model, device=0)
    eng.reserve(1)
    codes = CODES[args.wt]
    dev = torch.device("cuda", 0)
    x = torch.empty(T * D, dtype=torch.float32, device=dev)
    taps = [torch.empty(T * (F if i == 3 else D), dtype=torch.float16, device=dev) for i in range(4)]
    ident, chained = [], []
    for l in range(L):
        b0 = 3 + 33 * l
        x.copy_(torch.from_numpy(node(b0)))
        eng.test_block_taps(l, x.data_ptr(), 1, [t.data_ptr() for t in taps])
        torch.cuda.synchronize()
        out = x.cpu().numpy()
        r = {"layer": l}
        r["out_max_rel"], r["out_rel_l2"] = relerr(out, node(b0 + 33))
        for i, (nm, off) in enumerate(POINTS.items()):
            mine = taps[i].cpu().numpy()
            if args.wt == "f16":
                mine = mine.view(np.int16)
            else:
                mine = mine.astype(np.float32).astype(np.int16)
            r[f"flips_{nm}"] = int((mine != codes(node(b0 + off)).reshape(-1)).sum())
        ident.append(r)
        print("identical-input", r, flush=True)
    x.copy_(torch.from_numpy(node(3)))
    for l in range(L):
        eng.test_block(l, x.data_ptr(), 1)
        torch.cuda.synchronize()
        mx, l2 = relerr(x.cpu().numpy(), node(3 + 33 * l + 33))
        chained.append({"layer": l, "out_max_rel": mx, "out_rel_l2": l2})
        print("chained", chained[-1], flush=True)
    eng.close()
    res = {"about": "engine (libq2a.so, MI355X) vs the reference CPU path (oracle/_ref, AVX2 build), full-size "
                    f"{args.wt} model, clip 0; diag/layer_trace.py",
           "wt": args.wt, "identical_input": ident, "chained": chained}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    shutil.rmtree(dump, ignore_errors=True)
    print("wrote", args.out, flush=True)


if __name__ == "__main__":
    main()
