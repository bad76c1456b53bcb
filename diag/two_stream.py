"""Diagnostic: does splitting one GPU's batch over two engines (shared weights, one HIP stream each) overlap the
bandwidth-bound kernels of one half with the MFMA-bound kernels of the other?

    python3 diag/two_stream.py [--config q4k64] [--steps 5] [--splits 1 2 3 4]

Prints ms per 64-clip step for each split count and checks every split's output equals the single-engine encode
bit for bit (the engine is batch-invariant)."""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="q4k64")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import q2a
    wt, clips, _ = bench.CONFIGS[args.config]
    workdir = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
    os.makedirs(workdir, exist_ok=True)
    path = bench.make_model(wt, workdir, 16)
    base = q2a.Engine(path, 0)
    L = q2a.lib()
    L.q2a_open_shared.restype = C.c_void_p
    L.q2a_open_shared.argtypes = [C.c_void_p]
    engines = [base]
    for _ in range(max(args.splits) - 1):
        h = L.q2a_open_shared(C.c_void_p(base.h))
        assert h, L.q2a_last_error().decode()
        e = q2a.Engine.__new__(q2a.Engine)
        e.h = h
        e.info = q2a.Info()
        q2a._check(L.q2a_get_info(C.c_void_p(h), C.byref(e.info)))
        engines.append(e)
    pcm = torch.from_numpy(bench.synth_clips(0, clips)).cuda()
    outs = {}
    N = bench.N_SAMPLES
    for s in args.splits:
        per = [clips // s + (1 if i < clips % s else 0) for i in range(s)]
        starts = [sum(per[:i]) for i in range(s)]
        for i in range(s):
            engines[i].reserve(per[i])
        out = torch.empty((clips,) + base.out_shape, dtype=torch.float32, device="cuda")

        def step():
            for i in range(s):
                engines[i].encode_device(pcm[starts[i]].data_ptr(), N, [N] * per[i], out[starts[i]].data_ptr())

        step()
        torch.cuda.synchronize()
        outs[s] = out.clone()
        for r in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            print(f"splits={s} rep={r} ms/step={ms:.2f} frames/s={clips * 3000 / ms * 1e3:.0f}", flush=True)
        same = torch.equal(outs[s], outs[args.splits[0]])
        print(f"splits={s} bit-identical to splits={args.splits[0]}: {same}", flush=True)
    for e in engines[1:]:
        e.close()
    base.close()


if __name__ == "__main__":
    main()
