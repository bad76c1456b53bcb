"""Diagnostic: encode N synthetic 30 s clips (bench.py's generator) with the full-size model of WEIGHTS through whichever
libq2a.so Q2A_LIB_PATH names, batched, and save embd_enc — for bit-equality checks between two library builds.
    python3 diag/encode_dump.py WEIGHTS N OUT.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
import bench  # noqa: E402


def main():
    import q2a
    wt, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    wd = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
    os.makedirs(wd, exist_ok=True)
    e = q2a.Engine(bench.make_model(wt, wd, 16), 0)
    res, st = e.encode_host(list(bench.synth_clips(0, n)))
    assert list(st) == [0] * n
    np.save(out, res)
    e.close()


if __name__ == "__main__":
    main()
