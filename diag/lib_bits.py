"""Output bits of the engine library that q2a loads (Q2A_LIB_PATH selects an A/B build): SHA-256 of every clip's
embd_enc for full-size F16 / Q8_0 (4 clips) and Q4_K (4 clips, and 64 clips = the 8-phase regime), one JSON line.
Run once per library on the same box and compare the lines (diagnostic, not a test)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (model generation + synthetic clips, cached under Q2A_BENCH_DIR)
import q2a  # noqa: E402

workdir = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
os.makedirs(workdir, exist_ok=True)
res = {"lib": q2a.LIB_PATH}
for wt, n in (("f16", 4), ("q8_0", 4), ("q4_k", 4), ("q4_k", 64)):
    path = bench.make_model(wt, workdir, 16)
    pcm = bench.synth_clips(0, n)
    eng = q2a.Engine(path, device=0)
    out, st = eng.encode_host([pcm[i] for i in range(n)])
    eng.close()
    res[f"{wt}x{n}"] = [hashlib.sha256(out[i].tobytes()).hexdigest()[:16] for i in range(n)]
print(json.dumps(res))
