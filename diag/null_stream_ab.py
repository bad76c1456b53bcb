"""configs[1] (one clip, F16): the same encode issued with a NULL stream (the engine's stream ordered against the
legacy default stream by an event each way, include/q2a_encoder.h) and with an explicit stream (the caller's torch
stream, no cross-stream events), alternating; wall time per encode over back-to-back calls (round 6)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import q2a  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "f16x1"
wt, clips, _ = bench.CONFIGS[cfg]
wd = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
os.makedirs(wd, exist_ok=True)
path = bench.make_model(wt, wd, 16)
eng = q2a.Engine(path, device=0)
pcm = torch.from_numpy(bench.synth_clips(0, clips)).cuda()
out = torch.empty((clips,) + eng.out_shape, dtype=torch.float32, device="cuda")
ns = [bench.N_SAMPLES] * clips
side = torch.cuda.Stream()   # (the default torch stream IS the legacy stream 0: a side stream is an explicit one)
torch.cuda.synchronize()
cs = side.cuda_stream
res = {}
for rep in range(3):
    for mode in ("null", "explicit"):
        st = cs if mode == "explicit" else None
        for _ in range(3):
            eng.encode_device(pcm.data_ptr(), bench.N_SAMPLES, ns, out.data_ptr(), stream=st)
        torch.cuda.synchronize()
        n = 40
        t = time.perf_counter()
        for _ in range(n):
            eng.encode_device(pcm.data_ptr(), bench.N_SAMPLES, ns, out.data_ptr(), stream=st)
        torch.cuda.synchronize()
        res.setdefault(mode, []).append(round((time.perf_counter() - t) / n * 1e3, 4))
print(json.dumps({"config": cfg, "ms_per_encode": res}))
