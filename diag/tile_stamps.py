"""Where a tile's time goes inside the 8-phase GEMM (timing diagnostic on a Q2A_DIAG_STAMPS build, never the product
library): s_memtime stamps of waves 0 and 4 of every workgroup of the LAST launch of the stamped epilogue class in one
64-clip Q4_K encode (fc1 = PRE_H for a Q2A_DIAG_STAMPS=7 build, O/fc2 for =1).
usage: Q2A_LIB_PATH=diag/<stamps build>/libq2a.so python diag/tile_stamps.py [label]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
import bench  # noqa: E402
import q2a  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "stamps"
workdir = os.environ.get("Q2A_BENCH_DIR", "/tmp/q2ab")
os.makedirs(workdir, exist_ok=True)
B = 64
eng = q2a.Engine(bench.make_model("q4_k", workdir, 16), device=0)
eng.reserve(B)
pcm = torch.from_numpy(bench.synth_clips(0, B)).cuda()
out = torch.empty((B,) + eng.out_shape, dtype=torch.float32, device="cuda")
L = q2a.lib()
for _ in range(2):
    eng.encode_device(pcm.data_ptr(), bench.N_SAMPLES, [bench.N_SAMPLES] * B, out.data_ptr())
torch.cuda.synchronize()
L.q2a_diag_stamps_clear()
eng.encode_device(pcm.data_ptr(), bench.N_SAMPLES, [bench.N_SAMPLES] * B, out.data_ptr())
torch.cuda.synchronize()
n = 16384 * 2 * 16
st = np.zeros(n, dtype=np.uint64)
assert L.q2a_diag_stamps(C.c_void_p(st.ctypes.data), C.c_int64(n)) == 0
st = st.reshape(16384, 2, 16).astype(np.int64)
nwg = int(np.max(np.nonzero(st[:, 0, 0])[0])) + 1
s = st[:nwg]
res = {"label": label, "lib": os.environ.get("Q2A_LIB_PATH", "default"), "workgroups": nwg}
rt0, rt1 = s[:, 0, 8], s[:, 0, 9]
clk = (s[:, 0, 6] - s[:, 0, 0]) / np.maximum(rt1 - rt0, 1) / 10.0      # shader clocks per ns = GHz
res["clock_ghz_median"] = round(float(np.median(clk)), 3)
seg = {"prologue(1-0)": (1, 0), "mainloop(2-1)": (2, 1), "final+drain(3-2)": (3, 2), "stage(4-3)": (4, 3),
       "store_issue(5-4)": (5, 4), "store_drain(6-5)": (6, 5), "total(6-0)": (6, 0)}
for w in (0, 1):
    d = {}
    for k, (a, b) in seg.items():
        v = s[:, w, a] - s[:, w, b]
        if a == 4 and not np.any(s[:, w, 4]):
            continue
        d[k] = {"p10": int(np.percentile(v, 10)), "median": int(np.median(v)), "p90": int(np.percentile(v, 90))}
    d["block_starts(7)"] = {"median": int(np.median(s[:, w, 7]))}
    res["wave%d" % (4 * w)] = d
# dispatch structure: entry times (realtime, 10 ns ticks) relative to the first workgroup, by round of 256
t = (rt0 - rt0.min()) * 10 / 1000.0   # us
e = (rt1 - rt0.min()) * 10 / 1000.0
rounds = []
for r in range(0, nwg, 256):
    rounds.append({"round": r // 256, "start_us_min": round(float(t[r:r + 256].min()), 2),
                   "start_us_max": round(float(t[r:r + 256].max()), 2), "end_us_max": round(float(e[r:r + 256].max()), 2)})
res["rounds"] = rounds[:4] + rounds[-3:]
res["launch_us"] = round(float(e.max()), 2)
print(json.dumps(res))
