"""Print per-kernel ms/step of the A/B timing runs (diag/ab.sh) side by side."""
import glob
import json
import sys

cfg = sys.argv[1] if len(sys.argv) > 1 else "q4k64"
rows = {}
for f in sorted(glob.glob(f"gpurun_out/ab_*_{cfg}.json")):
    v = f.split("ab_")[1][: -len(cfg) - 6]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows[v] = (d["ms_per_step"], {k: x["ms_per_step"] for k, x in d["per_kernel"].items()})
keys = list(next(iter(rows.values()))[1])
print(f"{'variant':12s} {'step':>8s} " + " ".join(f"{k[:10]:>10s}" for k in keys))
for v, (st, pk) in rows.items():
    print(f"{v:12s} {st:8.2f} " + " ".join(f"{pk[k]:10.2f}" for k in keys))
