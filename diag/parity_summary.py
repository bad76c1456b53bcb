"""Clip-averaged parity statistics of a Q2A_PARITY_LOG file next to the bars the tests hold them to.

    python diag/parity_summary.py LOG.jsonl [LOG2.jsonl ...]

For each test id: the mean max-rel / rel-L2 over its logged comparisons (the tests log one line per compared clip)
and, where the test is a clip-averaged cross-build comparison, the bar (tests/conftest.py: tiny_avg_bar /
xbuild_avg_bar, x1.0) and the ratio."""
import json
import os
import re
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CB = json.load(open(os.path.join(ROOT, "tests", "golden", "crossbuild.json")))


def avg_bar(prefix0, prefix, keys):
    clips = sorted(int(k[len(prefix):]) for k in CB if k.startswith(prefix))
    entries = [CB[prefix0]] + [CB[f"{prefix}{c}"] for c in clips]
    common = set(entries[0]["pairs"])
    for e in entries[1:]:
        common &= set(e["pairs"])
    return {o: max(float(np.mean([e["pairs"][pn][k] for e in entries])) for pn in common) for o, k in keys.items()}


def bar_for(test):
    m = re.search(r"\[(f16|q4_k|q8_0|q4_0)\]", test)
    if not m:
        return None
    wt = m.group(1)
    if "tiny" in test:
        return avg_bar(f"tiny_{wt}", f"tiny_{wt}_clip", {"max_rel": "rows_max_rel", "rel_l2": "rows_rel_l2"})
    if "full" in test and wt in CB:
        return avg_bar(wt, f"{wt}_clip", {"max_rel": "sampled_max_rel", "rel_l2": "sampled_rel_l2"})
    return None


for path in sys.argv[1:]:
    per = defaultdict(list)
    for line in open(path):
        d = json.loads(line)
        per[d["test"]].append((d["max_rel"], d["rel_l2"]))
    print(f"== {path}")
    for t, v in per.items():
        mx, l2 = float(np.mean([x[0] for x in v])), float(np.mean([x[1] for x in v]))
        b = bar_for(t) if len(v) >= 3 else None
        s = f"  {t.split('::')[-1][:70]:70s} n={len(v)} max_rel {mx:.4g} rel_l2 {l2:.4g}"
        if b:
            s += f"   bar {b['max_rel']:.4g} / {b['rel_l2']:.4g}  ratio {mx / b['max_rel']:.3f} / {l2 / b['rel_l2']:.3f}"
        print(s)
