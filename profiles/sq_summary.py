#!/usr/bin/env python3
"""Summarise the SQ counter passes of profiles/collect_sq.sh into per-kernel-class MFMA utilisation evidence.

    python profiles/sq_summary.py SQ2_counter_collection.csv SQ_counter_collection.csv OUT.json "source text"

Per kernel class (pmc_summary.classify), averaged per dispatch:
  mfma_busy_frac   SQ_VALU_MFMA_BUSY_CYCLES (per-SIMD busy cycles, summed over the 1024 SIMDs) /
                   (GRBM_GUI_ACTIVE / 8 XCDs (rocprofv3 sums the XCDs) x 1024 SIMDs)   — rocprof's MfmaUtil
  mfma_flop        SQ_INSTS_VALU_MFMA_MOPS_F16 x 512 (fp16 MFMA flop actually issued, incl. the 3-term attention split)
  wait/active      SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_* as fractions of SQ_WAVE_CYCLES
  lds_bank_conflict_per_wave_cycle
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import classify  # noqa: E402

N_SIMD = 1024
N_XCD = 8


def load(path):
    per = defaultdict(lambda: defaultdict(list))
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            names[k] = classify(k)
    return per, names


def main():
    sq2, sq1, out, source = sys.argv[1:5]
    res = {"source": source, "kernels": {}}
    for path in (sq2, sq1):
        if not os.path.exists(path):
            continue
        per, names = load(path)
        for k, cnt in per.items():
            e = res["kernels"].setdefault(names[k] + " | " + k[:120], {"class": names[k]})
            for c, v in cnt.items():
                e[c] = sum(v) / len(v)
                e["dispatches"] = len(v)
    for e in res["kernels"].values():
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and "GRBM_GUI_ACTIVE" in e:
            e["mfma_busy_frac"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / N_XCD * N_SIMD)
        if "SQ_INSTS_VALU_MFMA_MOPS_F16" in e:
            e["mfma_flop_f16"] = e["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512
        if e.get("SQ_WAVE_CYCLES"):
            w = e["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA"):
                if c in e:
                    e[c.lower().replace("sq_", "") + "_frac"] = e[c] / w
            if "SQ_LDS_BANK_CONFLICT" in e:
                e["lds_bank_conflict_per_wave_cycle"] = e["SQ_LDS_BANK_CONFLICT"] / w
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, e in sorted(res["kernels"].items()):
        print(f"{k[:100]:100s} mfma_busy={e.get('mfma_busy_frac', float('nan')):.3f} "
              f"wait_any={e.get('wait_any_frac', float('nan')):.3f} valu={e.get('active_inst_valu_frac', float('nan')):.3f}")


if __name__ == "__main__":
    main()
