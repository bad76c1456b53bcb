#!/usr/bin/env python3
"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench.py run into per-kernel HBM bytes.

    python profiles/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json "source text"

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (TCC, summed over channels). gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE x2, because 16-B-per-lane streaming reads are counted at half size. Kernel classes are
mapped to the engine's launch sites by template signature (k_gemm<BM, BN, WM, WN, EPI, BLK, PIPE>).
"""
import csv
import json
import re
import sys
from collections import defaultdict

EPI = {0: "qkv", 1: "resid", 2: "gelu_h", 3: "conv2", 4: "gelu_f", 5: "store_f", 6: "gelu_q8k", 7: "pre_h"}


def classify(name: str) -> str:
    if "k_attn" in name:
        return "attention"
    m = re.search(r"k_gemm<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", name)
    if not m:
        return name.split("(")[0].strip()[:60]
    epi, blk = int(m.group(5)), int(m.group(6))
    if blk == 2:   # Q2A_BLK_EXACT: the conv GEMMs (f64-summed K-steps)
        return "conv2" if epi == 3 else "conv1" if epi == 2 else "conv (ggml backend)"
    if epi == 0:
        return "gemm_qkv"
    if epi == 1:
        return "gemm_o+gemm_fc2"
    if epi == 3:
        return "conv2"
    if epi in (2, 4, 6, 7):
        return "gemm_fc1"
    return EPI.get(epi, str(epi))


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def resid_split(path, counter):
    """O and fc2 share the residual-epilogue kernels: per layer the O launch comes first, then fc2's (its main rounds,
    plus at 64 clips the 128x128 partial-round tail right after them). Dispatch order splits them: a RESID dispatch
    that is not a 128x128 tail alternates O / fc2; a tail belongs to the fc2 launch before it. Returns the per-layer
    KiB of each (fc2 = main + tail)."""
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            m = re.search(r"k_gemm<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", row.get("Kernel_Name", ""))
            if row.get("Counter_Name") == counter and m and int(m.group(5)) == 1 and int(m.group(6)) != 2:
                tail = int(m.group(1)) == 128 and int(m.group(2)) == 128
                rows.append((int(row["Dispatch_Id"]), tail, float(row["Counter_Value"])))
    rows.sort()
    o, fc2 = [], []
    nxt_o = True
    for _, tail, v in rows:
        if tail and fc2:
            fc2[-1] += v
        elif nxt_o:
            o.append(v)
            nxt_o = False
        else:
            fc2.append(v)
            nxt_o = True
    return o, fc2


def main():
    fetch_csv, write_csv, out, source = sys.argv[1:5]
    fetch, write = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    res = {}
    # the kernel with the most dispatches of a class keeps the class name (e.g. the 8-phase O / fc2 kernel), smaller
    # parts of the same launches (fc2's 128x128 partial-round tail) get primed keys
    for k in sorted(set(fetch) | set(write), key=lambda n: (-max(len(fetch.get(n, [])), len(write.get(n, []))), n)):
        cls = classify(k)
        f = fetch.get(k, [])
        w = write.get(k, [])
        e = {"kernel": k, "dispatches": max(len(f), len(w))}
        if f:
            e["FETCH_SIZE_KiB_avg"] = sum(f) / len(f)
        if w:
            e["WRITE_SIZE_KiB_avg"] = sum(w) / len(w)
        if f and w:
            e["hbm_bytes_per_launch_corrected"] = (2 * e["FETCH_SIZE_KiB_avg"] + e["WRITE_SIZE_KiB_avg"]) * 1024
        key = cls
        while key in res:
            key += "'"
        res[key] = e
    of, ff = resid_split(fetch_csv, "FETCH_SIZE")
    ow, fw = resid_split(write_csv, "WRITE_SIZE")
    for cls, f, w in (("gemm_o", of, ow), ("gemm_fc2", ff, fw)):
        if f and w:
            e = {"class": cls, "kernel": "residual-epilogue kernels split by dispatch order (profiles/pmc_summary.py "
                 "resid_split)", "dispatches": min(len(f), len(w)), "FETCH_SIZE_KiB_avg": sum(f) / len(f),
                 "WRITE_SIZE_KiB_avg": sum(w) / len(w)}
            e["hbm_bytes_per_launch_corrected"] = (2 * e["FETCH_SIZE_KiB_avg"] + e["WRITE_SIZE_KiB_avg"]) * 1024
            res[cls] = e
    with open(out, "w") as fo:
        json.dump({"source": source,
                   "units": "FETCH_SIZE/WRITE_SIZE in KiB per dispatch; gfx950 correction: FETCH_SIZE x2 (16-B/lane "
                            "streaming reads count half, MI355X_MICROARCH.md HBM section); Infinity-Cache hits are "
                            "included in these counters",
                   "kernels": res}, fo, indent=1)


if __name__ == "__main__":
    main()
