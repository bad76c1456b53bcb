"""Per-kernel averages of every counter in one or more rocprofv3 counter_collection.csv files (diagnostic).
usage: python diag/pmc_kernels.py CSV [CSV ...]"""
import csv
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for path in sys.argv[1:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:60]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in vals.items():
    print(f"{k}  (dispatches {len(next(iter(cs.values())))}, ~{sum(dur[k]) / len(dur[k]):.1f} us under counters)")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}")
