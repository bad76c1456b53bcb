"""Per-kernel VGPR / spill summary of a hipcc -Rpass-analysis=kernel-resource-usage report (stderr saved to a file):
python diag/regs.py REPORT [substring]"""
import re
import sys

cur = None
rows = {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
for k, v in rows.items():
    if len(sys.argv) < 3 or sys.argv[2] in k:
        print(k.replace("_ZN12_GLOBAL__N_1", "")[:70], v)
