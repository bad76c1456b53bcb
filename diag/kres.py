"""Summarise hipcc's kernel-resource-usage remarks: one line per kernel (VGPR, AGPR, spills, LDS, occupancy).
usage: python diag/kres.py csrc/q2a_gemm.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
       "-Iqwen2-audio-whisper-ggml_amd/csrc", "-w"] + sys.argv[3:] + ["-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f"{r['name'][:90]:90s} V{r.get('VGPRs','?'):>4} A{r.get('AGPRs','?'):>4} spV{r.get('VGPRs Spill','?'):>3} "
          f"spS{r.get('SGPRs Spill','?'):>3} scr{r.get('ScratchSize [bytes/lane]','?'):>3} LDS{r.get('LDS Size [bytes/block]','?'):>7} occ{r.get('Occupancy [waves/SIMD]','?')}")
