"""CPU-only ISA check of the built gfx950 code objects: the bandwidth and front-end kernels must not wait for each of
their loads one at a time. A load placed by the compiler under a per-chunk branch (`if (c < nch) { v = x[c]; s += v; }`)
or inside a range branch (a GELU-table read under `x > -10`) compiles to `global_load` + `s_waitcnt vmcnt(0)` per
element: serial HBM / L2 round trips. Round 6 found and removed five such cases; this keeps them out.
Disassembles build/*.o (the .hip_fatbin bundle) with the ROCm LLVM tools; skipped when either is absent."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"


def _disasm(obj: str, tmp_path) -> str:
    for tool in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not found")
    path = os.path.join(BUILD, obj)
    if not os.path.exists(path):
        pytest.skip(f"{obj} not built")
    fat, co = str(tmp_path / (obj + ".fatbin")), str(tmp_path / (obj + ".co"))
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", path,
                    str(tmp_path / "unused.o")], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                   check=True, capture_output=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def _serial_loads(text: str) -> dict:
    """kernel symbol -> (global loads, loads whose next instruction is s_waitcnt vmcnt(0))"""
    out, cur, prev_load = {}, None, False
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur, prev_load = m.group(1), False
            out[cur] = [0, 0]
            continue
        ins = line.strip().split()
        if cur is None or not ins:
            continue
        op = ins[0]
        if prev_load and op == "s_waitcnt" and "vmcnt(0)" in line:
            out[cur][1] += 1
        prev_load = op.startswith("global_load")
        if prev_load:
            out[cur][0] += 1
    return out


def _pick(stats: dict, pattern: str) -> list:
    ks = [k for k in stats if re.search(pattern, k)]
    assert ks, pattern
    return ks


@pytest.mark.parametrize("obj,pattern,limit", [
    ("q2a_exact.o", r"k_rownorm5ILi1ELb1E", 0),      # LayerNorm + Q8_K, D = 1280
    ("q2a_exact.o", r"k_rownorm5ILi0ELb1E", 0),      # LayerNorm + fp16
    ("q2a_exact.o", r"k_rownormILi0ELb1ELb0E", 0),   # LayerNorm + fp16, any D
    ("q2a_exact.o", r"k_pool_ln", 1),                # AvgPool + final LayerNorm (one scalar load of the clip flag)
    ("q2a_exact.o", r"k_mel_frames", 3),             # log-mel frames (the clip's scalars)
    ("q2a_gemm.o", r"k_gemmILi64ELi128ELi2ELi2ELi3ELi2ELi0E", 2),   # conv2 (GELU + positions epilogue)
    ("q2a_gemm.o", r"k_gemmILi64ELi128ELi2ELi2ELi2ELi2ELi0E", 2),   # conv1 (GELU epilogue)
    ("q2a_gemm.o", r"k_gemmILi128ELi128ELi2ELi2ELi2ELi0ELi0E", 2),  # one-clip F16 fc1 (GELU epilogue)
])
def test_no_serialised_loads(tmp_path, obj, pattern, limit):
    stats = _serial_loads(_disasm(obj, tmp_path))
    for k in _pick(stats, pattern):
        loads, serial = stats[k]
        assert loads > 0, k
        assert serial <= limit, (k, loads, serial)
