"""CPU-side checks of the C-ABI library: it loads without a GPU and exports every symbol include/*.h declares
(no compute calls are made here)."""
import ctypes as C
import glob
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT


@pytest.fixture(scope="module")
def libq2a():
    subprocess.check_call(["make", "-C", PKG, "-j8", "all"], stdout=subprocess.DEVNULL)
    return C.CDLL(os.path.join(PKG, "lib", "libq2a.so"))


def declared_functions():
    names = []
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        names += re.findall(r"\b(q2a_\w+|whisper_\w+)\s*\(", src)
    return sorted(set(n for n in names if not n.endswith("_t")))


def test_every_declared_symbol_is_exported(libq2a):
    names = declared_functions()
    assert len(names) >= 14
    missing = [n for n in names if not hasattr(libq2a, n)]
    assert not missing, missing


def test_no_device_gives_clean_error(libq2a):
    """Without a GPU the engine must fail loudly (error code + message), never fall back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    libq2a.q2a_open.restype = C.c_void_p
    libq2a.q2a_last_error.restype = C.c_char_p
    h = libq2a.q2a_open(b"/nonexistent.bin", 0)
    assert not h
    assert libq2a.q2a_last_error()


def test_python_mirror_exports_match(libq2a):
    import q2a
    for n in q2a.EXPORTS:
        assert hasattr(libq2a, n), n
