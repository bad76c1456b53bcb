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


def test_ggml_backend_plugin_exports(libq2a):
    """lib/libggml-q2a.so (the ggml backend, include/ggml-q2a.h) defines every entry point its header declares and
    leaves ggml's own functions to the application's ggml (undefined here, resolved at load time)."""
    so = os.path.join(PKG, "lib", "libggml-q2a.so")
    if not os.path.exists(so):
        pytest.skip("built only where ggml's headers are present (GGML_DIR)")
    src = open(os.path.join(ROOT, "include", "ggml-q2a.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = sorted(set(re.findall(r"\b(ggml_backend_q2a_\w+|ggml_backend_is_q2a)\s*\(", src)))
    assert len(names) >= 7
    defined = subprocess.check_output(["nm", "-D", "--defined-only", so], text=True).split()
    assert not [n for n in names if n not in defined]
    undefined = subprocess.check_output(["nm", "-D", "--undefined-only", so], text=True)
    assert "ggml_backend_buffer_init" in undefined and "ggml_nbytes" in undefined
