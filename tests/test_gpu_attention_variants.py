"""The F32-class attention schedules measured and not adopted against an fp64 reference. They live in
diag/attn_variants.hip and are built only into diagnostic libraries (`make -C diag test-variants`, on demand; the
product build does not make them and the GPU box does not receive them, .gpurunignore), each loaded in its own process
through Q2A_LIB_PATH — the shipped lib/libq2a.so carries none of them and reads no
kernel-selecting environment variable. k_attn_g32 (32-key tiles), k_attn_p32 (QK^T of the next tile interleaved with
the softmax) and k_attn_pp32 (8-wave ping-pong over three LDS-DMA stages) share one per-element operation sequence, so
they must agree BIT FOR BIT — a missing barrier or an early read of a DMA'd stage shows up here as a mismatch; every
variant, the register-staged k_attn and the shipped kernel must meet the attention bar against float64."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from attn_variant_worker import B, D, T, inputs  # noqa: E402
from conftest import rel_errors  # noqa: E402

ROOT = os.path.dirname(HERE)
VARIANTS = {"default": None, "k_attn": "diag/attnv_k_attn/libq2a.so", "g32": "diag/attnv_g32/libq2a.so",
            "p32": "diag/attnv_p32/libq2a.so", "pp32": "diag/attnv_pp32/libq2a.so"}


BUILT = {n: lib for n, lib in VARIANTS.items() if lib is None or os.path.exists(os.path.join(ROOT, lib))}


@pytest.fixture(scope="module")
def outputs(make_model, tmp_path_factory):
    if len(BUILT) < len(VARIANTS):
        pytest.skip("diagnostic attention libraries not built (make -C diag test-variants)")
    model = make_model("tiny", "f16")
    d = tmp_path_factory.mktemp("attn_variants")
    res = {}
    for name, lib in VARIANTS.items():
        path = str(d / f"{name}.npy")
        e = {k: v for k, v in os.environ.items() if k != "Q2A_LIB_PATH"}
        if lib:
            e["Q2A_LIB_PATH"] = os.path.join(ROOT, lib)
        subprocess.run([sys.executable, os.path.join(HERE, "attn_variant_worker.py"), model, path], env=e, check=True,
                       timeout=240)
        res[name] = np.load(path)
    return res


def test_32_key_variants_bit_identical(outputs):
    assert np.array_equal(outputs["p32"], outputs["g32"])
    assert np.array_equal(outputs["pp32"], outputs["g32"])


@pytest.mark.parametrize("name", list(VARIANTS))
def test_variant_matches_fp64(outputs, name):
    import torch
    q, k, v = (torch.from_numpy(a).double() for a in inputs())
    H = D // 64
    qh = q.view(B, T, H, 64).permute(0, 2, 1, 3)
    kh = k.view(B, T, H, 64).permute(0, 2, 1, 3)
    vh = v.view(B, T, H, 64).permute(0, 2, 1, 3)
    ref = (torch.softmax(qh @ kh.transpose(-1, -2), dim=-1) @ vh).permute(0, 2, 1, 3).reshape(B * T, D).numpy()
    mx, l2 = rel_errors(outputs[name], ref)
    assert mx < 2e-3 and l2 < 5e-4, (name, mx, l2)
