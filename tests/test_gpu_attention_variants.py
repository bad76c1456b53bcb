"""The opt-in F32-class attention schedules against the default kernel and an fp64 reference, each in its
own process (the launcher reads Q2A_ATTN_* once per process): k_attn_g32 (32-key tiles), k_attn_p32 (QK^T of the next
tile interleaved with the softmax) and k_attn_pp32 (8-wave ping-pong over three LDS-DMA stages) share one per-element
operation sequence, so they must agree BIT FOR BIT — a missing barrier or an early read of a DMA'd stage shows up
here as a mismatch; every variant, and the register-staged k_attn, must meet the attention bar of
test_gpu_parity.py against float64."""
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

VARIANTS = {"default": {}, "k_attn": {"Q2A_ATTN_G": "0"}, "g32": {"Q2A_ATTN_G32": "1"}, "p32": {"Q2A_ATTN_P32": "1"},
            "pp32": {"Q2A_ATTN_PP32": "1"}}


@pytest.fixture(scope="module")
def outputs(make_model, tmp_path_factory):
    model = make_model("tiny", "f16")
    d = tmp_path_factory.mktemp("attn_variants")
    res = {}
    for name, env in VARIANTS.items():
        path = str(d / f"{name}.npy")
        e = {k: v for k, v in os.environ.items() if not k.startswith("Q2A_ATTN_")}
        e.update(env)
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
