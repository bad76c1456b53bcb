"""All-F32 model files (ftype 0): the reference's default model (examples/main/main.cpp:77, ggml-model-f32.bin) and
the only file type its unmodified sched runs end to end. Reference outputs: tests/golden/
golden_f32.{npz,json}, made by the reference CPU path itself (tests/golden/make_golden_f32.py).

The engine computes every F32 x F32 product class of ggml_vec_dot_f32 with fp16 hi/lo operand splits on the fp16
MFMA ([Ah | Al | Ah] . [Wh | Wh | Wl], only the lo x lo term dropped, ~2^-22 relative); the ggml backend runs the
F32 weight MUL_MATs on its exact-f32 MFMA GEMM."""
import os

import numpy as np
import pytest

from conftest import rel_errors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine_f32(make_model):
    import q2a
    e = q2a.Engine(make_model("tiny", "f32"), device=0)
    yield e
    e.close()


@pytest.mark.parametrize("clip", [0, 2])
def test_engine_tiny_f32_vs_reference(engine_f32, make_clip, golden_f32, clip):
    _, g = golden_f32
    out, st = engine_f32.encode_host([make_clip(clip)])
    assert st[0] == 0
    mx, l2 = rel_errors(out[0][g["rows_stride5"]], g[f"tiny_f32_c{clip}_rows"])
    assert mx < 1e-3 and l2 < 1e-4, (mx, l2)


def test_engine_f32_linear_is_f32_class(engine_f32, make_model):
    """One F32 linear: the three-term split must sit at f32 rounding level against a float64 product."""
    import torch
    from q2a import ggmlfile
    mf = ggmlfile.read(make_model("tiny", "f32"))
    w = mf.t("layers.0.fc1.weight").as_f32().astype(np.float64)   # [1024][256]
    M, K = 1537, 256
    x = np.random.default_rng(3).standard_normal((M, K)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty((M, w.shape[0]), dtype=torch.float32, device="cuda")
    engine_f32.test_linear(0, 2, xd.data_ptr(), M, yd.data_ptr())
    torch.cuda.synchronize()
    ref = x.astype(np.float64) @ w.T
    mx, l2 = rel_errors(yd.cpu().numpy(), ref)
    assert mx < 1e-5 and l2 < 2e-6, (mx, l2)


def test_engine_full_f32_vs_reference(make_model, make_clip, golden_f32):
    import q2a
    _, g = golden_f32
    e = q2a.Engine(make_model("full", "f32"), device=0)
    out, st = e.encode_host([make_clip(0)])
    e.close()
    o = out[0].reshape(-1)
    mxs, l2s = rel_errors(o[g["full_f32_c0_idx"]], g["full_f32_c0_val"])
    rn = np.linalg.norm(out[0].astype(np.float64), axis=1)
    rnerr = np.abs(rn - g["full_f32_c0_rownorm"]).max() / g["full_f32_c0_rownorm"].max()
    assert mxs < 1e-3 and l2s < 1e-3 and rnerr < 1e-4, (mxs, l2s, rnerr)


def test_ggml_backend_tiny_f32(make_model, make_clip, golden_f32, tmp_path):
    """The reference's own whisper_full on the Q2A backend with an F32 file (weights on the exact-f32 GEMM)."""
    from test_gpu_ggml_backend import HARNESS, run
    if not os.path.exists(HARNESS):
        pytest.fail("oracle/_ref/ggml_harness missing")
    _, g = golden_f32
    emb, info = run(HARNESS, make_model("tiny", "f32"), make_clip(0), tmp_path)
    assert info["mul_mat_f32"] == 6 * 2 and info["attn_fused"] == 2, info
    mx, l2 = rel_errors(emb[g["rows_stride5"]], g["tiny_f32_c0_rows"])
    assert mx < 1e-3 and l2 < 1e-4, (mx, l2)
