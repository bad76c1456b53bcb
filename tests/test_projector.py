"""The downstream consumer: the Qwen2-Audio multi-modal projector, audio_features =
Linear(d_model -> text hidden, bias)(embd_enc) (transformers modeling_qwen2_audio.py Qwen2AudioMultiModalProjector).
The reference path ends at embd_enc (qwen2-whisper.cpp:2185) and has no projector, so parity here is UNPINNED by
reference fixtures: the checker is the CPU oracle's restatement of a ggml MUL_MAT of the projector's weight type
(tests/oracle_py.gemm: the same ggml dot products the encoder's GEMMs are pinned to) plus the bias in f32."""
import os
import subprocess

import numpy as np
import pytest

from conftest import TOOL, rel_errors
import oracle_py
from q2a import ggmlfile

D_IN, D_OUT = 1280, 4096   # Qwen2AudioConfig defaults: audio d_model, text hidden_size


@pytest.fixture(scope="module")
def projector_file(host_build, workdir):
    def make(wt):
        base = os.path.join(workdir, "projector-f16.bin")
        if not os.path.exists(base):
            subprocess.check_call([TOOL, "gen-projector", base, str(D_IN), str(D_OUT), "f16", "0x51A2"])
        if wt == "f16":
            return base
        path = os.path.join(workdir, f"projector-{wt}.bin")
        if not os.path.exists(path):
            subprocess.check_call([TOOL, "quantize", base, path, wt, "8"])
        return path
    return make


@pytest.mark.parametrize("wt,tid", [("f16", 1), ("q4_k", 12), ("q8_0", 8)])
def test_projector_file_layout(projector_file, wt, tid):
    mf = ggmlfile.read(projector_file(wt))
    w = mf.t("multi_modal_projector.linear.weight")
    b = mf.t("multi_modal_projector.linear.bias")
    assert w.type == tid and tuple(w.ne[:2]) == (D_IN, D_OUT)
    assert b.type == 0 and b.ne[0] == D_OUT


@pytest.mark.gpu
@pytest.mark.parametrize("wt", ["f16", "q4_k", "q8_0"])
@pytest.mark.parametrize("rows", [750, 64 * 750])
def test_projector_matches_oracle(projector_file, wt, rows):
    torch = pytest.importorskip("torch")
    import q2a
    path = projector_file(wt)
    mf = ggmlfile.read(path)
    w = np.ascontiguousarray(mf.t("multi_modal_projector.linear.weight").data)
    bias = mf.t("multi_modal_projector.linear.bias").as_f32().reshape(-1)
    pr = q2a.Projector(path, device=0)
    try:
        assert (pr.d_in, pr.d_out) == (D_IN, D_OUT)
        rng = np.random.default_rng(rows)
        n_check = 300   # oracle rows (the CPU dot products are slow); the GPU runs all rows
        x = rng.standard_normal((rows, D_IN)).astype(np.float32)
        xd = torch.from_numpy(x).cuda()
        yd = torch.empty((rows, D_OUT), dtype=torch.float32, device="cuda")
        pr.apply(xd.data_ptr(), rows, yd.data_ptr())
        torch.cuda.synchronize()
        sel = np.unique(np.concatenate([np.arange(8), rng.integers(0, rows, n_check), [rows - 1]]))
        ref = oracle_py.gemm(mf.wtype, w, x[sel], D_OUT) + bias[None, :]
        y = yd.cpu().numpy()[sel]
        mx, l2 = rel_errors(y, ref)
        assert mx < 1e-5 and l2 < 1e-6, (mx, l2)
    finally:
        pr.close()


@pytest.mark.gpu
def test_encoder_then_projector(make_model, make_clip, projector_file):
    """embd_enc of a batch straight from HBM into the projector: rows of one clip do not depend on the batch (bit for
    bit vs the single-clip path), and the projection of the engine's own output matches the oracle."""
    torch = pytest.importorskip("torch")
    import q2a
    eng = q2a.Engine(make_model("full", "q4_k"), device=0)
    pr = q2a.Projector(projector_file("q4_k"), device=0)
    try:
        clips = [make_clip(0), make_clip(1)]
        pcm = torch.from_numpy(np.stack(clips)).cuda()
        emb = torch.empty((2,) + eng.out_shape, dtype=torch.float32, device="cuda")
        eng.encode_device(pcm.data_ptr(), pcm.shape[1], [pcm.shape[1]] * 2, emb.data_ptr())
        torch.cuda.synchronize()
        rows = 2 * eng.out_shape[0]
        y = torch.empty((rows, D_OUT), dtype=torch.float32, device="cuda")
        pr.apply(emb.data_ptr(), rows, y.data_ptr())
        y1 = torch.empty((rows // 2, D_OUT), dtype=torch.float32, device="cuda")
        pr.apply(emb.data_ptr(), rows // 2, y1.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(y[: rows // 2], y1)
        mf = ggmlfile.read(projector_file("q4_k"))
        w = np.ascontiguousarray(mf.t("multi_modal_projector.linear.weight").data)
        bias = mf.t("multi_modal_projector.linear.bias").as_f32().reshape(-1)
        e = emb.cpu().numpy().reshape(rows, -1)
        sel = np.arange(0, rows, 17)
        ref = oracle_py.gemm(mf.wtype, w, e[sel], D_OUT) + bias[None, :]
        mx, l2 = rel_errors(y.cpu().numpy()[sel], ref)
        assert mx < 1e-5 and l2 < 1e-6, (mx, l2)
    finally:
        pr.close()
        eng.close()
