"""Isolated parity of the two ends of the path, which the end-to-end tests cover only through 32
layers: the front end (PCM -> log-mel -> conv1 + GELU -> conv2 + GELU -> + positions, the first block's input) and
AvgPool1d(2) + final LayerNorm. The checker is the oracle run with ZERO encoder layers (oracle/q2a_oracle.c: its conv
output is then pooled and normalised directly), plus the reference's own layer-0 input samples (tests/golden,
tiny_f16_l0_conv_out, from the reference build itself)."""
import numpy as np
import pytest

from conftest import rel_errors
import oracle_py
from q2a import ggmlfile

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def frontend(make_model, make_clip):
    """(cfg) -> engine X [T][D], oracle conv_out [T][D], oracle pool+LN of conv_out [T/2][D], engine handle."""
    import q2a
    cache = {}

    def get(cfg):
        if cfg in cache:
            return cache[cfg]
        path = make_model(cfg, "f16")
        e = q2a.Engine(path, device=0)
        pcm = make_clip(0)
        T, D = e.info.n_audio_ctx, e.info.n_audio_state
        pd = torch.from_numpy(pcm).cuda()
        xd = torch.empty((T, D), dtype=torch.float32, device="cuda")
        e.test_frontend(pd.data_ptr(), len(pcm), [len(pcm)], xd.data_ptr())
        torch.cuda.synchronize()
        o = oracle_py.Oracle(ggmlfile.read(path))
        o.m.n_layer = 0                       # conv -> pool + LN directly
        out0, dumps = o.encode(o.mel_window(o.log_mel(pcm)), dump=True)
        cache[cfg] = (xd.cpu().numpy(), dumps["conv_out"], out0, e)
        return cache[cfg]

    yield get
    for v in cache.values():
        v[3].close()


@pytest.mark.parametrize("cfg", ["tiny", "full"])
def test_frontend_matches_oracle(frontend, frontend_bar, cfg):
    """mel bit-exact, conv operands exact (mel hi|lo x fp16 kernel, fp32 accumulation), ggml's fp16 GELU table: only
    the fp32 summation order differs — but a 1-ulp f32 difference at a GELU input rounds to the neighbouring fp16 table
    entry now and then (1 fp16 ulp of that element: the max-rel), exactly as between two builds of the reference. Bar:
    the reference's own widest cross-build disagreement on this output (frontend_bar, x1.0)."""
    x, ref, _, _ = frontend(cfg)
    mx, l2 = rel_errors(x, ref)
    bar = frontend_bar(cfg)
    assert mx <= bar["max_rel"] and l2 <= bar["rel_l2"], (cfg, mx, l2, bar)


def test_frontend_matches_reference_samples(frontend, frontend_bar, golden):
    """The same output against samples of the REFERENCE's own layer-0 input (tiny F16 model, clip 0)."""
    _, g = golden
    x, _, _, _ = frontend("tiny")
    idx, val = g["tiny_f16_l0_conv_out_idx"], g["tiny_f16_l0_conv_out_val"]
    mx, l2 = rel_errors(x.reshape(-1)[idx], val)
    bar = frontend_bar("tiny")
    assert mx <= bar["max_rel"] and l2 <= bar["rel_l2"], (mx, l2, bar)


@pytest.mark.parametrize("cfg", ["tiny", "full"])
def test_pool_ln_matches_oracle(frontend, cfg):
    """k_pool_ln on the ORACLE's conv output (so nothing upstream differs): AvgPool1d(2) as ggml's drow = 0; += a;
    += b; /= 2, LayerNorm with double sums and ggml's f32 operation order — agrees to an f32 ulp or so."""
    _, conv_ref, out_ref, e = frontend(cfg)
    T, D = conv_ref.shape
    xd = torch.from_numpy(np.ascontiguousarray(conv_ref)).cuda()
    yd = torch.empty((T // 2, D), dtype=torch.float32, device="cuda")
    e.test_pool_ln(xd.data_ptr(), 1, yd.data_ptr())
    torch.cuda.synchronize()
    mx, l2 = rel_errors(yd.cpu().numpy(), out_ref)
    assert mx < 1e-6 and l2 < 1e-7, (cfg, mx, l2)


def test_pool_ln_two_clips_independent(frontend):
    """Two clips through one launch: each equals its single-clip result bit for bit (rows never mix across clips)."""
    _, conv_ref, _, e = frontend("tiny")
    T, D = conv_ref.shape
    rng = np.random.default_rng(5)
    other = (rng.standard_normal((T, D)) * 3.0).astype(np.float32)
    both = torch.from_numpy(np.concatenate([conv_ref, other])).cuda()
    y2 = torch.empty((2, T // 2, D), dtype=torch.float32, device="cuda")
    e.test_pool_ln(both.data_ptr(), 2, y2.data_ptr())
    y1 = torch.empty((T // 2, D), dtype=torch.float32, device="cuda")
    e.test_pool_ln(both[T:].data_ptr(), 1, y1.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(y2[1], y1)
