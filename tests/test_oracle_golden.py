"""Pin the CPU oracle (oracle/q2a_oracle.c) and our format tooling against the golden vectors that the REAL
reference produced (tests/golden/make_golden.py -> oracle/_ref/ref_harness). CPU only."""
import ctypes as C

import numpy as np
import pytest

from conftest import PKG, rel_errors
import oracle_py
from q2a import ggmlfile


def host_lib():
    import os
    return C.CDLL(os.path.join(PKG, "lib", "libq2a_host.so"))


def test_model_generator_and_quantizer_hashes(make_model):
    # make_model asserts the SHA-256 recorded when the reference quantize flow produced identical bytes
    for wt in ("f16", "q4_k", "q8_0", "q4_0"):
        make_model("tiny", wt)


def test_weight_quantizers_byte_exact(host_build, golden):
    _, g = golden
    x = g["kat_x"]
    hl = host_lib()
    for kind, fn, rs in (("q4k", hl.q2a_quantize_row_q4_K, 144 * 1280 // 256),
                         ("q80", hl.q2a_quantize_row_q8_0, 34 * 1280 // 32)):
        out = np.empty(8 * rs, dtype=np.uint8)
        for r in range(8):
            row = np.ascontiguousarray(x[r])
            fn(row.ctypes.data_as(C.c_void_p), C.c_void_p(out.ctypes.data + r * rs), C.c_int64(1280))
        assert np.array_equal(out, g[f"kat_{kind}"]), kind


def test_fp16_conversion_matches_ggml(host_build, golden):
    _, g = golden
    x = g["kat_x"].reshape(-1)
    hl = host_lib()
    hl.q2a_fp32_to_fp16.restype = C.c_uint16
    hl.q2a_fp32_to_fp16.argtypes = [C.c_float]
    mine = np.array([hl.q2a_fp32_to_fp16(float(v)) for v in x[:4096]], dtype=np.uint16)
    assert np.array_equal(mine, g["kat_f16"].view(np.uint16)[:4096])
    orc = np.array([oracle_py.lib().oracle_fp32_to_fp16(float(v)) for v in x[:4096]], dtype=np.uint16)
    assert np.array_equal(orc, mine)
    # edge cases: subnormals, rounding ties, overflow, inf/nan
    edge = np.array([0.0, -0.0, 6.1e-5, 5.96e-8, 2.98e-8, 65504.0, 65519.0, 65520.0, 1e9, -1e9,
                     1.0009765625, 1.00048828125, np.inf, -np.inf], dtype=np.float32)
    for v in edge:
        assert hl.q2a_fp32_to_fp16(float(v)) == np.float32(v).astype(np.float16).view(np.uint16), v


def test_activation_quantizers_match_ggml(host_build, golden):
    _, g = golden
    x = g["kat_x"]
    assert np.array_equal(oracle_py.quantize_act("q8k", x), g["kat_act_q8k"])
    assert np.array_equal(oracle_py.quantize_act("q80", x), g["kat_act_q80"])


@pytest.mark.parametrize("kind,wt", [("f16", 1), ("q4k", 12), ("q80", 8)])
def test_oracle_gemm_matches_ggml_vec_dot(host_build, golden, kind, wt):
    _, g = golden
    w, xa = g["kat_w"], g["kat_xa"]
    hl = host_lib()
    if wt == 1:
        wraw = w.astype(np.float16).view(np.uint8)
    else:
        rs = 144 * 1280 // 256 if wt == 12 else 34 * 1280 // 32
        fn = hl.q2a_quantize_row_q4_K if wt == 12 else hl.q2a_quantize_row_q8_0
        wraw = np.empty(w.shape[0] * rs, dtype=np.uint8)
        for r in range(w.shape[0]):
            row = np.ascontiguousarray(w[r])
            fn(row.ctypes.data_as(C.c_void_p), C.c_void_p(wraw.ctypes.data + r * rs), C.c_int64(1280))
    y = oracle_py.gemm(wt, wraw, xa, w.shape[0])
    mx, l2 = rel_errors(y, g[f"kat_gemm_{kind}"])
    assert mx < 1e-6 and l2 < 1e-6, (mx, l2)


@pytest.mark.parametrize("clip", [0, 2, 3])
def test_oracle_mel_bit_exact(make_model, make_clip, golden, clip):
    meta, g = golden
    mf = ggmlfile.read(make_model("tiny", "f16"))
    o = oracle_py.Oracle(mf)
    mel = o.log_mel(make_clip(clip))
    info = meta["outputs"][f"mel{clip}"]
    assert mel.shape == (info["n_mel"], info["n_len"])
    # bit-exact: same float op order as log_mel_spectrogram, both built without FMA contraction
    assert np.array_equal(mel.reshape(-1)[g[f"mel{clip}_idx"]], g[f"mel{clip}_val"])
    np.testing.assert_allclose(mel.astype(np.float64).sum(axis=1), g[f"mel{clip}_rowsum"], rtol=1e-12)


def test_oracle_encoder_tiny_f16(make_model, make_clip, golden):
    _, g = golden
    mf = ggmlfile.read(make_model("tiny", "f16"))
    o = oracle_py.Oracle(mf)
    out, dumps = o.encode(o.mel_window(o.log_mel(make_clip(0))), dump=True)
    ref = g["tiny_f16_c0"]
    mx, l2 = rel_errors(out, ref)
    assert mx < 2e-4 and l2 < 5e-5, (mx, l2)
    # layer-0 intermediates (ggml node outputs of the same call)
    for nm, tol in (("conv_out", 3e-4), ("ln1", 3e-4), ("q", 3e-4), ("k", 3e-4), ("v", 3e-4), ("attn", 3e-4),
                    ("x1", 3e-4), ("gelu", 1.5e-3), ("x2", 3e-4)):
        idx, val = g[f"tiny_f16_l0_{nm}_idx"], g[f"tiny_f16_l0_{nm}_val"]
        mine = dumps[nm].reshape(-1)[idx]
        err = np.abs(mine - val).max() / max(np.abs(val).max(), 1e-6)
        assert err < tol, (nm, err)


@pytest.mark.parametrize("wt", ["q4_k", "q8_0", "q4_0"])
def test_oracle_encoder_tiny_quantized(make_model, make_clip, golden, wt):
    """Quantized paths: activations are re-quantized to Q8_K/Q8_0 before every GEMM, so a 1e-7 difference
    in F32 summation order flips single int8 codes (one flip moves affected outputs by ~1e-3 relative).
    Two faithful implementations therefore agree to ~3e-4 relative L2, not bitwise; bound accordingly."""
    meta, g = golden
    mf = ggmlfile.read(make_model("tiny", wt))
    o = oracle_py.Oracle(mf)
    out = o.encode(o.mel_window(o.log_mel(make_clip(0))))
    ref_rows = g[f"tiny_{wt}_c0_rows"]
    mx, l2 = rel_errors(out[g["rows_stride5"]], ref_rows)
    assert l2 < 1e-3 and mx < 3e-3, (mx, l2)
    assert abs(np.linalg.norm(out) / meta["outputs"][f"tiny_{wt}_c0"]["l2"] - 1) < 1e-3


@pytest.mark.parametrize("clip", [1, 2, 3])
def test_oracle_encoder_other_clips(make_model, make_clip, golden, clip):
    """Second 30 s clip, a 7.3 s clip (zero-padded window) and a 41 s clip (truncated to the first 30 s,
    normalised over the whole mel, qwen2-whisper.cpp:2633-2649, 2366-2372)."""
    _, g = golden
    mf = ggmlfile.read(make_model("tiny", "f16"))
    o = oracle_py.Oracle(mf)
    out = o.encode(o.mel_window(o.log_mel(make_clip(clip))))
    mx, l2 = rel_errors(out[g["rows_stride5"]], g[f"tiny_f16_c{clip}_rows"])
    assert mx < 2e-4 and l2 < 5e-5, (mx, l2)


def test_compact_gelu_lookup_equals_the_full_table():
    """The GELU lookups that use only the |x| < 10 image of ggml's fp16 table (the GEMM epilogues' LDS table, and the
    fc1 -> fc2 quantizer with Q2A_GELU_COMPACT): for every fp16 input h the selection `x >= 10 -> x; x <= -10 -> -0
    (+0 for -inf, ggml's x <= -10 branch); else table_c[index(h)]` is bit for bit the full table (with the quantizer's
    -inf -> +0 entry), exhaustively over all 65 536 inputs but the NaNs, which that kernel reads from the full table."""
    tab = np.zeros(65536, dtype=np.uint16)
    host_lib().q2a_make_gelu_table(tab.ctypes.data_as(C.c_void_p))
    full = tab.copy()
    full[0xFC00] = 0
    HALF = 0x4901
    comp = np.concatenate([tab[:HALF], tab[0x8000:0x8000 + HALF]])
    u = np.arange(65536, dtype=np.uint32)
    x = u.astype(np.uint16).view(np.float16).astype(np.float32)
    idx = np.minimum(u & 0x7FFF, HALF - 1) + np.where(u & 0x8000, HALF, 0)
    got = comp[idx]
    got = np.where(x >= 10, u.astype(np.uint16), got)
    got = np.where(x <= -10, np.where(np.isneginf(x), np.uint16(0), np.uint16(0x8000)), got)
    ok = ~np.isnan(x)
    assert np.array_equal(got[ok], full[ok])
