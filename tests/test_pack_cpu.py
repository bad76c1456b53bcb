"""CPU checks of the host-side packer behind q2a_pack_model_ex (no GPU needed: packing is host code).

The blob is self-describing (csrc/q2a_engine.hip `blob_header`): its header records the activation contract, and
under Q2A_ACT_BF16 every linear weight is ggml's dequantize_row_* rounded to bf16 — checked here bit
for bit against a numpy restatement of dequantize_row_q8_0 (ggml-quants.c) for the fused q|k|v matrix of layer 0.
"""
import ctypes as C
import struct

import numpy as np
import pytest

from q2a import ggmlfile

# blob_header layout: u32 magic, version | 11 x i32 hparams | i32 wtype, blk, n_bins, act, compact | u64 total |
# u64 goff[11] | u64 loff[64][32]
OFF_WTYPE, OFF_BLK, OFF_ACT, OFF_COMPACT, OFF_TOTAL, OFF_GOFF = 52, 56, 64, 68, 72, 80
G_COUNT, L_COUNT, L_MAT0, A_COUNT, A_W, A_DX = 11, 32, 8, 6, 0, 1


def header(blob: bytes):
    wtype, blk = struct.unpack_from("<ii", blob, OFF_WTYPE)
    act, = struct.unpack_from("<i", blob, OFF_ACT)
    total, = struct.unpack_from("<Q", blob, OFF_TOTAL)
    loff0 = struct.unpack_from(f"<{L_COUNT}Q", blob, OFF_GOFF + 8 * G_COUNT)
    return wtype, blk, act, total, loff0


def bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def dequant_q8_0(t) -> np.ndarray:
    K = t.ne[0]
    rows = int(np.prod(t.ne)) // K
    blk = t.data.reshape(rows, K // 32, 34)
    d = blk[:, :, :2].copy().view(np.float16).astype(np.float32)
    q = blk[:, :, 2:].copy().view(np.int8).astype(np.float32)
    return (q * d).reshape(rows, K)


def test_bf16_blob_holds_dequantized_bf16_weights(make_model):
    import q2a
    path = make_model("tiny", "q8_0")
    ref_blob = q2a.pack_model(path)
    bf_blob = q2a.pack_model(path, q2a.ACT_BF16)
    wt, blk, act, total, _ = header(ref_blob)
    assert (wt, blk, act, total) == (8, 32, q2a.ACT_REFERENCE, len(ref_blob))
    wt, blk, act, total, loff0 = header(bf_blob)
    assert (wt, blk, act, total) == (8, 0, q2a.ACT_BF16, len(bf_blob))
    assert loff0[L_MAT0 + A_DX] == 0   # no block-scale arrays in the bf16 layout
    mf = ggmlfile.read(path)
    D = 256
    want = np.concatenate([bf16_bits(dequant_q8_0(mf.t(f"layers.0.self_attn.{n}_proj.weight"))) for n in "qkv"])
    off = loff0[L_MAT0 + A_W]
    got = np.frombuffer(bf_blob, dtype=np.uint16, count=3 * D * D, offset=off).reshape(3 * D, D)
    assert np.array_equal(got, want)


def test_unknown_activation_contract_is_rejected(make_model):
    """q2a_open_ex / q2a_pack_model_ex validate the contract before touching a device."""
    import q2a
    path = make_model("tiny", "f16")
    L = q2a.lib()
    assert not L.q2a_open_ex(path.encode(), 0, 7)
    assert b"activation mode" in L.q2a_last_error()
    p = C.c_void_p()
    assert L.q2a_pack_model_ex(path.encode(), 7, C.byref(p)) < 0
    with pytest.raises(q2a.Q2AError):
        q2a.pack_model(path, 7)


def test_blob_version_tracks_the_q4k_layout(make_model):
    """Blob version 3 = Q4_K gamma stored negated (-(dmin/dx)); version 4 = conv1 taps against the three-part mel
    operand; version 5 = the compact transport flag in the header. The Q4_K gamma section of a packed blob must be
    <= 0 everywhere, and the header must say 5 so an older build's blob is refused on open."""
    import q2a
    path = make_model("tiny", "q4_k")
    blob = q2a.pack_model(path)
    magic, version = struct.unpack_from("<II", blob, 0)
    assert magic == 0x42413251 and version == 5
    _, blk, _, _, loff0 = header(blob)
    assert blk == 256
    A_GAMMA = 5
    off = loff0[L_MAT0 + A_GAMMA]
    gamma = np.frombuffer(blob, dtype=np.float32, count=(256 // 256) * 3 * 256, offset=off)
    assert np.all(gamma <= 0) and np.any(gamma < 0)


@pytest.mark.parametrize("cfg,wt", [("tiny", "q4_k"), ("tiny", "q8_0"), ("tiny", "q4_0"), ("tiny", "f16"), ("full", "q4_k")])
def test_compact_blob_is_the_file_rows_plus_small_sections(make_model, cfg, wt):
    """The compact transport blob (q2a_pack_model_compact): same header (compact = 1, goff / loff of the device layout),
    the small sections verbatim, and every linear weight as the model file's own ggml rows (QKV = q | k | v rows).
    For the full-size Q4_K model it is <= 0.4 GB against the 1.40 GB device layout (SURVEY.md §8e's 354 MB of Q4_K
    weights plus the F16 conv kernels, positions and tables). The GPU test expands it and compares bytes."""
    import q2a
    path = make_model(cfg, wt)
    full = q2a.pack_model(path)
    comp = q2a.pack_model(path, compact=True)
    assert struct.unpack_from("<i", comp, OFF_COMPACT)[0] == 1 and struct.unpack_from("<i", full, OFF_COMPACT)[0] == 0
    # the header is the device layout's but for the flag
    hf, hc = bytearray(full[:32768]), bytearray(comp[:32768])
    hc[OFF_COMPACT:OFF_COMPACT + 4] = b"\0\0\0\0"
    assert hf == hc
    dev, tr = q2a.blob_device_size(comp)
    assert dev == len(full) and tr == len(comp)
    assert q2a.blob_device_size(full) == (len(full), len(full))
    if (cfg, wt) == ("full", "q4_k"):
        assert len(comp) <= 0.4e9 < 1.3e9 < len(full)
    # layout (compact_of): global run, per-layer small runs, then the raw rows of layer 0's q | k | v first
    _, _, _, total, loff0 = header(full)
    L = struct.unpack_from("<i", full, 8 + 4 * 4)[0]
    g_len = loff0[0] - 32768
    assert comp[32768:32768 + g_len] == full[32768:32768 + g_len]
    off = 32768 + ((g_len + 255) & ~255)
    for l in range(L):
        lo = struct.unpack_from(f"<{L_COUNT}Q", full, OFF_GOFF + 8 * G_COUNT + 8 * L_COUNT * l)
        n = lo[L_MAT0 + A_W] - lo[0]
        assert comp[off:off + n] == full[lo[0]:lo[0] + n]
        off += (n + 255) & ~255
    mf = ggmlfile.read(path)
    qkv = b"".join(np.ascontiguousarray(mf.t(f"layers.0.self_attn.{n}_proj.weight").data).tobytes() for n in "qkv")
    assert comp[off:off + len(qkv)] == qkv


def test_corrupt_header_is_refused_before_any_size_is_derived(make_model):
    """a header with the right magic / version but a layer count past MAX_LAYERS (64), or offsets that are
    not what the packer lays out, must come back as 'not a q2a weight blob' (Q2A_ERR_FORMAT) from q2a_blob_device_size
    — the same check q2a_open_device_blob and q2a_expand_blob run first — instead of indexing the fixed per-layer
    arrays with it."""
    import q2a
    blob = q2a.pack_model(make_model("tiny", "q4_k"), compact=True)
    head = bytearray(blob[:32768])
    assert q2a.blob_device_size(head)[1] == len(blob)
    for mutate in (lambda h: struct.pack_into("<i", h, 8 + 4 * 4, 1000),          # n_audio_layer = 1000
                   lambda h: struct.pack_into("<i", h, 8 + 4 * 4, 0),             # no layers
                   lambda h: struct.pack_into("<i", h, 8 + 4 * 2, 250),           # D not a multiple of 128
                   lambda h: struct.pack_into("<Q", h, OFF_TOTAL, 1 << 40),       # device size not the plan's
                   lambda h: struct.pack_into("<Q", h, OFF_GOFF + 8 * G_COUNT, 7),  # layer 0's first offset moved
                   lambda h: struct.pack_into("<i", h, OFF_COMPACT, 5),
                   lambda h: struct.pack_into("<i", h, OFF_WTYPE, 99)):
        bad = bytearray(head)
        mutate(bad)
        with pytest.raises(q2a.Q2AError, match="not a q2a weight blob"):
            q2a.blob_device_size(bad)
