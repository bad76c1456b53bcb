"""Python host mirror of the MI355X encoder path (ctypes over the C ABI in include/q2a_encoder.h).

The product is lib/libq2a.so (HIP kernels for gfx950). This module only marshals arguments; there is no
CPU fallback: if the library or a GPU is missing every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("Q2A_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libq2a.so")   # override: A/B builds
HOST_LIB_PATH = os.path.join(PKG_DIR, "lib", "libq2a_host.so")
TOOL_PATH = os.path.join(PKG_DIR, "bin", "q2a_tool")

EXPORTS = (
    "q2a_last_error", "q2a_open", "q2a_pack_model", "q2a_free_host_blob", "q2a_open_device_blob", "q2a_close",
    "q2a_get_info", "q2a_reserve", "q2a_encode_device", "q2a_encode_host", "q2a_pcm_to_mel",
    "q2a_encode_host_ex", "q2a_test_linear", "q2a_test_block", "q2a_test_block_taps", "q2a_test_attention", "q2a_test_fc1_path",
    "q2a_test_frontend", "q2a_test_pool_ln",
    "q2a_projector_open", "q2a_projector_close", "q2a_projector_get_dims", "q2a_projector_apply",
    "q2a_pack_model_compact", "q2a_blob_device_size", "q2a_expand_blob",
    "q2a_device_count", "q2a_group_open", "q2a_group_close", "q2a_group_size", "q2a_group_engine", "q2a_group_split",
    "q2a_group_encode_host", "q2a_group_setup_times", "q2a_group_open_with", "q2a_whisper_context_engine",
)

# per-clip status of the encode calls (include/q2a_encoder.h): FAILED = the host call returned an error before this
# clip's output reached the caller
CLIP_ENCODED, CLIP_SKIPPED, CLIP_FAILED = 0, 1, 2


class Q2AError(RuntimeError):
    pass


class Info(C.Structure):
    _fields_ = [("n_audio_ctx", C.c_int32), ("n_audio_state", C.c_int32), ("n_audio_head", C.c_int32),
                ("n_audio_layer", C.c_int32), ("n_mels", C.c_int32), ("wtype", C.c_int32), ("n_out", C.c_int32),
                ("device", C.c_int32), ("weight_bytes", C.c_int64), ("workspace_bytes", C.c_int64),
                ("act", C.c_int32), ("reserved", C.c_int32)]


# activation contracts (include/q2a_encoder.h)
ACT_REFERENCE = 0
ACT_BF16 = 1


_lib = None


def lib() -> C.CDLL:
    """Load libq2a.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Q2AError(f"{LIB_PATH} not built; run `make -C {PKG_DIR}` (hipcc --offload-arch=gfx950)")
        L = C.CDLL(LIB_PATH)
        vp, i32p, f32p = C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_float)
        L.q2a_last_error.restype = C.c_char_p
        L.q2a_open.restype = vp
        L.q2a_open.argtypes = [C.c_char_p, C.c_int]
        L.q2a_open_ex.restype = vp
        L.q2a_open_ex.argtypes = [C.c_char_p, C.c_int, C.c_int]
        L.q2a_pack_model.restype = C.c_int64
        L.q2a_pack_model.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.q2a_pack_model_ex.restype = C.c_int64
        L.q2a_pack_model_ex.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
        L.q2a_free_host_blob.argtypes = [vp]
        if hasattr(L, "q2a_pack_model_compact"):   # round 4 (optional: earlier diagnostic builds load too)
            L.q2a_pack_model_compact.restype = C.c_int64
            L.q2a_pack_model_compact.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
            L.q2a_blob_device_size.restype = C.c_int64
            L.q2a_blob_device_size.argtypes = [vp, C.c_int64, C.POINTER(C.c_int64)]
            L.q2a_expand_blob.argtypes = [vp, C.c_int64, vp, C.c_int64, C.c_int, vp]
        L.q2a_open_device_blob.restype = vp
        L.q2a_open_device_blob.argtypes = [vp, C.c_int64, C.c_int]
        L.q2a_close.argtypes = [vp]
        L.q2a_get_info.argtypes = [vp, C.POINTER(Info)]
        L.q2a_reserve.argtypes = [vp, C.c_int, C.c_int64]
        L.q2a_encode_device.argtypes = [vp, vp, C.c_int64, i32p, C.c_int, C.c_int, vp, i32p, vp]
        L.q2a_encode_host.argtypes = [vp, C.POINTER(vp), i32p, C.c_int, C.c_int, vp, i32p]
        L.q2a_encode_host_ex.argtypes = [vp, C.POINTER(vp), i32p, i32p, C.c_int, C.c_int, vp, i32p]
        L.q2a_pcm_to_mel.argtypes = [vp, vp, C.c_int, vp, C.c_int64, i32p]
        L.q2a_test_linear.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int, vp, vp]
        L.q2a_test_block.argtypes = [vp, C.c_int, vp, C.c_int, vp]
        L.q2a_test_block_taps.argtypes = [vp, C.c_int, vp, C.c_int, C.POINTER(vp), vp]
        L.q2a_test_attention.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp]
        # test hooks added in round 3: optional, so a diagnostic library of an earlier revision (diag/build_rev_lib.sh,
        # A/B runs) still loads; the shipped library exports them (tests/test_library_abi.py checks EXPORTS)
        for name, at in (("q2a_test_fc1_path", [vp, C.c_int]), ("q2a_test_frontend", [vp, vp, C.c_int64, i32p, C.c_int, vp, vp]),
                         ("q2a_test_pool_ln", [vp, vp, C.c_int, vp, vp])):
            if hasattr(L, name):
                getattr(L, name).argtypes = at
        if hasattr(L, "q2a_group_open"):   # round 5 (optional: earlier diagnostic builds load too)
            L.q2a_group_open.restype = vp
            L.q2a_group_open.argtypes = [C.c_char_p, i32p, C.c_int, C.c_int]
            L.q2a_group_open_with.restype = vp
            L.q2a_group_open_with.argtypes = [vp, i32p, C.c_int]
            L.q2a_group_close.argtypes = [vp]
            L.q2a_group_size.argtypes = [vp]
            L.q2a_group_engine.restype = vp
            L.q2a_group_engine.argtypes = [vp, C.c_int]
            L.q2a_group_split.argtypes = [C.c_int, C.c_int, C.c_int, i32p, i32p]
            L.q2a_group_encode_host.argtypes = [vp, C.POINTER(vp), i32p, i32p, C.c_int, C.c_int, vp, i32p]
            L.q2a_group_setup_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        L.q2a_projector_open.restype = vp
        L.q2a_projector_open.argtypes = [C.c_char_p, C.c_int]
        L.q2a_projector_close.argtypes = [vp]
        L.q2a_projector_get_dims.argtypes = [vp, i32p, i32p, i32p]
        L.q2a_projector_apply.argtypes = [vp, vp, C.c_int64, vp, vp]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise Q2AError(f"q2a error {rc}: {lib().q2a_last_error().decode()}")


class Engine:
    """One encoder engine on one HIP device (the analogue of a whisper_context + whisper_state)."""

    def __init__(self, model_path: str | None = None, device: int = 0, device_blob: int | None = None,
                 blob_size: int | None = None, act: int = ACT_REFERENCE):
        L = lib()
        if device_blob is not None:   # the blob carries its own activation contract
            h = L.q2a_open_device_blob(C.c_void_p(device_blob), C.c_int64(blob_size), device)
        else:
            h = L.q2a_open_ex(model_path.encode(), device, act)
        if not h:
            raise Q2AError(L.q2a_last_error().decode())
        self.h = h
        self.info = Info()
        _check(L.q2a_get_info(self.h, C.byref(self.info)))

    def close(self):
        if self.h:
            lib().q2a_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def out_shape(self):
        return (self.info.n_out, self.info.n_audio_state)

    def reserve(self, n_clips: int, max_samples: int = 0):
        _check(lib().q2a_reserve(self.h, n_clips, max_samples))
        _check(lib().q2a_get_info(self.h, C.byref(self.info)))

    def encode_device(self, pcm_ptr: int, pcm_stride: int, n_samples, out_ptr: int, offset_ms: int = 0,
                      stream: int | None = None):
        ns = np.ascontiguousarray(n_samples, dtype=np.int32)
        st = np.zeros(len(ns), dtype=np.int32)
        _check(lib().q2a_encode_device(self.h, C.c_void_p(pcm_ptr), C.c_int64(pcm_stride),
                                       ns.ctypes.data_as(C.POINTER(C.c_int32)), len(ns), offset_ms,
                                       C.c_void_p(out_ptr), st.ctypes.data_as(C.POINTER(C.c_int32)),
                                       C.c_void_p(stream) if stream else None))
        return st

    def encode_host(self, clips, offset_ms: int = 0, out: np.ndarray | None = None, offsets_ms=None,
                    raise_on_error: bool = True):
        """Encode host PCM clips. offsets_ms: per-clip window offsets (q2a_encode_host_ex). With raise_on_error=False a
        failing call returns (out, status, rc) instead of raising: status then marks every clip whose output never
        reached `out` as CLIP_FAILED."""
        clips = [np.ascontiguousarray(c, dtype=np.float32) for c in clips]
        n = len(clips)
        if out is None:
            out = np.zeros((n,) + self.out_shape, dtype=np.float32)
        ptrs = (C.c_void_p * n)(*[c.ctypes.data for c in clips])
        ns = np.array([len(c) for c in clips], dtype=np.int32)
        st = np.full(n, -1, dtype=np.int32)
        i32p = C.POINTER(C.c_int32)
        if offsets_ms is None:
            rc = lib().q2a_encode_host(self.h, ptrs, ns.ctypes.data_as(i32p), n, offset_ms,
                                       C.c_void_p(out.ctypes.data), st.ctypes.data_as(i32p))
        else:
            offs = np.ascontiguousarray(offsets_ms, dtype=np.int32)
            assert len(offs) == n
            rc = lib().q2a_encode_host_ex(self.h, ptrs, ns.ctypes.data_as(i32p), offs.ctypes.data_as(i32p), n, offset_ms,
                                          C.c_void_p(out.ctypes.data), st.ctypes.data_as(i32p))
        if not raise_on_error:
            return out, st, rc
        _check(rc)
        return out, st

    def pcm_to_mel(self, pcm: np.ndarray) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        n_len = (len(pcm) + 480000) // 160
        out = np.empty((self.info.n_mels, n_len), dtype=np.float32)
        got = C.c_int32(0)
        _check(lib().q2a_pcm_to_mel(self.h, C.c_void_p(pcm.ctypes.data), len(pcm), C.c_void_p(out.ctypes.data),
                                    C.c_int64(out.size), C.byref(got)))
        assert got.value == n_len
        return out

    # kernel-level entry points on device pointers (parity tests)
    def test_linear(self, layer, which, x_ptr, M, y_ptr, stream=None):
        _check(lib().q2a_test_linear(self.h, layer, which, C.c_void_p(x_ptr), M, C.c_void_p(y_ptr),
                                     C.c_void_p(stream) if stream else None))

    def test_block(self, layer, x_ptr, n_clips, stream=None):
        _check(lib().q2a_test_block(self.h, layer, C.c_void_p(x_ptr), n_clips, C.c_void_p(stream) if stream else None))

    def test_block_taps(self, layer, x_ptr, n_clips, tap_ptrs, stream=None):
        arr = (C.c_void_p * 4)(*[C.c_void_p(t) if t else None for t in tap_ptrs])
        _check(lib().q2a_test_block_taps(self.h, layer, C.c_void_p(x_ptr), n_clips, arr,
                                         C.c_void_p(stream) if stream else None))

    def test_frontend(self, pcm_ptr, pcm_stride, n_samples, x_ptr, stream=None):
        ns = np.ascontiguousarray(n_samples, dtype=np.int32)
        _check(lib().q2a_test_frontend(self.h, C.c_void_p(pcm_ptr), C.c_int64(pcm_stride),
                                       ns.ctypes.data_as(C.POINTER(C.c_int32)), len(ns), C.c_void_p(x_ptr),
                                       C.c_void_p(stream) if stream else None))

    def test_pool_ln(self, x_ptr, n_clips, out_ptr, stream=None):
        _check(lib().q2a_test_pool_ln(self.h, C.c_void_p(x_ptr), n_clips, C.c_void_p(out_ptr),
                                      C.c_void_p(stream) if stream else None))

    def test_fc1_path(self, path):
        _check(lib().q2a_test_fc1_path(self.h, path))

    def test_attention(self, q_ptr, k_ptr, v_ptr, n_clips, out_ptr, stream=None):
        _check(lib().q2a_test_attention(self.h, C.c_void_p(q_ptr), C.c_void_p(k_ptr), C.c_void_p(v_ptr), n_clips,
                                        C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None))


def group_split(n_clips: int, n_devices: int) -> list[range]:
    """The contiguous clip ranges q2a_group gives each device (q2a_group_split)."""
    out = []
    for i in range(n_devices):
        f, c = C.c_int32(), C.c_int32()
        _check(lib().q2a_group_split(n_clips, n_devices, i, C.byref(f), C.byref(c)))
        out.append(range(f.value, f.value + c.value))
    return out


class Group:
    """Several GPUs in ONE process (q2a_group_*): one RCCL broadcast of the weights at open, then clip batches split
    into contiguous ranges, a host thread per device. devices=None: every visible device.
    From a model file (q2a_group_open: the compact blob packed once on the host), or with engine= an open Engine
    (q2a_group_open_with: its own device-layout weights are the broadcast's root, its device's group engine shares
    them; the Engine must outlive the group)."""

    def __init__(self, model_path: str | None = None, devices=None, act: int = ACT_REFERENCE, engine=None):
        L = lib()
        devs = np.ascontiguousarray(devices if devices is not None else [], dtype=np.int32)
        dptr = devs.ctypes.data_as(C.POINTER(C.c_int32)) if len(devs) else None
        if engine is not None:
            self.h = L.q2a_group_open_with(C.c_void_p(engine.h), dptr, len(devs))
        else:
            self.h = L.q2a_group_open(model_path.encode(), dptr, len(devs), act)
        if not self.h:
            raise Q2AError(L.q2a_last_error().decode())
        self.size = L.q2a_group_size(self.h)
        info = Info()
        _check(L.q2a_get_info(L.q2a_group_engine(self.h, 0), C.byref(info)))
        self.out_shape = (info.n_out, info.n_audio_state)

    def setup_times(self) -> dict:
        a, b, c, n = C.c_double(), C.c_double(), C.c_double(), C.c_int64()
        _check(lib().q2a_group_setup_times(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(n)))
        return {"pack_s": a.value, "broadcast_s": b.value, "open_s": c.value, "blob_bytes": n.value}

    def encode_host(self, clips, offset_ms: int = 0, offsets_ms=None, out: np.ndarray | None = None):
        clips = [np.ascontiguousarray(c, dtype=np.float32) for c in clips]
        n = len(clips)
        if out is None:
            out = np.zeros((n,) + self.out_shape, dtype=np.float32)
        ptrs = (C.c_void_p * n)(*[c.ctypes.data for c in clips])
        ns = np.array([len(c) for c in clips], dtype=np.int32)
        st = np.full(n, -1, dtype=np.int32)
        i32p = C.POINTER(C.c_int32)
        offs = None if offsets_ms is None else np.ascontiguousarray(offsets_ms, dtype=np.int32)
        if offs is not None and len(offs) != n:
            raise ValueError(f"offsets_ms has {len(offs)} entries for {n} clips")
        _check(lib().q2a_group_encode_host(self.h, ptrs, ns.ctypes.data_as(i32p),
                                           offs.ctypes.data_as(i32p) if offs is not None else None, n, offset_ms,
                                           C.c_void_p(out.ctypes.data), st.ctypes.data_as(i32p)))
        return out, st

    def close(self):
        if self.h:
            lib().q2a_group_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Projector:
    """The Qwen2-Audio multi-modal projector (Linear d_model -> text hidden, bias) on the GPU: the consumer of embd_enc
    (include/q2a_encoder.h, q2a_projector_*). No CPU fallback."""

    def __init__(self, path: str, device: int = 0):
        self.h = lib().q2a_projector_open(path.encode(), device)
        if not self.h:
            raise Q2AError(lib().q2a_last_error().decode())
        a, b, w = C.c_int32(), C.c_int32(), C.c_int32()
        _check(lib().q2a_projector_get_dims(self.h, C.byref(a), C.byref(b), C.byref(w)))
        self.d_in, self.d_out, self.wtype = a.value, b.value, w.value

    def apply(self, x_ptr: int, rows: int, y_ptr: int, stream=None):
        _check(lib().q2a_projector_apply(self.h, C.c_void_p(x_ptr), rows, C.c_void_p(y_ptr),
                                         C.c_void_p(stream) if stream else None))

    def close(self):
        if self.h:
            lib().q2a_projector_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def pack_model(path: str, act: int = ACT_REFERENCE, compact: bool = False) -> bytearray:
    """Pack a model file into a blob (host bytes, one copy out of the library's buffer): the device layout, or with
    compact=True its transport form (ggml weight rows, expanded on the GPU by Engine(device_blob=...)), e.g. for the
    RCCL broadcast."""
    p = C.c_void_p()
    f = lib().q2a_pack_model_compact if compact else lib().q2a_pack_model_ex
    n = f(path.encode(), act, C.byref(p))
    if n < 0:
        raise Q2AError(lib().q2a_last_error().decode())
    try:
        out = bytearray(n)
        C.memmove((C.c_char * n).from_buffer(out), p, n)
        return out
    finally:
        lib().q2a_free_host_blob(p)


def blob_device_size(blob) -> tuple[int, int]:
    """(device-layout bytes, transport bytes) of a host blob (its header)."""
    head = (C.c_char * 32768).from_buffer_copy(bytes(blob[:32768]))
    tb = C.c_int64(0)
    n = lib().q2a_blob_device_size(C.cast(head, C.c_void_p), 32768, C.byref(tb))
    if n < 0:
        raise Q2AError(lib().q2a_last_error().decode())
    return int(n), int(tb.value)


def expand_blob(dev_ptr: int, size: int, out_ptr: int, out_bytes: int, device: int = 0, stream=None):
    """Expand a compact blob on the device into the device layout (what q2a_open_device_blob does internally)."""
    _check(lib().q2a_expand_blob(C.c_void_p(dev_ptr), C.c_int64(size), C.c_void_p(out_ptr), C.c_int64(out_bytes),
                                 device, C.c_void_p(stream) if stream else None))
