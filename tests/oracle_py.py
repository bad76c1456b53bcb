"""ctypes bindings of the CPU oracle (oracle/_build/libq2a_oracle.so) — TEST INFRASTRUCTURE ONLY.

The oracle is the checker: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libq2a_oracle.so")
REF_HARNESS = os.path.join(ORACLE_DIR, "_ref", "ref_harness")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-C", ORACLE_DIR, "oracle"], stdout=subprocess.DEVNULL)
        _lib = C.CDLL(LIB_PATH)
        _lib.oracle_log_mel.restype = C.c_int
        _lib.oracle_encode.restype = C.c_int
        _lib.oracle_gelu.restype = C.c_float
        _lib.oracle_gelu.argtypes = [C.c_float]
        _lib.oracle_fp32_to_fp16.restype = C.c_uint16
        _lib.oracle_fp32_to_fp16.argtypes = [C.c_float]
    return _lib


PV = C.c_void_p
PF = C.POINTER(C.c_float)


class OracleModel(C.Structure):
    _fields_ = [("n_layer", C.c_int), ("d", C.c_int), ("n_head", C.c_int), ("n_mels", C.c_int), ("n_ctx", C.c_int),
                ("wtype", C.c_int), ("conv_type", C.c_int),
                ("conv1_w", PV), ("conv1_b", PV), ("conv2_w", PV), ("conv2_b", PV), ("pe", PV),
                ("ln_post_w", PV), ("ln_post_b", PV),
                ("q_w", C.POINTER(PV)), ("q_b", C.POINTER(PV)), ("k_w", C.POINTER(PV)),
                ("v_w", C.POINTER(PV)), ("v_b", C.POINTER(PV)), ("o_w", C.POINTER(PV)), ("o_b", C.POINTER(PV)),
                ("ln1_w", C.POINTER(PV)), ("ln1_b", C.POINTER(PV)),
                ("fc1_w", C.POINTER(PV)), ("fc1_b", C.POINTER(PV)),
                ("fc2_w", C.POINTER(PV)), ("fc2_b", C.POINTER(PV)),
                ("ln2_w", C.POINTER(PV)), ("ln2_b", C.POINTER(PV))]


class OracleDump(C.Structure):
    _fields_ = [(n, PV) for n in ("conv_out", "ln1", "q", "k", "v", "attn", "x1", "gelu", "x2")]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(PV)


class Oracle:
    """Holds a parsed ggml model (q2a.ggmlfile.ModelFile) as an oracle_model struct."""

    def __init__(self, mf):
        self.mf = mf
        hp = mf.hparams
        L = hp["n_audio_layer"]
        self._keep = []
        m = OracleModel()
        m.n_layer, m.d, m.n_head, m.n_mels, m.n_ctx = L, hp["n_audio_state"], hp["n_audio_head"], hp["n_mels"], hp["n_audio_ctx"]
        m.wtype = mf.wtype
        m.conv_type = mf.t("conv1.weight").type

        def raw(name):
            a = np.ascontiguousarray(mf.t(name).data)
            self._keep.append(a)
            return _ptr(a)

        m.conv1_w, m.conv1_b = raw("conv1.weight"), raw("conv1.bias")
        m.conv2_w, m.conv2_b = raw("conv2.weight"), raw("conv2.bias")
        m.pe = raw("embed_positions.weight")
        m.ln_post_w, m.ln_post_b = raw("layer_norm.weight"), raw("layer_norm.bias")
        per = {"q_w": "self_attn.q_proj.weight", "q_b": "self_attn.q_proj.bias", "k_w": "self_attn.k_proj.weight",
               "v_w": "self_attn.v_proj.weight", "v_b": "self_attn.v_proj.bias",
               "o_w": "self_attn.out_proj.weight", "o_b": "self_attn.out_proj.bias",
               "ln1_w": "self_attn_layer_norm.weight", "ln1_b": "self_attn_layer_norm.bias",
               "fc1_w": "fc1.weight", "fc1_b": "fc1.bias", "fc2_w": "fc2.weight", "fc2_b": "fc2.bias",
               "ln2_w": "final_layer_norm.weight", "ln2_b": "final_layer_norm.bias"}
        for field, suffix in per.items():
            arr = (PV * L)(*[raw(f"layers.{i}.{suffix}") for i in range(L)])
            self._keep.append(arr)
            setattr(m, field, C.cast(arr, C.POINTER(PV)))
        self.m = m

    def log_mel(self, pcm: np.ndarray, n_threads: int = 8) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        n_mel, n_fft = self.mf.filters.shape
        cap = (len(pcm) + 480000) // 160 + 1
        out = np.empty((n_mel, cap), dtype=np.float32)
        filt = np.ascontiguousarray(self.mf.filters)
        n_len = lib().oracle_log_mel(_ptr(pcm), C.c_int(len(pcm)), _ptr(filt), C.c_int(n_mel), C.c_int(n_fft),
                                     C.c_int(n_threads), _ptr(out), C.c_int(cap))
        assert n_len > 0
        return np.ascontiguousarray(out.reshape(-1)[: n_mel * n_len].reshape(n_mel, n_len))

    def mel_window(self, mel: np.ndarray, seek: int = 0) -> np.ndarray:
        """whisper_encode_qwen2_internal input copy (qwen2-whisper.cpp:2264-2286)."""
        n_ctx = self.m.n_ctx
        win = np.zeros((mel.shape[0], 2 * n_ctx), dtype=np.float32)
        i0, i1 = min(seek, mel.shape[1]), min(seek + 2 * n_ctx, mel.shape[1])
        win[:, : i1 - i0] = mel[:, i0:i1]
        return win

    def encode(self, window: np.ndarray, n_threads: int = 8, dump: bool = False):
        window = np.ascontiguousarray(window, dtype=np.float32)
        D, T = self.m.d, self.m.n_ctx
        out = np.empty((T // 2, D), dtype=np.float32)
        d = None
        dumps = {}
        if dump:
            d = OracleDump()
            for name, _ in OracleDump._fields_:
                a = np.empty((T, 4 * D if name == "gelu" else D), dtype=np.float32)
                dumps[name] = a
                setattr(d, name, _ptr(a))
        rc = lib().oracle_encode(C.byref(self.m), _ptr(window), _ptr(out), C.byref(d) if d is not None else None,
                                 C.c_int(n_threads))
        assert rc == 0
        return (out, dumps) if dump else out


def gemm(wtype: int, w_raw: np.ndarray, x: np.ndarray, n: int, n_threads: int = 8) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    M, K = x.shape
    y = np.empty((M, n), dtype=np.float32)
    w_raw = np.ascontiguousarray(w_raw)
    lib().oracle_gemm(C.c_int(wtype), _ptr(w_raw), _ptr(x), C.c_int(M), C.c_int(n), C.c_int(K), _ptr(y),
                      C.c_int(n_threads))
    return y


def quantize_act(kind: str, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    M, K = x.shape
    if kind == "q8k":
        out = np.empty(M * (K // 256) * 292, dtype=np.uint8)
        f = lib().oracle_quantize_act_q8_K
    else:
        out = np.empty(M * (K // 32) * 34, dtype=np.uint8)
        f = lib().oracle_quantize_act_q8_0
    rs = len(out) // M
    for r in range(M):
        f(_ptr(x[r]), C.c_void_p(out.ctypes.data + r * rs), C.c_int64(K))
    return out
