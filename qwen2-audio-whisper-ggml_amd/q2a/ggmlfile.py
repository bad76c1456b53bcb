"""Reader for the reference's unchanged ggml model file (numpy, no execution of file content).

Layout restated from models/convert-pt-to-ggml.py:268-337 and whisper_model_load
(src/qwen2-whisper.cpp:1350-1872).
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

MAGIC = 0x67676D6C
TYPE_F32, TYPE_F16, TYPE_Q4_0, TYPE_Q8_0, TYPE_Q4_K, TYPE_Q8_K = 0, 1, 2, 8, 12, 15
FTYPE_TO_WTYPE = {0: TYPE_F32, 1: TYPE_F16, 2: TYPE_Q4_0, 7: TYPE_Q8_0, 12: TYPE_Q4_K}
HPARAM_NAMES = ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer", "n_mels", "ftype")


def row_size(t: int, n: int) -> int:
    if t == TYPE_F32:
        return 4 * n
    if t == TYPE_F16:
        return 2 * n
    if t == TYPE_Q4_0:
        return (n // 32) * 18
    if t == TYPE_Q8_0:
        return (n // 32) * 34
    if t == TYPE_Q4_K:
        return (n // 256) * 144
    if t == TYPE_Q8_K:
        return (n // 256) * 292
    raise ValueError(f"unsupported ggml type {t}")


@dataclasses.dataclass
class Tensor:
    name: str
    type: int
    ne: tuple          # ggml order: ne[0] fastest
    data: np.ndarray   # raw bytes (uint8) or typed view for F32/F16

    def as_f32(self) -> np.ndarray:
        if self.type == TYPE_F32:
            return self.data.view(np.float32).reshape(tuple(reversed(self.ne)))
        if self.type == TYPE_F16:
            return self.data.view(np.float16).astype(np.float32).reshape(tuple(reversed(self.ne)))
        raise ValueError("quantized tensor has no plain f32 view")


@dataclasses.dataclass
class ModelFile:
    hparams: dict
    qntvr: int
    wtype: int
    filters: np.ndarray  # [n_mel][n_fft]
    tensors: dict

    def t(self, name: str) -> Tensor:
        return self.tensors[name]


def read(path: str) -> ModelFile:
    buf = np.fromfile(path, dtype=np.uint8)
    mv = memoryview(buf)
    off = 0

    def i32():
        nonlocal off
        v = struct.unpack_from("<i", mv, off)[0]
        off += 4
        return v

    magic = struct.unpack_from("<I", mv, 0)[0]
    off = 4
    if magic != MAGIC:
        raise ValueError("invalid model data (bad magic)")
    hp = {k: i32() for k in HPARAM_NAMES}
    qntvr = hp["ftype"] // 1000
    ft = hp["ftype"] % 1000
    if ft not in FTYPE_TO_WTYPE:
        raise ValueError(f"unsupported ftype {ft}")
    n_mel, n_fft = i32(), i32()
    filters = buf[off:off + 4 * n_mel * n_fft].view(np.float32).reshape(n_mel, n_fft)
    off += 4 * n_mel * n_fft
    n_vocab = i32()
    for _ in range(n_vocab):
        ln = struct.unpack_from("<I", mv, off)[0]
        off += 4 + ln
    tensors = {}
    while off < len(buf):
        n_dims, ln, ttype = i32(), i32(), i32()
        ne = tuple(i32() for _ in range(n_dims))
        name = bytes(buf[off:off + ln]).decode()
        off += ln
        nel = int(np.prod(ne))
        nbytes = row_size(ttype, ne[0]) * (nel // ne[0])
        tensors[name] = Tensor(name, ttype, ne, buf[off:off + nbytes])
        off += nbytes
    return ModelFile(hp, qntvr, FTYPE_TO_WTYPE[ft], filters, tensors)
