"""CPU checks of the audio ingestion and the reference-named API surface (no GPU work).

The WAV reader must reproduce examples/common.cpp read_wav (:642-748) exactly: 16 kHz 16-bit PCM only, mono
s16/32768, stereo mixed as (l + r)/65536. Expected values are computed here with numpy from the same int16 data.
"""
import ctypes as C
import os
import subprocess
import wave

import numpy as np
import pytest

from conftest import PKG


@pytest.fixture(scope="module")
def host():
    subprocess.check_call(["make", "-C", PKG, "host", "-j8"], stdout=subprocess.DEVNULL)
    L = C.CDLL(os.path.join(PKG, "lib", "libq2a_host.so"))
    L.q2a_read_wav.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int64),
                               C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.POINTER(C.c_float))]
    L.q2a_wav_free.argtypes = [C.c_void_p]
    return L


def write_wav(path, data16, rate=16000, channels=1, width=2):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(rate)
        w.writeframes(np.ascontiguousarray(data16).tobytes())


def read(host, path, split=False):
    p, l, r = C.POINTER(C.c_float)(), C.POINTER(C.c_float)(), C.POINTER(C.c_float)()
    n = C.c_int64()
    rc = host.q2a_read_wav(str(path).encode(), C.byref(p), C.byref(n), C.byref(l) if split else None,
                           C.byref(r) if split else None)
    if rc != 0:
        return rc, None, None, None
    out = np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0, np.float32)
    host.q2a_wav_free(p)
    lo = ro = None
    if split and l:
        lo = np.ctypeslib.as_array(l, shape=(n.value,)).copy()
        ro = np.ctypeslib.as_array(r, shape=(n.value,)).copy()
        host.q2a_wav_free(l)
        host.q2a_wav_free(r)
    return rc, out, lo, ro


def test_mono_matches_read_wav(host, tmp_path):
    rng = np.random.default_rng(1)
    s16 = rng.integers(-32768, 32768, 48017, dtype=np.int16)
    s16[:4] = [-32768, 32767, 0, -1]
    write_wav(tmp_path / "m.wav", s16)
    rc, x, _, _ = read(host, tmp_path / "m.wav")
    assert rc == 0
    assert np.array_equal(x, s16.astype(np.float32) / np.float32(32768.0))


def test_stereo_mix_and_split(host, tmp_path):
    rng = np.random.default_rng(2)
    s16 = rng.integers(-32768, 32768, (16000, 2), dtype=np.int16)
    write_wav(tmp_path / "s.wav", s16, channels=2)
    rc, x, l, r = read(host, tmp_path / "s.wav", split=True)
    assert rc == 0
    mix = (s16[:, 0].astype(np.int32) + s16[:, 1].astype(np.int32)).astype(np.float32) / np.float32(65536.0)
    assert np.array_equal(x, mix)
    assert np.array_equal(l, s16[:, 0].astype(np.float32) / np.float32(32768.0))
    assert np.array_equal(r, s16[:, 1].astype(np.float32) / np.float32(32768.0))


@pytest.mark.parametrize("rate,channels,width", [(44100, 1, 2), (16000, 3, 2), (16000, 1, 1), (16000, 1, 4)])
def test_rejects_what_read_wav_rejects(host, tmp_path, rate, channels, width):
    n = 1600
    data = np.zeros(n * channels * width, dtype=np.uint8)
    write_wav(tmp_path / "x.wav", data, rate=rate, channels=channels, width=width)
    rc, *_ = read(host, tmp_path / "x.wav")
    assert rc == -2


def test_not_a_wav(host, tmp_path):
    (tmp_path / "bad.wav").write_bytes(b"ID3\x03" + bytes(100))
    assert read(host, tmp_path / "bad.wav")[0] == -1
    assert read(host, tmp_path / "missing.wav")[0] == -1


def test_empty_data_chunk(host, tmp_path):
    write_wav(tmp_path / "e.wav", np.zeros(0, np.int16))
    rc, x, _, _ = read(host, tmp_path / "e.wav")
    assert rc == 0 and x.size == 0


class CtxParams(C.Structure):
    _fields_ = [("use_gpu", C.c_bool), ("flash_attn", C.c_bool), ("gpu_device", C.c_int),
                ("dtw_token_timestamps", C.c_bool), ("dtw_aheads_preset", C.c_int), ("dtw_n_top", C.c_int),
                ("dtw_mem_size", C.c_size_t)]


def test_whisper_api_without_gpu_fails_cleanly():
    """whisper_init_* returns NULL (reference convention) when there is no HIP device or use_gpu is false:
    there is no CPU fallback behind the reference-named API either."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    subprocess.check_call(["make", "-C", PKG, "-j8", "all"], stdout=subprocess.DEVNULL)
    L = C.CDLL(os.path.join(PKG, "lib", "libq2a.so"))
    L.whisper_context_default_params.restype = CtxParams
    L.whisper_init_from_file_with_params.restype = C.c_void_p
    L.whisper_init_from_file_with_params.argtypes = [C.c_char_p, CtxParams]
    L.whisper_lang_id.argtypes = [C.c_char_p]
    cp = L.whisper_context_default_params()
    assert cp.use_gpu and cp.gpu_device == 0 and cp.dtw_n_top == -1
    assert not L.whisper_init_from_file_with_params(b"/nonexistent.bin", cp)
    cp.use_gpu = False
    assert not L.whisper_init_from_file_with_params(b"/nonexistent.bin", cp)
    assert L.whisper_lang_id(b"en") == 0 and L.whisper_lang_id(b"de") == 2 and L.whisper_lang_id(b"xx") == -1
    assert L.whisper_lang_max_id() == 99
