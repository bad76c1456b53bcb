"""GPU tests of the reference-named API (include/q2a_whisper.h) and the drivers built on it.

* bin/q2a_main (our examples/main counterpart) on a WAV file equals the engine's own encode of the same PCM, bit
  for bit, and prints the reference's whisper_print_emb_enc line format;
* the reference's UNCHANGED examples/main/main.cpp compiled against our header (oracle/_ref/main_on_q2a, built by
  oracle/Makefile where /root/reference exists) runs its 100 x whisper_full loop on our library and prints the
  same embeddings;
* long recordings: every 30 s window encoded in one batch equals whisper_full at that offset;
* whisper_full_parallel (declared but undefined in the reference): chunk i equals encoding chunk i alone.
"""
import os
import subprocess
import wave

import numpy as np
import pytest

import oracle_py
from conftest import PKG, ROOT, rel_errors
from q2a import Engine, ggmlfile

pytestmark = pytest.mark.gpu

MAIN = os.path.join(PKG, "bin", "q2a_main")
REF_MAIN = os.path.join(ROOT, "oracle", "_ref", "main_on_q2a")


def to_wav(path, pcm):
    s16 = np.clip(np.round(pcm * 32767.0), -32768, 32767).astype(np.int16)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(s16.tobytes())
    return s16.astype(np.float32) / np.float32(32768.0)   # what read_wav hands to whisper_full


def lines_of(stdout):
    return [ln for ln in stdout.splitlines() if ln.startswith(" ") and len(ln.split()) == 20]


def fmt20(v):
    return "".join(" %.3f" % x for x in v[:20])


@pytest.fixture(scope="module")
def tiny(make_model):
    import q2a
    # the drivers load lib/libq2a.so through their rpath, the Python engine q2a.LIB_PATH: comparing the two is only
    # meaningful when they are the same build (a diag/ A/B run may set Q2A_LIB_PATH)
    if os.path.realpath(q2a.LIB_PATH) != os.path.realpath(os.path.join(PKG, "lib", "libq2a.so")):
        pytest.skip("Q2A_LIB_PATH names another build than the one the drivers link")
    path = make_model("tiny", "f16")
    e = Engine(path)
    yield path, e
    e.close()


def test_q2a_main_matches_engine(tiny, make_clip, tmp_path):
    path, e = tiny
    pcm = to_wav(tmp_path / "c0.wav", make_clip(0))
    out = tmp_path / "emb.f32"
    r = subprocess.run([MAIN, "-m", path, "-np", "-r", "3", "-oemb", str(out), str(tmp_path / "c0.wav")],
                       capture_output=True, text=True, timeout=300, check=True)
    emb = np.fromfile(out, dtype=np.float32).reshape(e.out_shape)
    ref, st = e.encode_host([pcm])
    assert st[0] == 0
    assert np.array_equal(emb, ref[0])
    ls = lines_of(r.stdout)
    assert ls == [fmt20(ref[0].reshape(-1))] * 3


def test_reference_main_unchanged_on_q2a(tiny, make_clip, tmp_path):
    """examples/main/main.cpp of the reference, compiled against include/q2a_whisper.h, linked to libq2a.so."""
    if not os.path.exists(REF_MAIN):
        pytest.skip("oracle/_ref/main_on_q2a not built (needs /root/reference at build time)")
    path, e = tiny
    pcm = to_wav(tmp_path / "c1.wav", make_clip(1))
    r = subprocess.run([REF_MAIN, "-m", path, "-np", "-f", str(tmp_path / "c1.wav")], capture_output=True, text=True,
                       timeout=600, check=True)
    ls = lines_of(r.stdout)
    ref, _ = e.encode_host([pcm])
    assert len(ls) == 100                                    # the reference driver's whisper_full loop
    assert set(ls) == {fmt20(ref[0].reshape(-1))}
    # and the values are the reference's (tolerance of the tiny F16 parity case)
    mf = ggmlfile.read(path)
    o = oracle_py.Oracle(mf)
    want = o.encode(o.mel_window(o.log_mel(pcm)))
    mx, l2 = rel_errors(ref[0], want)
    assert mx < 1e-3 and l2 < 1e-4, (mx, l2)


def test_long_audio_windows(tiny, make_clip, tmp_path):
    path, e = tiny
    pcm = to_wav(tmp_path / "long.wav", make_clip(2, 75 * 16000))   # 75 s: windows at 0, 30, 60 s
    out = tmp_path / "long.f32"
    subprocess.run([MAIN, "-m", path, "-np", "-la", "-oemb", str(out), str(tmp_path / "long.wav")],
                   capture_output=True, text=True, timeout=300, check=True)
    emb = np.fromfile(out, dtype=np.float32).reshape((-1,) + e.out_shape)
    assert emb.shape[0] == 3
    for k in range(3):
        single, st = e.encode_host([pcm], offset_ms=30000 * k)
        assert st[0] == 0
        mx, _ = rel_errors(emb[k], single[0])
        assert mx < 1e-6, (k, mx)
    # window 1 against the CPU oracle: mel of the whole recording, window at frame 3000
    o = oracle_py.Oracle(ggmlfile.read(path))
    want = o.encode(o.mel_window(o.log_mel(pcm), seek=3000))
    mx, l2 = rel_errors(emb[1], want)
    assert mx < 1e-3 and l2 < 1e-4, (mx, l2)


def test_full_parallel_chunks(tiny, make_clip, tmp_path):
    path, e = tiny
    pcm = to_wav(tmp_path / "p.wav", make_clip(3, 40 * 16000))
    out = tmp_path / "p.f32"
    r = subprocess.run([MAIN, "-m", path, "-np", "-p", "2", "-oemb", str(out), str(tmp_path / "p.wav")],
                       capture_output=True, text=True, timeout=300, check=True)
    emb = np.fromfile(out, dtype=np.float32).reshape((-1,) + e.out_shape)
    assert emb.shape[0] == 2 and len(lines_of(r.stdout)) == 2
    half = len(pcm) // 2
    for k, chunk in enumerate([pcm[:half], pcm[half:]]):
        single, st = e.encode_host([chunk])
        mx, _ = rel_errors(emb[k], single[0])
        assert mx < 1e-6, (k, mx)
