"""GPU tests of the one-process multi-GPU path (q2a_group_*): the compact blob goes through RCCL
(ncclCommInitAll + ncclBroadcast) and every device's engine is opened on its received copy; a batch split over the
group equals the single-engine encode bit for bit. On a one-GPU box the group is N = 1 (the communicator, the
broadcast and the per-device thread all execute; the exchange between two devices needs a multi-GPU node)."""
import os
import subprocess

import numpy as np
import pytest
import torch

import q2a
from conftest import PKG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,wt,n", [("tiny", "f16", 5), ("tiny", "q4_k", 5), ("full", "q4_k", 2)])
def test_group_of_one_through_rccl_equals_engine(make_model, make_clip, cfg, wt, n):
    path = make_model(cfg, wt)
    clips = [make_clip(c, 480000) for c in range(n)]
    if n >= 5:
        clips[3] = clips[3][:12000]      # < 1 s: skipped like the reference
        clips[4] = clips[4][:200000]     # ragged length
    e = q2a.Engine(path, device=0)
    ref, st_ref = e.encode_host(clips)
    e.close()
    g = q2a.Group(path, devices=[0])
    assert g.size == 1
    t = g.setup_times()
    assert t["blob_bytes"] == len(q2a.pack_model(path, compact=True))
    out, st = g.encode_host(clips)
    g.close()
    assert list(st) == list(st_ref)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_group_of_every_visible_device(make_model, make_clip):
    path = make_model("tiny", "q4_k")
    g = q2a.Group(path)
    assert g.size == torch.cuda.device_count() == q2a.lib().q2a_device_count()
    clips = [make_clip(c, 480000) for c in range(2 * g.size + 1)]
    out, st = g.encode_host(clips)
    g.close()
    e = q2a.Engine(path, device=0)
    ref, _ = e.encode_host(clips)
    e.close()
    assert list(st) == [q2a.CLIP_ENCODED] * len(clips)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_q2a_main_batch_over_group(make_model, make_clip, tmp_path):
    """bin/q2a_main -b -ng 1: the batch runs through q2a_group (the route it takes by default when more than one
    device is visible) and dumps the same embeddings as the single-engine batch."""
    if os.path.realpath(q2a.LIB_PATH) != os.path.realpath(os.path.join(PKG, "lib", "libq2a.so")):
        pytest.skip("Q2A_LIB_PATH names another build than the one the driver links")
    import wave
    path = make_model("tiny", "f16")
    files = []
    for c in range(3):
        pcm = make_clip(c, 480000)
        s16 = np.clip(np.round(pcm * 32767.0), -32768, 32767).astype(np.int16)
        f = tmp_path / f"c{c}.wav"
        with wave.open(str(f), "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(16000)
            w.writeframes(s16.tobytes())
        files.append(str(f))
    main = os.path.join(PKG, "bin", "q2a_main")
    dumps = []
    for extra in ([], ["-ng", "1"]):
        d = tmp_path / f"emb{len(dumps)}.f32"
        subprocess.run([main, "-m", path, "-b", "-np", "-oemb", str(d)] + extra + files, check=True, timeout=120,
                       capture_output=True)
        dumps.append(np.fromfile(d, dtype=np.uint32))
    assert dumps[0].size == 3 * 750 * 256 and np.array_equal(dumps[0], dumps[1])


@pytest.mark.parametrize("wt", ["f16", "q4_k"])
def test_group_open_with_engine_keeps_one_replica_per_device(make_model, make_clip, wt):
    """q2a_group_open_with (what whisper_full_parallel and q2a_main -b run on): the open engine's own device-layout
    weights are the broadcast's root and its device's group engine shares them, so the device holding the engine
    grows by the group engine's workspace only — not by a second weight replica (the file-based group held
    two) — and the group's outputs equal the engine's bit for bit."""
    path = make_model("full", wt)
    clips = [make_clip(c, 480000) for c in range(3)]
    e = q2a.Engine(path, device=0)
    ref, st_ref = e.encode_host(clips)          # the engine's own workspace exists before the measurement
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(0)
    g = q2a.Group(engine=e, devices=[0])
    assert g.size == 1
    t = g.setup_times()
    assert t["blob_bytes"] == e.info.weight_bytes and t["pack_s"] == 0.0
    out, st = g.encode_host(clips)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(0)
    grew = free0 - free1
    g.close()
    e.close()
    assert list(st) == list(st_ref)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    # the group engine's workspace for 3 clips is ~0.2-0.4 GB; a replica alone would be 1.40 GB (Q4_K) / 1.26 GB (F16)
    assert grew < e.info.weight_bytes * 0.6, (grew, e.info.weight_bytes)


def test_group_open_with_rejects_a_device_list_without_the_engine(make_model):
    path = make_model("tiny", "f16")
    e = q2a.Engine(path, device=0)
    n = torch.cuda.device_count()
    if n > 1:
        with pytest.raises(q2a.Q2AError, match="not in the device list"):
            q2a.Group(engine=e, devices=[1])
    with pytest.raises(q2a.Q2AError, match="listed twice"):
        q2a.Group(engine=e, devices=[0, 0])
    e.close()
