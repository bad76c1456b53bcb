"""The N>1 data-parallel path through the ENGINE on the GPU (2 ranks sharing device 0, gloo for the one broadcast):
the gathered per-rank outputs must equal the single-process encode of the whole batch bit for bit (SURVEY.md §8e:
clips are independent, the work is deterministic). The reference has no multi-device path for the encoder
(qwen2-whisper.cpp:1217-1279); the design is SURVEY §8e."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("cfg,wt,per_rank", [("tiny", "q4_k", 3), ("full", "q4_k", 2)])
def test_two_rank_engine_shards_equal_single_process(make_model, make_clip, tmp_path, cfg, wt, per_rank):
    import q2a
    model = make_model(cfg, wt)
    pcm = np.stack([make_clip(c) for c in (0, 1)] + [make_clip(200 + i, 480000) for i in range(2 * per_rank - 2)])
    clips_path = str(tmp_path / "clips.npy")
    np.save(clips_path, pcm)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_dist_worker.py"), model, clips_path,
                                       str(per_rank), str(tmp_path)], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0, 0], rcs
    gathered = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(2)])
    eng = q2a.Engine(model, device=0)
    try:
        single, st = eng.encode_host(list(pcm))
    finally:
        eng.close()
    assert gathered.shape == single.shape
    assert np.array_equal(gathered, single)
