"""The N>1 data-parallel path on CPU (gloo, world_size 2): the same placement code bench.py runs over RCCL.

Checks: the weight blob broadcast from rank 0 is byte-identical to what every rank packs
itself; clip ranges are disjoint and cover the batch; sharded per-rank encodes, gathered on rank 0, equal the
single-process encode of the whole batch bit for bit (encodes by the CPU oracle here: no GPU in this leg);
the step time is the max over ranks.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG

WS = 2
CLIPS_PER_RANK = 2
N_SAMPLES = 48000   # 3 s clips keep the oracle leg short


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _clips(first, n):
    host = C.CDLL(os.path.join(PKG, "lib", "libq2a_host.so"))
    out = np.empty((n, N_SAMPLES), dtype=np.float32)
    for i in range(n):
        host.q2a_synth_clip(C.c_void_p(out[i].ctypes.data), C.c_int64(N_SAMPLES), C.c_int(first + i))
    return out


def _encode(model_path, pcm):
    import oracle_py
    from q2a import ggmlfile
    o = oracle_py.Oracle(ggmlfile.read(model_path))
    return np.stack([o.encode(o.mel_window(o.log_mel(p)), n_threads=2) for p in pcm])


def _worker(rank, port, model_path, outdir):
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import q2a
    from q2a import dist as qd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        own = q2a.pack_model(model_path)
        blob = qd.broadcast_blob(dist, own if rank == 0 else None, rank, "cpu")
        assert qd.blob_digest(blob) == qd.blob_digest(torch.frombuffer(bytearray(own), dtype=torch.uint8))
        r = qd.clip_range(rank, WS, CLIPS_PER_RANK)
        out = torch.from_numpy(_encode(model_path, _clips(r.start, len(r))))
        full = qd.gather_to_rank0(dist, out, rank, WS)
        t = qd.max_over_ranks(dist, 1.0 + rank, "cpu")
        if rank == 0:
            np.save(os.path.join(outdir, "gathered.npy"), full.numpy())
            with open(os.path.join(outdir, "tmax.txt"), "w") as f:
                f.write(repr(t))
    finally:
        dist.destroy_process_group()


def test_clip_ranges():
    from q2a import dist as qd
    rs = [qd.clip_range(r, 8, 64) for r in range(8)]
    assert [x for r in rs for x in r] == list(range(512))
    with pytest.raises(ValueError):
        qd.clip_range(8, 8, 64)
    sp = qd.split_batch(13, 4)
    assert [len(r) for r in sp] == [4, 3, 3, 3] and [x for r in sp for x in r] == list(range(13))


def test_two_rank_gloo_shards_match_single(make_model, tmp_path):
    model = make_model("tiny", "f16")
    mp.start_processes(_worker, args=(_free_port(), model, str(tmp_path)), nprocs=WS, join=True,
                       start_method="spawn")
    gathered = np.load(tmp_path / "gathered.npy")
    single = _encode(model, _clips(0, WS * CLIPS_PER_RANK))
    assert gathered.shape == single.shape
    assert np.array_equal(gathered, single)
    assert float(open(tmp_path / "tmax.txt").read()) == float(WS)
