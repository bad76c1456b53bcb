"""One rank of the 2-rank data-parallel rehearsal on ONE GPU (tests/test_gpu_dist.py): the placement code bench.py runs
over RCCL — rank 0 packs the weight blob, one broadcast to every rank (gloo on host tensors here, since both ranks share
device 0), an engine opened on the device copy, this rank's contiguous clip range encoded through libq2a.so. Writes
its outputs to OUTDIR/rank{r}.npy."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))


def main():
    model, clips_path, per_rank, outdir = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    import torch
    import torch.distributed as dist
    import q2a
    from q2a import dist as qd
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    try:
        torch.cuda.set_device(0)
        blob_host = q2a.pack_model(model) if rank == 0 else None
        blob = qd.broadcast_blob(dist, blob_host, rank, "cpu").cuda()
        eng = q2a.Engine(device=0, device_blob=blob.data_ptr(), blob_size=blob.numel())
        r = qd.clip_range(rank, ws, per_rank)
        pcm = np.load(clips_path)[r.start:r.stop]
        out, st = eng.encode_host(list(pcm))
        assert list(st) == [0] * len(r)
        np.save(os.path.join(outdir, f"rank{rank}.npy"), out)
        eng.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
