"""Data-parallel placement of the encoder over ranks: one process per GPU, contiguous clip
ranges per rank, one broadcast of the packed weight blob at start-up, no per-step collective.

The reference has no multi-device path for the encoder (`whisper_backend_init_gpu`,
src/qwen2-whisper.cpp:1217-1279, picks a single device); clips are independent, so ranks never exchange
activations. Backend-agnostic: `nccl` (RCCL over xGMI) on the GPU box, `gloo` on CPU tensors in the tests.
"""
from __future__ import annotations

import hashlib

import torch


def clip_range(rank: int, world_size: int, clips_per_rank: int) -> range:
    """Global clip indices owned by `rank` (weak scaling: every rank holds the same number of clips)."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside world of {world_size}")
    return range(rank * clips_per_rank, (rank + 1) * clips_per_rank)


def split_batch(n_clips: int, world_size: int) -> list[range]:
    """Contiguous near-equal ranges for a fixed global batch (strong-scaling split, ragged tail allowed)."""
    base, extra = divmod(n_clips, world_size)
    out, s = [], 0
    for r in range(world_size):
        n = base + (1 if r < extra else 0)
        out.append(range(s, s + n))
        s += n
    return out


def broadcast_blob(dist, blob_host: bytes | bytearray | None, rank: int, device) -> torch.Tensor:
    """Rank 0 owns the packed weight blob (q2a_pack_model output); every rank returns it as a uint8 tensor on
    `device` after one size broadcast and one data broadcast (RCCL over xGMI on the GPU box)."""
    size_t = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == 0:
        size_t[0] = len(blob_host)
    if dist is not None:
        dist.broadcast(size_t, 0)
    nbytes = int(size_t.item())
    blob = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if rank == 0:   # a bytearray (q2a.pack_model) is viewed, not copied; other buffers are copied once
        src = blob_host if isinstance(blob_host, bytearray) else bytearray(blob_host)
        blob.copy_(torch.frombuffer(src, dtype=torch.uint8))
    if dist is not None:
        dist.broadcast(blob, 0)
    return blob


def blob_digest(blob: torch.Tensor) -> str:
    return hashlib.sha256(blob.cpu().numpy().tobytes()).hexdigest()


def max_over_ranks(dist, value: float, device) -> float:
    """The bench's step time: the slowest rank bounds the job."""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_rank0(dist, out: torch.Tensor, rank: int, world_size: int) -> torch.Tensor | None:
    """Concatenate every rank's [clips][...] output on rank 0 (convenience only; outside the timed region)."""
    if dist is None or world_size == 1:
        return out
    parts = [torch.empty_like(out) for _ in range(world_size)] if rank == 0 else None
    if out.device.type == "cpu":
        dist.gather(out, parts, dst=0)
    else:   # RCCL has no gather in every build: all_gather then drop on non-zero ranks
        parts_all = [torch.empty_like(out) for _ in range(world_size)]
        dist.all_gather(parts_all, out)
        parts = parts_all if rank == 0 else None
    return torch.cat(parts, 0) if rank == 0 else None
