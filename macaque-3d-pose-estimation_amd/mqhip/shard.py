"""Frame sharding across GPUs: one process per GPU, contiguous frame blocks,
one collective -- the all-gather of per-view 2D keypoints before the temporally coupled
step-4 stages.

Everything per frame (crop -> ViT -> decode -> per-frame triangulation) is rank-local;
weights are replicated.  ``gather_keypoints`` moves fixed-size per-rank buffers
([F_block, C, A, J, 3] f32, zero-padded to the largest block) so the collective is a single
RCCL all-gather over xGMI (backend "nccl") -- or gloo in the CPU tests.
"""
from __future__ import annotations

import torch


def frame_block(n_frames: int, world: int, rank: int):
    """Contiguous [start, stop) of rank's frames; the first n_frames % world ranks get one extra."""
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_keypoints(kp_local: torch.Tensor, n_frames: int, world: int, group=None):
    """kp_local (F_local, ...) on this rank -> (n_frames, ...) on every rank, in frame order."""
    import torch.distributed as dist
    block = frame_block(n_frames, world, 0)[1]          # largest block (rank 0 never has fewer)
    shape = (block,) + tuple(kp_local.shape[1:])
    buf = torch.zeros(shape, dtype=kp_local.dtype, device=kp_local.device)
    buf[:kp_local.shape[0]] = kp_local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = []
    for r in range(world):
        s, e = frame_block(n_frames, world, r)
        out.append(parts[r][:e - s])
    return torch.cat(out, dim=0)
