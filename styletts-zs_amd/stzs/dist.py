"""Multi-GPU plumbing: utterances shard embarrassingly across ranks, one process
per GPU; the ONLY collective is the initial weight broadcast from rank 0 — the whole packed arena
(one contiguous uint8 buffer) in a single RCCL broadcast over xGMI, plus the small hosted front-end
tensors.  No collective runs on the synthesis data path.  The same code runs under gloo on CPU
(tests/test_dist.py)."""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int):
    """contiguous shard [lo, hi) of n_items for `rank` (sizes differ by at most one)."""
    q, r = divmod(n_items, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def broadcast_arena(buf: torch.Tensor, src: int = 0):
    dist.broadcast(buf, src=src)


def broadcast_weights(eng, src: int = 0) -> float:
    """broadcast the engine's weight arena (+ front-end params) from `src`; returns wall ms."""
    if eng.device.type == "cuda":
        torch.cuda.synchronize(eng.device)
    t0 = time.perf_counter()
    broadcast_arena(eng.W.arena.buf, src)
    for k in sorted(eng.fe):
        dist.broadcast(eng.fe[k], src=src)
    if eng.device.type == "cuda":
        torch.cuda.synchronize(eng.device)
    return (time.perf_counter() - t0) * 1e3
