"""Multi-GPU plumbing: utterances shard embarrassingly across ranks, one process
per GPU; the ONLY collectives are the initial broadcasts from rank 0 -- the whole packed arena
(one contiguous uint8 buffer holding every parameter the engine reads, front end included) in a
single RCCL broadcast over xGMI, and in shared-speaker mode the reference prompt's discrete codes -- plus
one max-reduction of the timings after the timed region.  No collective runs on the synthesis data path.  The same code runs
under gloo on CPU (tests/test_dist.py)."""
from __future__ import annotations

import hashlib
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


def _packed(obj):
    """StyleTTSZS engine or PackedModel -> PackedModel."""
    return obj.W if hasattr(obj, "W") else obj


def broadcast_weights(obj, src: int = 0) -> float:
    """Broadcast the weight arena of an engine (or a PackedModel) from `src`; returns wall ms.

    The arena is the engine's complete parameter state: every packed conv / linear / LSTM / norm table
    and the front-end constants (DFT basis, window, filterbank) live in it (stzs/weights.py:PackedModel),
    and the engine derives nothing else from host parameters.  So after this call all ranks hold
    byte-identical weights, which `arena_digest` checks."""
    W = _packed(obj)
    dev = W.arena.buf.device
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    broadcast_arena(W.arena.buf, src)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3


def broadcast_prompt_codes(idx, shape, device, src: int = 0) -> torch.Tensor:
    """Shared-speaker mode ("plus prompt codes (51 KB per speaker)"): the reference prompt is
    encoded ONCE, on rank `src` (StyleTTSZS.prompt_encode -> its discrete code indices int32 [1, L_s, G]), and
    every rank receives the indices with one broadcast; each rank then synthesizes with prompt_idx= (the
    codebook lookup of the same codes), so no rank repeats the front end.  idx: the indices on `src` (ignored
    elsewhere); -> the indices on every rank (device tensor)."""
    buf = torch.empty(tuple(shape), dtype=torch.int32, device=device)
    if dist.get_rank() == src:
        buf.copy_(idx.reshape(buf.shape))
    dist.broadcast(buf, src=src)
    return buf


def reduce_max(values, device) -> list:
    """max over ranks of a few host floats (the timed region's wall seconds): every rank reports the slowest
    rank's clock.  One small all_reduce, outside every timed region."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def arena_digest(obj) -> str:
    """sha256 of the arena bytes (host copy; for tests / start-up checks, not the data path)."""
    buf = _packed(obj).arena.buf
    return hashlib.sha256(buf.detach().cpu().numpy().tobytes()).hexdigest()
