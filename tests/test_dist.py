"""Multi-process path without GPUs (gloo, world_size 2): the weight-arena broadcast (the ONLY
collective of the design) and the utterance sharding."""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stzs.dist import broadcast_arena, shard_range
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import PackedModel
    W = PackedModel(SPEC_TINY, init_params(SPEC_TINY, seed=rank), "cpu")  # rank 1 starts with other bytes
    before = hashlib.sha256(W.arena.buf.numpy().tobytes()).hexdigest()
    broadcast_arena(W.arena.buf, src=0)
    after = hashlib.sha256(W.arena.buf.numpy().tobytes()).hexdigest()
    lo, hi = shard_range(512, rank, world)
    out[rank] = (before, after, lo, hi)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_weight_broadcast_and_shards():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    (b0, a0, lo0, hi0), (b1, a1, lo1, hi1) = out[0], out[1]
    assert b0 != b1            # different initial bytes
    assert a0 == a1 == b0      # rank 1 now holds rank 0's arena
    assert (lo0, hi0, lo1, hi1) == (0, 256, 256, 512)


def test_shard_range_partition():
    from stzs.dist import shard_range
    for n in (1, 7, 64, 512, 513):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(h - l for l, h in got) - min(h - l for l, h in got) <= 1
