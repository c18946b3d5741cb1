"""Multi-process path without GPUs (gloo, world_size 2 / 4): the weight-arena broadcast and the shared-speaker
prompt-code broadcast (the only data collectives of the design), the timed-loop max reduction and
the utterance sharding."""
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


def _bench_worker(rank, world, port, out):
    """bench.py's world > 1 set-up path (rank_weights -> stzs.dist.broadcast_weights, rank_inputs), up to the
    first GPU call, on CPU under gloo."""
    import sys
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from stzs.dist import arena_digest
    from stzs.spec import SPEC_TINY
    W, ms = bench.rank_weights(SPEC_TINY, rank, world, torch.device("cpu"))
    tok, ref, eps, dur, seeds = bench.rank_inputs(SPEC_TINY, 4, rank)
    out[rank] = dict(digest=arena_digest(W), ms=ms, seeds=seeds, tok=tok.tolist(),
                     eps=hashlib.sha256(eps.numpy().tobytes()).hexdigest(), nframes=int(dur[0].sum()))
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


def test_gloo_bench_rank_setup():
    """bench.py world-2 set-up under gloo: both ranks end with rank 0's arena (byte-identical to packing the
    seed-0 parameters directly), i.e. identical weights for synthesis; their input shards and source-noise
    seeds are disjoint."""
    import sys
    sys.path[:0] = [ROOT, PKG]
    from stzs.dist import arena_digest
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import PackedModel
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_worker, args=(world, port, out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    want = arena_digest(PackedModel(SPEC_TINY, init_params(SPEC_TINY, seed=0), "cpu"))
    assert r0["digest"] == r1["digest"] == want
    assert r1["ms"] >= 0.0
    assert set(r0["seeds"]).isdisjoint(r1["seeds"]) and r0["seeds"] == [0, 1, 2, 3]
    assert r0["tok"] != r1["tok"] and r0["eps"] != r1["eps"]
    assert r0["nframes"] == r1["nframes"]


def _speaker_worker(rank, world, port, out):
    """shared-speaker mode + the timed-loop reduction on CPU tensors: rank 0 holds the prompt's discrete codes
    (here seeded indices standing in for StyleTTSZS.prompt_encode's), every rank receives them byte for byte;
    reduce_max returns the slowest rank's clock on every rank (bench.py's max over ranks)."""
    import sys
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stzs.dist import broadcast_prompt_codes, reduce_max
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    G = S.code_dim // S.vq_group
    src = torch.randint(0, S.vq_size, (1, S.L_s, G), generator=torch.Generator().manual_seed(3),
                        dtype=torch.int32) if rank == 0 else None
    got = broadcast_prompt_codes(src, (1, S.L_s, G), torch.device("cpu"))
    mx = reduce_max([1.0 + rank, 10.0 - rank, 0.25 * (rank + 1)], torch.device("cpu"))
    out[rank] = dict(codes=hashlib.sha256(got.numpy().tobytes()).hexdigest(), shape=tuple(got.shape),
                     dtype=str(got.dtype), mx=mx,
                     want=hashlib.sha256(torch.randint(0, S.vq_size, (1, S.L_s, G),
                                                       generator=torch.Generator().manual_seed(3),
                                                       dtype=torch.int32).numpy().tobytes()).hexdigest())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shared_speaker_codes_and_time_reduction(world):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_speaker_worker, args=(world, port, out), nprocs=world, join=True)
    rs = [out[r] for r in range(world)]
    assert all(r["codes"] == rs[0]["want"] for r in rs)  # byte-identical prompt codes on every rank
    assert all(r["shape"] == rs[0]["shape"] and r["dtype"] == "torch.int32" for r in rs)
    want = [float(world), 10.0, 0.25 * world]
    assert all(r["mx"] == want for r in rs)


def test_broadcast_weights_accepts_engine_like():
    """broadcast_weights takes an engine (anything with .W) or a PackedModel; world 1 (gloo) is a no-op copy."""
    import sys
    sys.path[:0] = [ROOT, PKG]
    from stzs.dist import _packed
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import PackedModel

    W = PackedModel(SPEC_TINY, init_params(SPEC_TINY, seed=0), "cpu")

    class Eng:
        pass
    e = Eng()
    e.W = W
    assert _packed(e) is W and _packed(W) is W


def test_shard_range_partition():
    from stzs.dist import shard_range
    for n in (1, 7, 64, 512, 513):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(h - l for l, h in got) - min(h - l for l, h in got) <= 1


def test_bench_launcher_spawns_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE in the environment starts the 2 rank processes
    itself (bench.launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* per rank, rendezvous on 127.0.0.1) and the
    ranks run bench's world-2 set-up (here --dry-run: gloo, CPU, tiny spec, up to the first GPU call) -- rank 0's line
    says n_gpus 2, every rank holds rank 0's arena, the shards are disjoint; a --gpus / WORLD_SIZE mismatch fails."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["dry_run"] and line["n_gpus"] == 2 and line["weight_broadcast_ms"] > 0
    ranks = line["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert ranks[0]["digest"] == ranks[1]["digest"]
    assert ranks[0]["pid"] != ranks[1]["pid"] and ranks[1]["env"] == dict(LOCAL_RANK="1", MASTER_ADDR="127.0.0.1")
    assert set(ranks[0]["seeds"]).isdisjoint(ranks[1]["seeds"])
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         env=dict(env, WORLD_SIZE="1"), capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
