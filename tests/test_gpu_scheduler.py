"""Length-bucketing scheduler (stzs/scheduler.py): mixed token counts, reference
lengths and predicted frame counts; every waveform must equal the same request synthesized alone (the
kernels compute rows independently, and the padding tokens of a regrouped batch carry duration 0).
Tolerance: bit-identical expected; asserted max-abs <= 1e-6 of max|ref|."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bucket_scheduler_matches_single_requests(gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    from stzs.scheduler import BucketScheduler, Request
    S = tiny
    eng = StyleTTSZS(S, tiny_params, device=gpu_device)
    g = torch.Generator().manual_seed(21)
    reqs = []
    for k, (T, nref, forced) in enumerate([(8, S.sr, None), (12, S.sr, None), (12, S.sr, None),
                                           (8, S.sr + S.sr // 2, None), (10, S.sr, [4] * 10), (8, S.sr, [5] * 8),
                                           (6, S.sr, None)]):
        reqs.append(Request(tokens=torch.randint(1, S.n_symbols, (T,), generator=g),
                            ref_wav=torch.randn(nref, generator=g) * 0.1,
                            noise=torch.randn(S.L_s, S.code_dim, generator=g), seed=100 + k,
                            durations=torch.tensor(forced, dtype=torch.int32) if forced else None))
    sch = BucketScheduler(eng, max_batch=4, steps=2, cfg_scale=5.0)
    outs = sch.synth(reqs)
    print("scheduler", sch.stats)
    assert 40 in sch.stats["frame_buckets"]  # the two forced requests (T_txt 10 and 8) share a bucket
    for r, w in zip(reqs, outs):
        one = eng.synth(r.tokens[None], r.ref_wav[None], steps=2, cfg_scale=5.0, noise=r.noise[None],
                        durations=r.durations[None] if r.durations is not None else None, seeds=[r.seed])["wav"][0]
        assert w.shape == one.shape
        err = ((w - one).abs().max() / one.abs().max()).item()
        print("len", w.shape[0], "equal" if torch.equal(w, one) else f"max-rel {err:.2e}")
        assert err <= 1e-6


def test_buffer_cache_plateaus_over_lengths(gpu_device, tiny, tiny_params):
    """the buffer cache is keyed by (name, dtype) and reused by capacity, so a stream of distinct
    request shapes no larger than one already seen allocates nothing; and a smaller shape served from a larger
    storage (padding re-zeroed on the shape change) is bit-identical to a fresh engine's result."""
    from stzs.engine import StyleTTSZS
    S = tiny
    eng = StyleTTSZS(S, tiny_params, device=gpu_device)
    g = torch.Generator().manual_seed(5)

    def req(B, T, nref, dur):
        return (torch.randint(1, S.n_symbols, (B, T), generator=g), torch.randn(B, nref, generator=g) * 0.1,
                torch.randn(B, S.L_s, S.code_dim, generator=g), torch.full((B, T), dur, dtype=torch.int32))

    def run(e, r):
        tok, ref, eps, dur = r
        return e.synth(tok, ref, steps=2, cfg_scale=5.0, noise=eps, durations=dur,
                       seeds=list(range(tok.shape[0])))["wav"]

    run(eng, req(4, 16, 2 * S.sr, 6))  # the largest shape first
    torch.cuda.synchronize()
    held, alloc = eng.buffer_bytes(), torch.cuda.memory_allocated(gpu_device)
    shapes = [(1, 5, S.sr, 2), (3, 9, S.sr + 123, 4), (2, 16, S.sr, 3), (4, 7, 2 * S.sr, 6), (1, 11, S.sr // 2 + 7, 5),
              (2, 13, S.sr, 1), (3, 6, S.sr, 5), (4, 15, S.sr + S.sr // 3, 2), (1, 16, 2 * S.sr, 6), (2, 4, S.sr, 3)]
    last = None
    for sh in shapes:
        last = (sh, req(*sh), run(eng, req(*sh)))
    torch.cuda.synchronize()
    print(f"buffer cache {held / 2**20:.1f} MiB -> {eng.buffer_bytes() / 2**20:.1f} MiB, allocated "
          f"{alloc / 2**20:.1f} -> {torch.cuda.memory_allocated(gpu_device) / 2**20:.1f} MiB")
    assert eng.buffer_bytes() == held
    assert torch.cuda.memory_allocated(gpu_device) <= alloc + (1 << 20)
    # reuse of a larger storage at a new shape: same result as a fresh engine
    sh, r, _ = last
    w_reused = run(eng, r)
    w_fresh = run(StyleTTSZS(S, tiny_params, device=gpu_device), r)
    assert torch.equal(w_reused, w_fresh)
