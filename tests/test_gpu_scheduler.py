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
