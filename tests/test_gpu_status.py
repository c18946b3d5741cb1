"""LSTM exchange timeouts surface on every public path.

A spin that times out leaves wrong h-states; the kernels OR STZS_STATUS_LSTM_TIMEOUT into the engine's status
word.  Forced here with a 1-poll spin limit at batch 8 (v0 dims: 8 workgroups per direction, so some consumer
always waits longer than one poll over the ~300 hand-offs of a synth), every public entry must RAISE:
StyleTTSZS.synth (eager), torch.ops.stzs.synth / predict_prosody, BucketScheduler.synth, and a captured graph's
check() after replay.  A normal call afterwards is clean again.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

B, T = 8, 40


@pytest.fixture(scope="module")
def v0(gpu_device):
    from stzs.engine import StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    eng = StyleTTSZS(S, init_params(S, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(21)
    tok = torch.randint(1, S.n_symbols, (B, T), generator=g).to(torch.int32)
    ref = torch.randn(B, S.sr, generator=g) * 0.1
    eps = torch.randn(B, S.L_s, S.code_dim, generator=g)
    dur = torch.tensor([[3, 2] * (T // 2)] * B, dtype=torch.int32)
    return S, eng, (tok, ref, eps, dur)


def _forced(eng, fn, tries=3):
    """run fn under a 1-poll spin limit until it raises the timeout (a try that happens not to time out must
    then return normally); -> number of tries that raised"""
    raised = 0
    for _ in range(tries):
        eng.lstm_spin_limit = 1
        try:
            fn()
        except RuntimeError as e:
            assert "spin timed out" in str(e), e
            raised += 1
            break
        finally:
            eng.lstm_spin_limit = 0
    return raised


def test_synth_raises(v0):
    S, eng, (tok, ref, eps, dur) = v0
    eng.check_status()
    kw = dict(steps=2, cfg_scale=5.0, noise=eps, durations=dur, seeds=list(range(B)))
    assert _forced(eng, lambda: eng.synth(tok, ref, **kw)) == 1
    out = eng.synth(tok, ref, **kw)  # clean afterwards (the raising check cleared the word)
    assert int(out["status"].item()) == 0


def test_torch_ops_raise(v0):
    from stzs import ops
    S, eng, (tok, ref, eps, dur) = v0
    h = ops.register(eng)
    dev = eng.device
    eng.check_status()
    assert _forced(eng, lambda: torch.ops.stzs.synth(h, tok.to(dev), ref.to(dev), eps.to(dev), dur.to(dev), 2, 5.0,
                                                      list(range(B)))) == 1
    ht = torch.randn(B, T, S.d_txt, device=dev)
    codes = torch.randn(B, S.L_s, S.code_dim, device=dev) * 0.3
    assert _forced(eng, lambda: torch.ops.stzs.predict_prosody(h, ht, codes, dur.to(dev))) == 1
    torch.ops.stzs.predict_prosody(h, ht, codes, dur.to(dev))
    assert eng.check_status() == 0


def test_scheduler_raises(v0):
    from stzs.scheduler import BucketScheduler, Request
    S, eng, (tok, ref, eps, dur) = v0
    reqs = [Request(tokens=tok[i], ref_wav=ref[i], noise=eps[i], seed=i, durations=dur[i]) for i in range(B)]
    sch = BucketScheduler(eng, max_batch=B, steps=2, cfg_scale=5.0)
    eng.check_status()
    assert _forced(eng, lambda: sch.synth(reqs)) == 1
    assert eng.check_status() == 0


def test_captured_graph_check_raises(v0):
    """under capture synth() cannot sync: the CheckedGraph's check() after a replay raises instead."""
    S, eng, (tok, ref, eps, dur) = v0
    dev = eng.device
    tw = eng.twin()
    tok_d, ref_d, eps_d, dur_d = (t.to(dev) for t in (tok, ref, eps, dur))
    nf = int(dur[0].sum())
    fn = lambda: tw.synth(tok_d, ref_d, steps=2, cfg_scale=5.0, noise=eps_d, durations=dur_d, seeds=list(range(B)),
                          n_frames=nf, check=False)
    fn()
    g, _ = tw.capture(fn)
    g.replay()
    assert g.check() == 0
    # a graph captured with the 1-poll limit baked into its LSTM launches
    tw.lstm_spin_limit = 1
    try:
        g1, _ = tw.capture(fn)  # the warm-up call inside capture() runs eager and may time out: clear it
    finally:
        tw.lstm_spin_limit = 0
    tw.status.zero_()
    fired = 0
    for _ in range(3):
        g1.replay()
        try:
            g1.check()
        except RuntimeError as e:
            assert "spin timed out" in str(e)
            fired += 1
            break
    assert fired == 1
    g.replay()
    assert g.check() == 0
