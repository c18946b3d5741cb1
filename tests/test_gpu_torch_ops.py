"""torch.ops.stzs on the GPU: each operator against the CPU oracle's function of
the same row, or -- for the model-bound stage operators -- bit-identical to the engine method it wraps
(whose oracle parity is tests/test_gpu_stages.py).  Tolerances stated per test."""
import pytest
import torch

from refops import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def handle(gpu_device, tiny, tiny_params):
    from stzs import ops
    from stzs.engine import StyleTTSZS
    eng = StyleTTSZS(tiny, tiny_params, device=gpu_device)
    return ops.register(eng), eng


def test_duration_head_exact(gpu_device):
    """bit-exact integer durations vs oracle durations_from_logits (ties within 1e-4 of .5 excluded)."""
    from oracle import stzs_ref as R
    from stzs import ops  # noqa: F401
    g = torch.Generator().manual_seed(4)
    logits = torch.randn(3, 80, 50, generator=g) * 2
    dref, sref = R.durations_from_logits(logits)
    d, s = torch.ops.stzs.duration_head(logits.to(gpu_device))
    tie = (sref - sref.floor() - 0.5).abs() < 1e-4
    assert bool(((d.cpu() == dref) | tie).all())
    assert (s.cpu() - sref).abs().max().item() < 1e-4


def test_length_regulate_exact(gpu_device):
    from oracle import stzs_ref as R
    from stzs import ops  # noqa: F401
    g = torch.Generator().manual_seed(5)
    dur = torch.randint(1, 6, (3, 40), generator=g, dtype=torch.int32)
    dur[:, -1] = 200 - dur[:, :-1].sum(1)  # equal totals (200 frames)
    assert (dur > 0).all()
    idx = torch.ops.stzs.length_regulate(dur.to(gpu_device), 200)
    assert torch.equal(idx.cpu(), R.alignment_index(dur))


def test_cfg_euler_step(gpu_device):
    """vs the oracle's sampler update (oracle/stzs_ref.py sample_style), rel 1e-6."""
    from stzs import ops  # noqa: F401
    g = torch.Generator().manual_seed(6)
    B = 3
    x = torch.randn(B, 50, 256, generator=g)
    D = torch.randn(2 * B, 50, 256, generator=g)
    s0, s1, sc = 3.0, 0.5, 5.0
    Dg = D[B:] + sc * (D[:B] - D[B:])
    ref = x + (s1 - s0) * (x - Dg) / s0
    y = torch.ops.stzs.cfg_euler_step(torch.cat([x, x]).to(gpu_device), D.to(gpu_device), True, sc, s0, s1).cpu()
    assert rel_err(y[:B], ref) < 1e-6 and rel_err(y[B:], ref) < 1e-6


def test_istft_ops_vs_torch_and_stream(gpu_device):
    from stzs import ops  # noqa: F401
    g = torch.Generator().manual_seed(7)
    post = torch.zeros(2, 9601, 24)
    post[:, :, :11] = torch.randn(2, 9601, 11, generator=g) * 0.5
    post[:, :, 11:22] = torch.randn(2, 9601, 11, generator=g) * 2
    full = torch.ops.stzs.istft(post.to(gpu_device), 20, 5)
    spec = (torch.exp(post[:, :, :11]) * torch.exp(1j * torch.sin(post[:, :, 11:22]))).transpose(1, 2)
    ref = torch.istft(spec, 20, hop_length=5, win_length=20, window=torch.hann_window(20))
    assert rel_err(full.cpu(), ref) < 1e-5
    pd = post.to(gpu_device)
    tail = torch.zeros(2, 3, 24, device=gpu_device)
    parts, f0 = [], 0
    for Fc in (1000, 2, 4000, 4599):
        w, tail = torch.ops.stzs.istft_stream(pd[:, f0:f0 + Fc], tail, f0, f0 + Fc == 9601, 20, 5)
        parts.append(w)
        f0 += Fc
    assert torch.equal(torch.cat(parts, 1), full)


def test_stage_ops_match_engine(handle, tiny, tiny_params):
    """sample_style / predict_prosody / decode / synth operators == the engine methods (same kernels)."""
    from oracle import stzs_ref as R
    h, eng = handle
    S = tiny
    g = torch.Generator().manual_seed(8)
    B, T = 2, 12
    tok = torch.randint(1, S.n_symbols, (B, T), generator=g)
    ref = torch.randn(B, S.sr, generator=g) * 0.1
    eps = torch.randn(B, S.L_s, S.code_dim, generator=g)
    dur = torch.tensor([[3, 2] * (T // 2)] * B, dtype=torch.int32)
    dev = eng.device
    out = eng.synth(tok, ref, steps=2, cfg_scale=5.0, noise=eps, durations=dur, seeds=[0, 1])
    wav_e = out["wav"].clone()
    codes_e = out["codes"].clone()
    w = torch.ops.stzs.synth(h, tok.to(dev), ref.to(dev), eps.to(dev), dur.to(dev), 2, 5.0, [0, 1])
    assert torch.equal(w, wav_e)
    hf = R.text_encoder(tiny_params, S, tok).to(dev)
    pr = R.prompt_encoder(tiny_params, S, ref)[0].to(dev)
    c = torch.ops.stzs.sample_style(h, hf, pr, eps.to(dev), 2, 5.0)
    assert torch.isfinite(c).all() and c.shape == codes_e.shape
    d, idx, F0, N = torch.ops.stzs.predict_prosody(h, hf, codes_e, dur.to(dev))
    assert torch.equal(d.cpu(), dur) and idx.shape == (B, 30) and F0.shape == (B, 60)
    asr = hf[torch.arange(B)[:, None], idx.long()]
    wd = torch.ops.stzs.decode(h, asr, F0, N, codes_e, [0, 1])
    wr = R.decode(tiny_params, S, asr.cpu().to(torch.bfloat16).float(), F0.cpu(), N.cpu(), codes_e.cpu(), [0, 1])
    e = rel_err(wd.cpu(), wr)
    print("decode op vs oracle", e)
    assert e < 1e-1
