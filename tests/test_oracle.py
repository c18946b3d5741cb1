"""Pinning the CPU oracle (oracle/stzs_ref.py): each building block against an INDEPENDENT restatement,
then the whole oracle against the committed golden fixtures (tests/golden/, make_golden.py).
Parity with upstream StyleTTS-ZS is unpinned: upstream publishes no code or vectors."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT

from oracle import stzs_ref as R


def test_bilstm_vs_manual_recurrence(tiny, tiny_params):
    P = tiny_params
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 7, tiny.pr_in, generator=g)
    y = R.bilstm(x, P, "pr.de0")
    H = tiny.lstm_h

    def run(sfx, seq):
        Wi, Wh = P["pr.de0.w_ih" + sfx], P["pr.de0.w_hh" + sfx]
        b = P["pr.de0.b_ih" + sfx] + P["pr.de0.b_hh" + sfx]
        h = torch.zeros(2, H)
        c = torch.zeros(2, H)
        out = []
        for t in seq:
            z = x[:, t] @ Wi.t() + h @ Wh.t() + b
            i, f, gg, o = z.chunk(4, -1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            out.append(h)
        return out

    fw = torch.stack(run("", range(7)), 1)
    bw = torch.stack(run("_rev", range(6, -1, -1))[::-1], 1)
    torch.testing.assert_close(y, torch.cat([fw, bw], -1), atol=1e-5, rtol=1e-5)


def test_istft_vs_manual_overlap_add():
    g = torch.Generator().manual_seed(1)
    Tf = 41
    post = torch.randn(1, 22, Tf, generator=g) * 0.5
    spec = torch.exp(post[:, :11]) * torch.exp(1j * torch.sin(post[:, 11:]))
    ref = torch.istft(spec, 20, hop_length=5, win_length=20, window=torch.hann_window(20))
    X = spec[0].numpy()
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(20) / 20)
    frames = np.fft.irfft(X.T, n=20) * w
    N = 5 * (Tf - 1) + 20
    y = np.zeros(N)
    env = np.zeros(N)
    for f in range(Tf):
        y[5 * f:5 * f + 20] += frames[f]
        env[5 * f:5 * f + 20] += w * w
    out = (y / np.where(env > 1e-11, env, 1))[10:10 + 5 * (Tf - 1)]
    np.testing.assert_allclose(ref[0].numpy(), out, atol=1e-5, rtol=1e-4)


def test_stft_features_vs_manual_dft(tiny, tiny_params):
    F0 = torch.full((1, 6), 180.0)
    har, src = R.source_features(tiny_params, tiny, F0, [3])
    s = np.pad(src[0].numpy().astype(np.float64), (10, 10), mode="reflect")
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(20) / 20)
    n = np.arange(20)
    for f in (0, 7, 100, har.shape[-1] - 1):
        fr = s[5 * f:5 * f + 20] * w
        X = np.array([np.sum(fr * np.exp(-2j * np.pi * k * n / 20)) for k in range(11)])
        np.testing.assert_allclose(har[0, :11, f].numpy(), X.real, atol=1e-5)
        np.testing.assert_allclose(har[0, 11:, f].numpy(), X.imag, atol=1e-5)


def test_harmonic_source_phase_and_noise(tiny, tiny_params):
    """voiced frames follow the closed-form sine phase; unvoiced frames are counter-RNG noise only."""
    S = tiny
    F0 = torch.tensor([[200.0] * 4 + [0.0] * 4])
    src = R.harmonic_source(tiny_params, S, F0, [9])
    assert src.shape == (1, 8 * S.hop)
    assert torch.isfinite(src).all() and src.abs().max() <= 1.0
    # frame-rate phase prefix wraps to [0, 1)
    pre = R.frame_phase_prefix(S, F0)
    assert (pre >= 0).all() and (pre < 1).all()
    np.testing.assert_allclose(pre[0, 0, 1], (S.hop * 200.0 / S.sr) % 1.0, atol=1e-12)
    # deterministic in the seed, different across seeds
    assert torch.equal(src, R.harmonic_source(tiny_params, S, F0, [9]))
    assert not torch.equal(src, R.harmonic_source(tiny_params, S, F0, [10]))


def test_counter_normal_statistics():
    z = R.counter_normal(R.stream_key(1, 2), np.arange(200000))
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1) < 0.01


def test_oracle_front_end_restatement_matches_product_front_end(tiny):
    """the oracle restates the front-end arithmetic instead of importing it: its counter RNG equals the
    product's (stzs.frontend, mirrored in csrc/source.hip) bit for bit, its filterbank / log-mel to fp32."""
    from stzs import frontend as FE
    for seed, stream in ((0, 0), (7, 3), (2 ** 31 + 5, 8), (0xFFFFFFFF, 1)):
        k_o, k_p = R.stream_key(seed, stream), FE.stream_key(seed, stream)
        assert int(k_o) == int(k_p)
        idx = np.arange(0, 5000, 7)
        assert np.array_equal(R.counter_normal(k_o, idx), FE.counter_normal(k_p, idx))
        assert R.initial_phase(k_o) == FE.initial_phase(k_p)
    fb_o = R.htk_mel_filterbank(80, 2048, 24000)
    fb_p = FE.mel_filterbank(80, 2048, 24000)
    torch.testing.assert_close(fb_o, fb_p, atol=1e-6, rtol=0)
    wav = torch.randn(2, 24000, generator=torch.Generator().manual_seed(5)) * 0.1
    from stzs.spec import SPEC_V0
    torch.testing.assert_close(R.log_mel(wav, SPEC_V0), FE.log_mel(wav, SPEC_V0), atol=2e-4, rtol=0)


def test_vq_matches_bruteforce_and_roundtrips(tiny, tiny_params):
    """discrete style codes: indices = argmin of the fp64 distances wherever the fp32 margin is clear, the
    dequantised rows are codebook rows, lookup(idx) == quantised codes, codebook rows are fixed points."""
    S, P = tiny, tiny_params
    z = torch.randn(3, S.L_s, S.code_dim, generator=torch.Generator().manual_seed(21)) * 0.2
    idx, q, margin = R.quantize_codes(P, S, z)
    G = S.code_dim // S.vq_group
    assert idx.shape == (3, S.L_s, G) and idx.dtype == torch.int32 and (margin >= 0).all()
    cb = P["pe.vq"].double()
    d = ((z.double().reshape(-1, G, 1, S.vq_group) - cb[None]) ** 2).sum(-1)
    clear = margin.reshape(-1, G) > 1e-5
    assert clear.float().mean() > 0.95
    assert torch.equal(d.argmin(-1)[clear], idx.reshape(-1, G).long()[clear])
    torch.testing.assert_close(R.lookup_codes(P, S, idx), q, atol=0, rtol=0)
    i2, q2, _ = R.quantize_codes(P, S, q)
    assert torch.equal(i2, idx) and torch.equal(q2, q)


def test_text_encoder_ends_in_bilstm(tiny, tiny_params):
    """StyleTTS2 TextEncoder: the CNN stack's output goes through the text BiLSTM (row f2)."""
    S, P = tiny, tiny_params
    tok = torch.randint(1, S.n_symbols, (2, 9), generator=torch.Generator().manual_seed(4))
    h = R.text_encoder(P, S, tok)
    x = P["te.emb"][tok.long()].transpose(1, 2)
    for i in range(S.te_layers):
        x = F.conv1d(x, P[f"te.conv{i}.w"], P[f"te.conv{i}.b"], padding=S.te_kernel // 2)
        x = F.leaky_relu(F.layer_norm(x.transpose(1, 2), (S.d_txt,), P[f"te.ln{i}.g"], P[f"te.ln{i}.b"]), 0.2)
        x = x.transpose(1, 2)
    torch.testing.assert_close(h, R.bilstm(x.transpose(1, 2), P, "te.lstm"), atol=0, rtol=0)
    assert h.shape == (2, 9, S.d_txt)


def test_convtranspose_polyphase_equivalence():
    """the ConvTranspose1d(k=2s) polyphase restatement used by the HIP kernel == F.conv_transpose1d"""
    g = torch.Generator().manual_seed(2)
    for s in (10, 6):
        Ci, Co, T = 5, 4, 9
        w = torch.randn(Ci, Co, 2 * s, generator=g)
        x = torch.randn(1, Ci, T, generator=g)
        ref = F.conv_transpose1d(x, w, stride=s, padding=s // 2)
        out = torch.zeros(Co, T * s)
        xp = F.pad(x[0], (1, 1))
        for q in range(T + 1):
            for p in range(s):
                t = q * s + p - s // 2
                if 0 <= t < T * s:
                    out[:, t] = w[:, :, p + s].t() @ xp[:, q] + w[:, :, p].t() @ xp[:, q + 1]
        torch.testing.assert_close(out, ref[0], atol=1e-5, rtol=1e-5)


def test_style_interpolation_matches_formula(tiny):
    codes = torch.randn(2, tiny.L_s, tiny.code_dim, generator=torch.Generator().manual_seed(11))
    T = 13
    st = R.style_per_token(tiny, codes, T)
    sp = codes[:, :, tiny.style_ac:]
    for t in range(T):
        src = max((t + 0.5) * tiny.L_s / T - 0.5, 0.0)
        i0 = int(src)
        i1 = min(i0 + 1, tiny.L_s - 1)
        l1 = src - i0
        torch.testing.assert_close(st[:, t], (1 - l1) * sp[:, i0] + l1 * sp[:, i1], atol=1e-6, rtol=1e-5)


def test_durations_and_alignment():
    logits = torch.tensor([[[10.0] * 3 + [-10.0] * 5, [-10.0] * 8]])
    dur, s = R.durations_from_logits(logits)
    assert dur.tolist() == [[3, 1]]  # clamp >= 1
    idx = R.alignment_index(torch.tensor([[2, 0, 3]], dtype=torch.int32))
    assert idx.tolist() == [[0, 0, 2, 2, 2]]
    d = torch.randint(0, 3, (3, 17), dtype=torch.int32, generator=torch.Generator().manual_seed(17))
    d[:, -1] = 40 - d[:, :-1].sum(1).int()  # equal totals (40); the first 16 sum to <= 32, so last >= 8
    idx = R.alignment_index(d)
    for b in range(3):
        assert idx[b].tolist() == torch.repeat_interleave(torch.arange(17), d[b].long()).tolist()


def test_sigma_schedule_and_sampler_limits(tiny, tiny_params):
    S = tiny
    sig = R.sigma_schedule(S, 10)
    assert len(sig) == 11 and sig[-1] == 0.0
    assert abs(sig[0] - S.sigma_max) < 1e-12 and abs(sig[9] - S.sigma_min) < 1e-12
    assert all(a > b for a, b in zip(sig[:-1], sig[1:]))
    assert R.sigma_schedule(S, 1) == [S.sigma_max, 0.0]
    assert R.sigma_schedule(S, 2) == [S.sigma_max, 0.5, 0.0]
    g = torch.Generator().manual_seed(3)
    h = torch.randn(1, 6, S.d_txt, generator=g)
    pr = torch.randn(1, S.L_s, S.code_dim, generator=g)
    eps = torch.randn(1, S.L_s, S.code_dim, generator=g)
    # 1-step Euler to sigma 0 returns the denoiser output D(x0, sigma_max) exactly
    kv, pool = R.denoiser_context(tiny_params, S, h, pr, cfg=False)
    D = R.denoiser(tiny_params, S, eps * S.sigma_max, S.sigma_max, kv, pool)
    torch.testing.assert_close(R.sample_style(tiny_params, S, h, pr, eps, 1, 1.0), D, atol=1e-6, rtol=1e-5)
    # CFG scale 1 == conditional only
    torch.testing.assert_close(R.sample_style(tiny_params, S, h, pr, eps, 2, 1.0),
                               R.sample_style(tiny_params, S, h, pr, eps, 2, 1.0 + 0.0), atol=0, rtol=0)


def test_adain_is_instance_norm_affine(tiny, tiny_params):
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 64, 30, generator=g) * 3 + 1
    s = torch.randn(2, tiny.style_pr, generator=g)
    y = R.adain(x, s, tiny_params, "pr.f00.norm1")
    h = s @ tiny_params["pr.f00.norm1.w"].t() + tiny_params["pr.f00.norm1.b"]
    g, b = h[:, :64], h[:, 64:]
    m = x.mean(-1, keepdim=True)
    v = x.var(-1, unbiased=False, keepdim=True)
    torch.testing.assert_close(y, (1 + g[..., None]) * (x - m) / torch.sqrt(v + 1e-5) + b[..., None], atol=1e-5,
                               rtol=1e-5)


def _load(name):
    from safetensors import safe_open
    p = os.path.join(ROOT, "tests", "golden", name)
    with safe_open(p, "pt") as f:
        return {k: f.get_tensor(k) for k in f.keys()}, f.metadata()


def test_golden_tiny_reproduces(tiny, tiny_params):
    """oracle drift guard: the tiny-spec synth (forced and predicted durations) equals the fixture."""
    from stzs.params import param_checksum
    t, meta = _load("tiny_synth.safetensors")
    assert meta["param_checksum"] == param_checksum(tiny_params)
    o = R.synth(tiny_params, tiny, t["tok"], t["ref"], 2, 5.0, t["eps"], t["dur"], seeds=[0, 1])
    assert torch.equal(o["prompt_idx"], t["prompt_idx"])
    for k in ("h_txt", "prompt", "codes", "F0", "N", "wav"):
        torch.testing.assert_close(o[k], t[k], atol=2e-5, rtol=1e-4, msg=k)
    pr = R.predict_prosody(tiny_params, tiny, o["h_txt"], o["codes"], None)
    assert torch.equal(pr["dur_pred"], t["dur_pred"])


@pytest.mark.slow
def test_golden_v0_reproduces():
    from stzs.params import init_params, param_checksum
    from stzs.spec import SPEC_V0
    t, meta = _load("v0_synth_1s.safetensors")
    P = init_params(SPEC_V0, 0)
    assert meta["param_checksum"] == param_checksum(P)
    o = R.synth(P, SPEC_V0, t["tok"], t["ref"], 1, 1.0, t["eps"], t["dur"], seeds=[5])
    assert torch.equal(o["prompt_idx"], t["prompt_idx"])
    for k in ("codes", "F0", "N", "wav"):
        torch.testing.assert_close(o[k], t[k], atol=1e-4, rtol=1e-3, msg=k)


def test_decode_chunked_reduces_to_decode(tiny, tiny_params):
    """the chunked decoder's restatement: with a halo covering the whole utterance every window IS the utterance,
    so the chunk frames concatenate to exactly the whole-utterance conv_post / waveform; with a short halo the
    chunk-local statistics make it a different (but finite, same-length) function."""
    from oracle import stzs_ref as R
    S, P = tiny, tiny_params
    g = torch.Generator().manual_seed(0)
    B, T40 = 2, 23
    asr = torch.randn(B, T40, S.d_txt, generator=g)
    F0 = 100 + 100 * torch.rand(B, 2 * T40, generator=g)
    N = torch.randn(B, 2 * T40, generator=g)
    codes = torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3
    full = R.decode(P, S, asr, F0, N, codes, [3, 4])
    wc, posts = R.decode_chunked(P, S, asr, F0, N, codes, [3, 4], chunk=8, halo=T40)
    assert torch.equal(wc, full)
    assert [p.shape[2] for p in posts] == [8 * 120, 8 * 120, 7 * 120 + 1]
    w3, _ = R.decode_chunked(P, S, asr, F0, N, codes, [3, 4], chunk=8, halo=3)
    assert w3.shape == full.shape and torch.isfinite(w3).all()
    assert ((w3 - full).norm() / full.norm()).item() > 1e-3
    # fixed-length windows (W = chunk + 2 halo = 14), the first and last shifted inward
    assert R.chunk_windows(23, 8, 3) == [(0, 8, 0, 14), (8, 16, 5, 19), (16, 23, 9, 23)]


def test_fp64_oracle_path(tiny, tiny_params):
    """the float64 oracle (tools/oracle_floor.py, DESIGN.md §3 "the oracle's own floor"): fp64 parameters / codes run every
    op in fp64 -- the BiLSTMs, the iSTFT window, the harmonic source (harmonic_source64: the same phase prefix, counter
    streams and formula as the fp32 source, no fp32 rounding) -- and land within fp32 rounding of the fp32 oracle."""
    S, P = tiny, tiny_params
    g = torch.Generator().manual_seed(5)
    F0 = 100 + 150 * torch.rand(1, 40, generator=g)
    F0[:, :4] = 0.0
    s32 = R.harmonic_source(P, S, F0, [3])
    s64 = R.harmonic_source(P, S, F0.double(), [3])
    assert s32.dtype == torch.float32 and s64.dtype == torch.float64
    assert (s64 - s32.double()).abs().max().item() < 1e-5
    T = 12
    tok = torch.randint(1, S.n_symbols, (1, T), generator=g)
    codes = torch.randn(1, S.L_s, S.code_dim, generator=g) * 0.3
    dur = torch.tensor([[3, 2] * (T // 2)], dtype=torch.int32)
    P64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in P.items()}
    with torch.no_grad():
        out = {}
        for name, PP, cc in (("32", P, codes), ("64", P64, codes.double())):
            h = R.text_encoder(PP, S, tok)
            pro = R.predict_prosody(PP, S, h, cc, dur)
            out[name] = (R.decode(PP, S, pro["asr"], pro["F0"], pro["N"], cc, [3]), pro["F0"])
    w32, f32 = out["32"]
    w64, f64 = out["64"]
    assert w64.dtype == torch.float64 and f64.dtype == torch.float64
    assert ((w64 - w32.double()).norm() / w64.norm()).item() < 1e-3
    assert ((f64 - f32.double()).norm() / f64.norm()).item() < 1e-5
