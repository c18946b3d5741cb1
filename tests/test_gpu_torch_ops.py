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


# ---------------------------------------------------------------- per-row operators vs the oracle (tiny spec)
def _bf(x):
    return x.to(torch.bfloat16).float()


def test_op_bilstm(handle, tiny, tiny_params):
    """stzs::bilstm vs oracle bilstm (nn.LSTM); bf16 input / output rows: rel-L2 <= 1e-2."""
    from oracle import stzs_ref as R
    h, eng = handle
    g = torch.Generator().manual_seed(41)
    for name, cin in (("te.lstm", tiny.d_txt), ("pr.de1", tiny.pr_in), ("pr.shared", tiny.pr_in)):
        x = _bf(torch.randn(3, 17, cin, generator=g))
        y = torch.ops.stzs.bilstm(h, name, x.to(eng.device)).cpu()
        e = rel_err(y, R.bilstm(x, tiny_params, name))
        print("bilstm", name, e)
        assert e < 1e-2


def test_op_denoiser_fwd(handle, tiny, tiny_params):
    """stzs::denoiser_fwd (one NFE, CFG rows) vs oracle denoiser: rel-L2 <= 8e-3 (the 1-NFE stage bound)."""
    from oracle import stzs_ref as R
    h, eng = handle
    S, P = tiny, tiny_params
    g = torch.Generator().manual_seed(42)
    ht = _bf(torch.randn(2, 11, S.d_txt, generator=g))
    prompt = torch.randn(2, S.L_s, S.code_dim, generator=g) * 0.2
    x = torch.randn(4, S.L_s, S.code_dim, generator=g) * 2.0
    for sigma in (3.0, 0.5):
        kv, pool = R.denoiser_context(P, S, ht, prompt, True)
        want = R.denoiser(P, S, x, sigma, kv, pool)
        got = torch.ops.stzs.denoiser_fwd(h, ht.to(eng.device), prompt.to(eng.device), x.to(eng.device), sigma,
                                          True).cpu()
        e = rel_err(got, want)
        print("denoiser_fwd sigma", sigma, e)
        assert e < 8e-3


def test_op_f0n_predictor(handle, tiny, tiny_params):
    """stzs::f0n_predictor vs oracle f0n_predictor: F0 rel-L2 <= 1e-4, N <= 3e-2 (the stage bounds)."""
    from oracle import stzs_ref as R
    h, eng = handle
    S, P = tiny, tiny_params
    g = torch.Generator().manual_seed(43)
    en = _bf(torch.randn(2, 30, S.pr_in, generator=g))
    codes = torch.randn(2, S.L_s, S.code_dim, generator=g) * 0.3
    F0r, Nr = R.f0n_predictor(P, S, en, codes)
    F0, N = torch.ops.stzs.f0n_predictor(h, en.to(eng.device), codes.to(eng.device))
    eF, eN = rel_err(F0.cpu(), F0r), rel_err(N.cpu(), Nr)
    print("f0n_predictor", eF, eN)
    assert eF < 1e-4 and eN < 3e-2


@pytest.fixture(scope="module")
def dec_inputs(tiny):
    S = tiny
    g = torch.Generator().manual_seed(44)
    T40 = 20
    asr = _bf(torch.randn(2, T40, S.d_txt, generator=g))
    F0 = 100 + 150 * torch.rand(2, 2 * T40, generator=g)
    F0[:, :3] = 0.0
    N = torch.randn(2, 2 * T40, generator=g)
    codes = torch.randn(2, S.L_s, S.code_dim, generator=g) * 0.3
    return asr, F0, N, codes


def test_op_decoder_pre(handle, tiny, tiny_params, dec_inputs):
    """stzs::decoder_pre vs oracle decoder_pre (5 AdaIN blocks, bf16 activations): rel-L2 <= 3e-2."""
    from oracle import stzs_ref as R
    h, eng = handle
    asr, F0, N, codes = dec_inputs
    want = R.decoder_pre(tiny_params, tiny, asr, F0, N, codes).transpose(1, 2)
    d = eng.device
    got = torch.ops.stzs.decoder_pre(h, asr.to(d), F0.to(d), N.to(d), codes.to(d)).cpu()
    e = rel_err(got, want)
    print("decoder_pre", e)
    assert e < 3e-2


def test_op_sine_gen(handle, tiny, tiny_params, dec_inputs):
    """stzs::sine_gen vs oracle source_features (STFT of the harmonic source; bf16 storage): rel-L2 <= 1e-2."""
    from oracle import stzs_ref as R
    h, eng = handle
    _, F0, _, _ = dec_inputs
    want, _ = R.source_features(tiny_params, tiny, F0, [3, 4])
    got = torch.ops.stzs.sine_gen(h, F0.to(eng.device), [3, 4]).cpu()
    e = rel_err(got, want.transpose(1, 2))
    print("sine_gen", e)
    assert e < 1e-2


@pytest.mark.parametrize("stage", [0, 1])
def test_op_conv_transpose_up_and_mrf(handle, tiny, tiny_params, dec_inputs, stage):
    """stzs::conv_transpose_up vs oracle upsample_stage (rel-L2 <= 2e-2) and stzs::mrf_resblock vs oracle
    mrf_stage (rel-L2 <= 3e-2), on bf16-rounded inputs."""
    from oracle import stzs_ref as R
    h, eng = handle
    S, P = tiny, tiny_params
    _, F0, _, codes = dec_inputs
    d = eng.device
    g = torch.Generator().manual_seed(45 + stage)
    cin = S.dec_out if stage == 0 else S.gen_ch[0]
    T = F0.shape[1] * (1 if stage == 0 else S.up_rates[0])
    x = _bf(torch.randn(2, T, cin, generator=g))
    har, _ = R.source_features(P, S, F0, [3, 4])
    har = _bf(har)
    want = R.upsample_stage(P, S, x.transpose(1, 2), har, stage).transpose(1, 2)
    got = torch.ops.stzs.conv_transpose_up(h, x.to(d), har.transpose(1, 2).contiguous().to(d), stage).cpu()
    e = rel_err(got, want)
    xm = _bf(want)
    s = R.decoder_style(S, codes)
    want_m = R.mrf_stage(P, S, xm.transpose(1, 2), s, stage).transpose(1, 2)
    got_m = torch.ops.stzs.mrf_resblock(h, xm.to(d), codes.to(d), stage).cpu()
    em = rel_err(got_m, want_m)
    print("conv_transpose_up", stage, e, "mrf_resblock", em)
    assert e < 2e-2 and em < 3e-2


def test_op_conv_post_istft(handle, tiny, tiny_params):
    """stzs::conv_post_istft vs oracle conv_post_istft: rel-L2 <= 2e-2 (bf16 input rows, fp32 conv output)."""
    from oracle import stzs_ref as R
    h, eng = handle
    g = torch.Generator().manual_seed(47)
    x = _bf(torch.randn(2, 481, tiny.gen_ch[-1], generator=g) * 0.5)
    want, _ = R.conv_post_istft(tiny_params, tiny, x.transpose(1, 2))
    got = torch.ops.stzs.conv_post_istft(h, x.to(eng.device)).cpu()
    e = rel_err(got, want)
    print("conv_post_istft", e)
    assert e < 2e-2


def test_ops_nct_layout(handle, tiny, tiny_params, dec_inputs):
    """the per-row operators with nct=True (torch Conv1d [B, C, T] tensors at the boundary): each is
    the channels-last call with its operands and result transposed, bit for bit (the transpose is folded into the
    operator's own buffer copies), and the oracle's NCT functions are matched directly."""
    from oracle import stzs_ref as R
    h, eng = handle
    S, P = tiny, tiny_params
    asr, F0, N, codes = dec_inputs
    d = eng.device
    asr_d, F0_d, N_d, c_d = asr.to(d), F0.to(d), N.to(d), codes.to(d)
    a = torch.ops.stzs.decoder_pre(h, asr_d, F0_d, N_d, c_d)
    b = torch.ops.stzs.decoder_pre(h, asr_d.transpose(1, 2).contiguous(), F0_d, N_d, c_d, nct=True)
    assert b.shape == (2, S.dec_out, 2 * asr.shape[1]) and torch.equal(b, a.transpose(1, 2))
    hs = torch.ops.stzs.sine_gen(h, F0_d, [3, 4])
    hn = torch.ops.stzs.sine_gen(h, F0_d, [3, 4], nct=True)
    assert torch.equal(hn, hs.transpose(1, 2))
    g = torch.Generator().manual_seed(48)
    for stage in (0, 1):
        cin = S.dec_out if stage == 0 else S.gen_ch[0]
        T = F0.shape[1] * (1 if stage == 0 else S.up_rates[0])
        x = _bf(torch.randn(2, T, cin, generator=g)).to(d)
        u = torch.ops.stzs.conv_transpose_up(h, x, hs, stage)
        un = torch.ops.stzs.conv_transpose_up(h, x.transpose(1, 2).contiguous(), hn, stage, nct=True)
        assert torch.equal(un, u.transpose(1, 2))
        m = torch.ops.stzs.mrf_resblock(h, u, c_d, stage)
        mn = torch.ops.stzs.mrf_resblock(h, u.transpose(1, 2).contiguous(), c_d, stage, nct=True)
        assert torch.equal(mn, m.transpose(1, 2))
        # the oracle takes NCT directly
        want = R.upsample_stage(P, S, x.float().cpu().transpose(1, 2), _bf(hn.cpu()), stage)
        assert rel_err(un.cpu(), want) < 2e-2
    xp = _bf(torch.randn(2, 481, S.gen_ch[-1], generator=g) * 0.5)
    w1 = torch.ops.stzs.conv_post_istft(h, xp.to(d))
    w2 = torch.ops.stzs.conv_post_istft(h, xp.transpose(1, 2).contiguous().to(d), nct=True)
    assert torch.equal(w1, w2)


def test_op_code_quantize(handle, tiny, tiny_params):
    """stzs::code_quantize vs oracle quantize_codes: indices and dequantised codes bit-exact."""
    from oracle import stzs_ref as R
    h, eng = handle
    z = torch.randn(3, tiny.L_s, tiny.code_dim, generator=torch.Generator().manual_seed(48)) * 0.2
    idx_w, q_w, _ = R.quantize_codes(tiny_params, tiny, z)
    idx, q = torch.ops.stzs.code_quantize(h, z.to(eng.device))
    assert torch.equal(idx.cpu(), idx_w) and torch.equal(q.cpu(), q_w)
