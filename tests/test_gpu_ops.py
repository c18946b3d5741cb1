"""Kernel-level parity: each HIP op (through the C-ABI) against a plain-torch fp32 restatement of
the op on identical bf16-representable inputs.  Tolerances are stated per test."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from refops import bf, conv_ref, convT_ref, max_rel, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    return StyleTTSZS(tiny, tiny_params, device=gpu_device)


def _pack(w, b, ups=0, lane16=False, narrow32=False, frag32=False):
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "t", w, b, ups=ups, lane16=lane16, narrow32=narrow32, frag32=frag32)
    A.finalize("cuda:0")
    cw.w = A[cw.w]
    cw.b = A[cw.b] if cw.b is not None else None
    return cw, A


def _act(t, C=None):
    from stzs.engine import Act
    return Act(t, 0, t.shape[-1] if C is None else C)


def _dev_ntc(x, ld, dtype=torch.bfloat16):
    B, T, Cc = x.shape
    t = torch.zeros(B, T, ld, dtype=dtype, device="cuda:0")
    t[:, :, :Cc] = x.to(dtype).cuda()
    return t


CONV_CASES = [
    # B, T, Ci, Co, k, dil, stride
    (2, 300, 96, 80, 3, 1, 1),
    (2, 1000, 128, 128, 11, 5, 1),
    (1, 257, 64, 256, 7, 3, 1),
    (2, 2401, 22, 32, 12, 1, 6),
    (3, 50, 514, 64, 3, 1, 1),
    (2, 700, 256, 256, 7, 3, 1),   # MRF stage-0 form: two 128-channel chunks, two column tiles
    (1, 3001, 128, 128, 3, 5, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_adain_snake(eng, case):
    """AdaIN prologue + Snake + dilated conv + residual/alpha/acc epilogue (MRF c2 form); bf16 out.
    tolerance: max-abs error <= 1.5e-2 of max|ref| (one bf16 ulp of the output + fp32 reorder)."""
    B, T, Ci, Co, k, dil, stride = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    pad = dil * (k - 1) // 2 if stride == 1 else (stride + 1) // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    mean = torch.randn(B, Ci, generator=g) * 0.1
    rstd = torch.rand(B, Ci, generator=g) + 0.5
    gb = torch.randn(B, 2 * Ci, generator=g) * 0.2
    alpha = torch.rand(Ci, generator=g) + 0.5
    T_out = (T + 2 * pad - dil * (k - 1) - 1) // stride + 1
    res = bf(torch.randn(B, T_out, Co, generator=g))
    acc = bf(torch.randn(B, T_out, Co, generator=g))
    sc = (1 + gb[:, :Ci]) * rstd
    sh = gb[:, Ci:] - mean * sc
    ref = conv_ref(x, w, b, pad=pad, dil=dil, stride=stride, sc=sc, sh=sh, pro_act="snake", alpha=alpha,
                   res=res, out_scale=1 / 3, acc_in=acc, beta=1.0)
    cw, _A = _pack(w, b)
    ld = (Ci + 7) // 8 * 8
    xd = _act(_dev_ntc(x, ld), Ci)
    yd = _act(torch.zeros(B, T_out, Co, dtype=torch.bfloat16, device="cuda:0"))
    from stzs import _lib as L
    stat_bs = Ci
    al = alpha.cuda()
    gbd = gb.cuda()  # keep alive: the kernel reads it asynchronously
    eng.conv(cw, xd, yd, pad=pad, dil=dil, stride=stride,
             pro=(mean.cuda(), rstd.cuda(), stat_bs, gbd.data_ptr(), 2 * Ci, Ci),
             pro_act=L.ACT_SNAKE, pro_alpha=al, res=_act(res.to(torch.bfloat16).cuda()), alpha=1 / 3,
             acc_in=_act(acc.to(torch.bfloat16).cuda()), beta=1.0)
    out = yd.t.float().cpu()
    e = max_rel(out, ref)
    print(case, "max_rel", e, "rel_l2", rel_err(out, ref))
    assert e < 1.5e-2


@pytest.mark.parametrize("dt_in,dt_out", [(torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32),
                                          (torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16)])
def test_linear_flat(eng, dt_in, dt_out):
    """ks=1 'flat' GEMM over rows spanning utterances: cscale prologue, GELU, per-(row-group) gate,
    batch-broadcast residual; tolerance 1e-2 (bf16 out) / 2e-3 (f32 out) of max|ref|."""
    g = torch.Generator().manual_seed(7)
    R, Lr, Ci, Co = 6, 50, 512, 384
    x = bf(torch.randn(R, Lr, Ci, generator=g))
    w = torch.randn(Co, Ci, generator=g) / math.sqrt(Ci)
    b = torch.randn(Co, generator=g) * 0.1
    gate = torch.randn(R, Co, generator=g)
    pos = bf(torch.randn(1, Lr, Co, generator=g)) if dt_out == torch.bfloat16 else torch.randn(1, Lr, Co, generator=g)
    cs = 0.7
    xs = bf(x * cs) if dt_in == torch.bfloat16 else bf(x * cs)
    ref = F.gelu(xs @ bf(w).t() + b) * gate[:, None, :] + pos
    cw, _A = _pack(w, b)
    xd = _act(x.to(dt_in).cuda())
    yd = _act(torch.zeros(R, Lr, Co, dtype=dt_out, device="cuda:0"))
    from stzs import _lib as L
    gated = gate.cuda()
    eng.conv(cw, xd, yd, cscale=cs, epi_act=L.ACT_GELU, gate=gated.data_ptr(), gate_bs=Co,
             res=_act(pos.to(dt_out).cuda()))
    out = yd.t.float().cpu()
    e = max_rel(out, ref)
    print(dt_in, dt_out, e)
    assert e < (1e-2 if dt_out == torch.bfloat16 else 2e-3)


@pytest.mark.parametrize("Ci,Co,s,refl,l16", [(64, 32, 10, 0, False), (32, 16, 6, 1, False), (512, 256, 10, 0, False),
                                               (256, 128, 6, 1, False), (512, 256, 10, 0, True), (256, 128, 6, 1, True),
                                               (200, 48, 4, 1, True)])
def test_convtranspose_polyphase(eng, Ci, Co, s, refl, l16):
    """polyphase ConvTranspose1d(k=2s) + LeakyReLU(0.1) prologue + ReflectionPad(1,0) + residual."""
    g = torch.Generator().manual_seed(Ci + s)
    B, T = 2, 40
    k, pad = 2 * s, s // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Ci, Co, k, generator=g) / math.sqrt(Co * k)
    b = torch.randn(Co, generator=g) * 0.1
    Tn = T * s + refl
    res = bf(torch.randn(B, Tn, Co, generator=g))
    ref = convT_ref(x, w, b, stride=s, pad=pad, refl=refl, pro_act="leaky", slope=0.1, res=res)
    cw, _A = _pack(w, b, ups=s, lane16=l16)  # l16: the MRF-family kernel's polyphase epilogue
    from stzs import _lib as L
    yd = _act(torch.zeros(B, Tn, Co, dtype=torch.bfloat16, device="cuda:0"))
    eng.conv(cw, _act(x.to(torch.bfloat16).cuda()), yd, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=pad,
             T_final=T * s, refl=refl, res=_act(res.to(torch.bfloat16).cuda()))
    out = yd.t.float().cpu()
    e = max_rel(out, ref)
    print(Ci, Co, s, refl, e)
    assert e < 1.5e-2


@pytest.mark.parametrize("B,T,Ci,Co,s,refl", [(2, 40, 512, 256, 10, 0), (3, 300, 256, 128, 6, 1), (2, 129, 384, 96, 4, 1),
                                              (1, 200, 512, 256, 10, 0), (2, 1000, 256, 128, 6, 1)])
def test_convtranspose_staged_once_bit_identical(eng, B, T, Ci, Co, s, refl):
    """the input-staged-once polyphase ConvTranspose (csrc/ups.hip, FRAG32 weights: every column tile of a
    workgroup over one resident input tile) == the MRF-family LANE16 form, BIT FOR BIT (same staged operands, same
    K order), and both within the bf16 tolerance of the fp32 reference."""
    g = torch.Generator().manual_seed(Ci + s + T)
    k, pad = 2 * s, s // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Ci, Co, k, generator=g) / math.sqrt(Co * k)
    b = torch.randn(Co, generator=g) * 0.1
    Tn = T * s + refl
    res = bf(torch.randn(B, Tn, Co, generator=g))
    ref = convT_ref(x, w, b, stride=s, pad=pad, refl=refl, pro_act="leaky", slope=0.1, res=res)
    from stzs import _lib as L
    outs = []
    for form in ("lane16", "frag32"):
        cw, _A = _pack(w, b, ups=s, lane16=form == "lane16", frag32=form == "frag32")
        yd = _act(torch.full((B, Tn, Co), float("nan"), dtype=torch.bfloat16, device="cuda:0"))
        eng.conv(cw, _act(x.to(torch.bfloat16).cuda()), yd, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=pad,
                 T_final=T * s, refl=refl, res=_act(res.to(torch.bfloat16).cuda()))
        torch.cuda.synchronize()
        outs.append(yd.t.clone())
    e = max_rel(outs[1].float().cpu(), ref)
    print(B, T, Ci, Co, s, refl, "staged-once vs ref", e)
    assert e < 1.5e-2
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,T,Ci,Co,s,Ch", [(2, 300, 256, 128, 6, 22), (3, 129, 256, 128, 6, 22), (1, 40, 512, 256, 4, 20)])
def test_convtranspose_fused_noise_conv(eng, B, T, Ci, Co, s, Ch):
    """STZS_CONV_UPS_NOISE (csrc/ups.hip): the last generator stage's ConvTranspose with its 1x1 noise conv fused as
    one more K-step per column tile == ReflectionPad(1,0)(convT(leaky(x))) + noise_conv(har) in fp32 (the unfused
    path rounds the noise conv's output to bf16 first), row 0 (the reflected row, which takes row 2's ConvTranspose
    value and row 0's noise term) included; and within bf16 of the unfused two-launch path."""
    from stzs import _lib as L
    from stzs.weights import Arena, pack_conv, pack_ups_noise
    g = torch.Generator().manual_seed(T + Ch)
    k, pad = 2 * s, s // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    wu = torch.randn(Ci, Co, k, generator=g) / math.sqrt(Co * k)
    bu = torch.randn(Co, generator=g) * 0.1
    wn = torch.randn(Co, Ch, 1, generator=g) / math.sqrt(Ch)
    bn = torch.randn(Co, generator=g) * 0.1
    Tn = T * s + 1
    har = bf(torch.randn(B, Tn, Ch, generator=g))
    har_d = torch.zeros(B, Tn, 32, dtype=torch.bfloat16, device="cuda:0")
    har_d[:, :, :Ch] = har.to(torch.bfloat16).cuda()
    xsrc = torch.einsum("btj,cj->btc", har.double(), bf(wn)[:, :, 0].double()) + bn.double()
    ref = convT_ref(x, wu, bu, stride=s, pad=pad, refl=1, pro_act="leaky", slope=0.1, res=xsrc.float())
    A = Arena()
    cw = pack_ups_noise(A, "t", wu, bu, wn, bn)
    A.finalize("cuda:0")
    cw.w, cw.b, cw.nz32 = A[cw.w], A[cw.b], A[cw.nz32]
    yd = _act(torch.full((B, Tn, Co), float("nan"), dtype=torch.bfloat16, device="cuda:0"))
    eng.conv(cw, _act(x.to(torch.bfloat16).cuda()), yd, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=pad, T_final=T * s,
             refl=1, res=_act(har_d), flags=L.CONV_UPS_NOISE, gate=cw.nz32.data_ptr())
    torch.cuda.synchronize()
    y = yd.t.float().cpu()
    e, e0 = max_rel(y, ref), max_rel(y[:, :1], ref[:, :1])
    # the unfused path: noise conv (bf16 output) as the ConvTranspose's residual
    cn, _An = _pack(wn, bn)
    xs = _act(torch.zeros(B, Tn, Co, dtype=torch.bfloat16, device="cuda:0"))
    eng.conv(cn, _act(har_d, Ch), xs)
    cu, _Au = _pack(wu, bu, ups=s, frag32=True)
    yu = _act(torch.zeros(B, Tn, Co, dtype=torch.bfloat16, device="cuda:0"))
    eng.conv(cu, _act(x.to(torch.bfloat16).cuda()), yu, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=pad,
             T_final=T * s, refl=1, res=xs)
    torch.cuda.synchronize()
    eu = max_rel(yu.t.float().cpu(), y)
    print(B, T, Ci, Co, s, "fused noise conv vs fp32", e, "row 0", e0, "vs unfused", eu)
    assert torch.isfinite(y).all()
    assert e < 1.5e-2 and e0 < 1.5e-2 and eu < 2e-2


@pytest.mark.parametrize("B,T80", [(2, 20), (3, 57)])
def test_noise_conv_super_rows(gpu_device, B, T80):
    """generator stage 0 with its stride-6 noise conv restated on super-rows of the harmonic source (engine.upsample,
    weights.noise_super_weights: a k3 stride-1 conv over 192 channels on the register-direct kernel) vs the oracle's
    upsample_stage (fp32: LeakyReLU, strided noise conv, ConvTranspose1d, sum) on the same bf16 inputs, and vs the
    stride-6 conv_mfma path (STZS_NOISE_SUPER=0): within bf16 rounding of each (v0 dims)."""
    from oracle import stzs_ref as R
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    P = init_params(S, seed=0)
    e = StyleTTSZS(S, P, device=gpu_device)
    assert e.W.noise_sup[0] is not None
    g = torch.Generator().manual_seed(B * 100 + T80)
    F0 = (100 + 150 * torch.rand(B, T80, generator=g)).to(gpu_device)
    har = e.sine_gen(F0, list(range(B)))
    x = bf(torch.randn(B, T80, S.dec_out, generator=g))
    ys = []
    for sup in (True, False):
        e.noise_super = sup
        ys.append(e.upsample(Act(x.to(torch.bfloat16).to(gpu_device)), har, 0).t.float().cpu().clone())
    torch.cuda.synchronize()
    Tf = T80 * S.hop // S.istft_hop + 1
    hn = har.t[:, :Tf, :S.har_ch].float().cpu().transpose(1, 2)
    ref = R.upsample_stage(P, S, x.transpose(1, 2), hn, 0).transpose(1, 2)
    e_ref, e_alt = max_rel(ys[0], ref), max_rel(ys[0], ys[1])
    print("noise conv on super-rows: vs oracle", e_ref, "vs stride-6 path", e_alt, "| stride-6 vs oracle", max_rel(ys[1], ref))
    assert ys[0].shape == ref.shape
    assert e_ref < 1.5e-2 and e_alt < 1.5e-2


def test_chan_stats(eng):
    """InstanceNorm statistics: fp32 partials + fixed-order fp64 combine; 1e-5 relative."""
    g = torch.Generator().manual_seed(3)
    B, T, C = 3, 24001, 128
    x = bf(torch.randn(B, T, C, generator=g) * 2 + 0.5)
    from stzs.engine import Act
    m, r, _ = eng.stats(Act(x.to(torch.bfloat16).cuda()), "t.stats")
    mr = x.double().mean(1)
    vr = x.double().var(1, unbiased=False)
    assert max_rel(m.cpu(), mr) < 1e-5
    assert max_rel(r.cpu(), 1 / torch.sqrt(vr + 1e-5)) < 1e-5


@pytest.mark.parametrize("B,T,Ci,Co,k,dil,dt_out", [(2, 1000, 128, 128, 11, 5, torch.bfloat16),
                                                   (3, 300, 96, 80, 3, 1, torch.bfloat16),
                                                   (2, 257, 64, 256, 7, 3, torch.float32)])
def test_conv_fused_stats(eng, B, T, Ci, Co, k, dil, dt_out):
    """InstanceNorm statistics fused into the conv epilogue (stat_part + stzs_chan_stats_final) equal
    the statistics of the tensor the conv stored, within 1e-5 (fp32 tile partials, fp64 combine)."""
    g = torch.Generator().manual_seed(B * T + Co)
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g)
    res = torch.randn(B, T, Co, generator=g)
    cw, _A = _pack(w, b)
    from stzs import _lib as L
    xd = _act(_dev_ntc(x, (Ci + 7) // 8 * 8), Ci)
    yd = _act(torch.zeros(B, T, Co, dtype=dt_out, device="cuda:0"))
    rd = _act(res.to(dt_out).cuda())
    al = (torch.rand(Ci, generator=g) + 0.5).cuda()
    _, (m, r, sb) = eng.conv(cw, xd, yd, pad=dil * (k - 1) // 2, dil=dil, pro_act=L.ACT_SNAKE, pro_alpha=al,
                             res=rd, stats_key="t.fstats")
    assert sb == Co
    y = yd.t.double().cpu()
    mr, vr = y.mean(1), y.var(1, unbiased=False)
    sd = vr.sqrt()
    assert float(((m.cpu().double() - mr).abs() / (mr.abs() + sd)).max()) < 1e-5
    assert max_rel(r.cpu(), 1 / torch.sqrt(vr + 1e-5)) < 1e-5


MRF_CASES = [
    # B, T, Ci, Co, k, dil, prologue, res, acc_in, stats, res_tdiv
    (3, 1000, 128, 128, 11, 5, "snake", False, False, True, 1),  # c1 form (fewer tiles than CUs)
    (40, 1000, 128, 128, 3, 1, "snake", True, True, False, 1),   # last c2 form (320 tiles)
    (9, 4000, 128, 128, 7, 3, "snake", True, False, True, 1),    # c2 form + stats (288 tiles)
    (2, 777, 256, 256, 7, 1, "snake", True, True, True, 1),      # stage-0 width: 2 input chunks x 2 column tiles
    (1, 129, 256, 256, 3, 5, "snake", False, False, True, 1),    # ragged: the second row tile has 1 valid row
    (2, 500, 384, 256, 11, 3, "snake", True, False, True, 1),    # 3 input chunks
    (2, 300, 256, 176, 3, 1, "snake", True, False, True, 1),     # Co < co_pad (masked column groups)
    (3, 400, 1090, 256, 3, 1, "leaky", True, False, True, 2),    # decoder block conv2: Ci 1090 (9 chunks), x2 shortcut
    (4, 200, 200, 96, 3, 1, "leaky", False, False, True, 1),     # predictor block conv1 (2 chunks, 1 column tile)
    (2, 300, 130, 64, 3, 1, "none", False, False, True, 1),      # up-block conv1 after the dw-ConvT: no prologue
    # k3, one 128-channel chunk (the stage-1 register-direct form, three workgroups per CU)
    (16, 24001, 128, 128, 3, 1, "snake", False, False, True, 1),  # stage-1 c1 shape: 3008 tiles, ~12 per CU
    (5, 24001, 128, 128, 3, 5, "snake", True, True, False, 1),    # stage-1 last c2 (residual + accumulate)
    (7, 3001, 128, 128, 3, 3, "snake", True, False, True, 1),     # c2 + stats, ragged last tile (3001 % 128)
    (300, 130, 128, 128, 3, 1, "snake", True, False, True, 1),    # 600 tiles of which every 2nd has 2 valid rows
    (3, 500, 128, 64, 3, 1, "leaky", True, False, True, 1),       # Co 64 (half the column tile), LeakyReLU
    (2, 333, 128, 128, 3, 2, "none", False, False, True, 1),      # no prologue
]


def _run_mrf(eng, case, form, flags=0, ref=True):
    B, T, Ci, Co, k, dil, act, hr, ha, st, tdiv = case
    g = torch.Generator().manual_seed(B * T + Ci + k)
    pad = dil * (k - 1) // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    mean = torch.randn(B, Ci, generator=g) * 0.1
    rstd = torch.rand(B, Ci, generator=g) + 0.5
    gb = torch.randn(B, 2 * Ci, generator=g) * 0.2
    alpha = torch.rand(Ci, generator=g) + 0.5
    res = bf(torch.randn(B, (T + tdiv - 1) // tdiv, Co, generator=g)) if hr else None
    acc = bf(torch.randn(B, T, Co, generator=g)) if ha else None
    sc = (1 + gb[:, :Ci]) * rstd
    sh = gb[:, Ci:] - mean * sc
    if act == "none":
        sc, sh = torch.ones(B, Ci), torch.zeros(B, Ci)
    osc = 1 / 3 if ha else (0.7071 if hr else 1.0)
    ref = conv_ref(x, w, b, pad=pad, dil=dil, stride=1, sc=sc, sh=sh, pro_act=None if act == "none" else act,
                   slope=0.2, alpha=alpha, res=res, res_tdiv=tdiv, out_scale=osc, acc_in=acc, beta=1.0) if ref else None
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "t", w, b, lane16=form == "lane16", frag32=form == "frag32")
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    from stzs import _lib as L
    xd = _act(_dev_ntc(x, (Ci + 7) // 8 * 8), Ci)
    yd = _act(torch.zeros(B, T, Co, dtype=torch.bfloat16, device="cuda:0"))
    keep = [mean.cuda(), rstd.cuda(), gb.cuda(), alpha.cuda()]
    rd = _act(res.to(torch.bfloat16).cuda()) if hr else None
    ad = _act(acc.to(torch.bfloat16).cuda()) if ha else None
    pro = None if act == "none" else (keep[0], keep[1], Ci, keep[2].data_ptr(), 2 * Ci, Ci)
    pa = {"snake": L.ACT_SNAKE, "leaky": L.ACT_LEAKY, "none": L.ACT_NONE}[act]
    out = eng.conv(cw, xd, yd, pad=pad, dil=dil, pro=pro, pro_act=pa, pro_slope=0.2,
                   pro_alpha=keep[3] if act == "snake" else None, res=rd, res_tdiv=tdiv, alpha=osc, acc_in=ad,
                   beta=1.0, stats_key=f"t.mrfst.{form}" if st else None, flags=flags)
    stats = (out[1][0].clone().cpu(), out[1][1].clone().cpu()) if st else None
    return yd.t.float().cpu(), stats, ref


@pytest.mark.parametrize("form", ["lane16", "frag32"])
@pytest.mark.parametrize("case", MRF_CASES)
def test_mrf_persistent_conv(eng, case, form):
    """MRF-family conv -- lane16: csrc/mrf.hip (LDS-DMA weight ring); frag32: csrc/mrfv.hip (register-direct
    weight fragments) -- AdaIN + Snake / LeakyReLU / identity prologue, residual (at t / res_tdiv) / alpha /
    acc_in epilogue and fused statistics vs the fp32 reference.  tolerance: max-abs error <= 1.5e-2 of
    max|ref| (bf16 output); statistics 1e-5 of the stored tensor."""
    st = case[9]
    got, stats, ref = _run_mrf(eng, case, form)
    e = max_rel(got, ref)
    print(case, form, "max_rel", e, "rel_l2", rel_err(got, ref))
    assert e < 1.5e-2
    if st:
        m, r = stats
        y = got.double()
        mr, vr = y.mean(1), y.var(1, unbiased=False)
        assert float(((m.double() - mr).abs() / (mr.abs() + vr.sqrt())).max()) < 1e-5
        assert max_rel(r, 1 / torch.sqrt(vr + 1e-5)) < 1e-5


@pytest.mark.parametrize("case", MRF_CASES)
def test_mrf_frag32_bit_identical(eng, case):
    """the register-direct kernel accumulates every output in the same K order from the same staged bf16
    operands as the LDS-ring kernel: outputs and fused statistics are bit-identical (tolerance 0)."""
    a, sa, _ = _run_mrf(eng, case, "lane16")
    b, sb, _ = _run_mrf(eng, case, "frag32")
    assert torch.equal(a, b)
    if sa is not None:
        assert torch.equal(sa[0], sb[0]) and torch.equal(sa[1], sb[1])


# multi-chunk Snake convs with >= 512 wide tiles (batch x row tiles x 256-channel tiles): the wide mrfv form
WIDE_CASES = [
    (20, 3300, 256, 256, 7, 3, "snake", True, True, True, 1),    # stage-0 width, residual + accumulate + stats
    (18, 3700, 384, 256, 11, 5, "snake", True, False, True, 1),  # 3 input chunks, ragged last row tile
    (20, 3300, 256, 176, 3, 1, "snake", False, False, True, 1),  # Co < co_pad: masked column groups
    # the AdaIN-block convs (r05: wide where the wide grid has >= two tiles per CU): LeakyReLU prologue, x2 shortcut
    (64, 200, 1090, 1024, 3, 1, "leaky", True, False, True, 2),   # decoder up-block conv2 form, 9 chunks
    (64, 400, 1090, 512, 3, 1, "none", False, False, True, 1),    # up-block conv1 after the depthwise ConvT
    (66, 203, 514, 1024, 3, 1, "leaky", False, False, True, 1),   # encode-block conv1, ragged last tile
]


@pytest.mark.parametrize("case", WIDE_CASES)
def test_mrf_wide_bit_identical(eng, case):
    """the wide register-direct form (256 output channels per workgroup, the default for multi-chunk Snake convs whose
    wide grid has >= 512 workgroups, and for the LeakyReLU / identity block convs likewise) vs the narrow one (STZS_CONV_MRFV_NARROW: 128 per workgroup): same staged
    operands, same K order per output -> outputs and fused statistics bit-identical (tolerance 0)."""
    from stzs import _lib as L
    a, sa, _ = _run_mrf(eng, case, "frag32", flags=L.CONV_MRFV_NARROW, ref=False)
    b, sb, _ = _run_mrf(eng, case, "frag32", ref=False)
    assert torch.equal(a, b)
    if sa is not None:
        assert torch.equal(sa[0], sb[0]) and torch.equal(sa[1], sb[1])


# Snake convs whose 128-row grid has fewer than two tiles per CU (batch 1): the 64-row-tile mrfv form
T64_CASES = [
    (1, 24001, 128, 128, 3, 1, "snake", False, False, True, 1),   # batch-1 stage-1 c1 (188 -> 376 workgroups)
    (1, 24001, 128, 128, 11, 5, "snake", True, True, False, 1),   # stage-1 last c2: residual + accumulate, dil 5 halo
    (1, 3001, 256, 256, 7, 3, "snake", True, False, True, 1),     # stage 0 (2 chunks), ragged: 3001 % 64 = 57
    (2, 4033, 384, 176, 11, 5, "snake", True, True, True, 1),     # 3 chunks, Co < co_pad, a 1-row last tile
    # the narrow AdaIN-block convs below 4 128-row tiles per CU (r05): LeakyReLU + x2 shortcut, identity prologue
    (8, 200, 1090, 1024, 3, 1, "leaky", True, False, True, 2),
    (6, 401, 512, 256, 3, 1, "none", False, False, True, 1),
]


@pytest.mark.parametrize("case", T64_CASES)
def test_mrf_t64_bit_identical(eng, case):
    """the 64-row-tile register-direct form (the launcher's choice when the 128-row grid has fewer than 2 workgroups per
    CU, or fewer than 4 for the LeakyReLU / identity block convs) vs the 128-row tiles (STZS_CONV_MRFV_T128): same staged operands, same K order per output, same 64-row
    statistics chunks -> outputs and fused statistics bit-identical (tolerance 0)."""
    from stzs import _lib as L
    a, sa, _ = _run_mrf(eng, case, "frag32", flags=L.CONV_MRFV_T128, ref=False)
    b, sb, _ = _run_mrf(eng, case, "frag32", ref=False)
    assert torch.equal(a, b)
    if sa is not None:
        assert torch.equal(sa[0], sb[0]) and torch.equal(sa[1], sb[1])


@pytest.mark.parametrize("B,T,Ci,Co,ld", [(64, 200, 1090, 1024, 1096), (2, 37, 514, 1024, 520), (3, 131, 1090, 512, 1160),
                                         (1, 200, 512, 256, 512), (200, 700, 512, 128, 512)])
def test_block_shortcut_frag32(eng, B, T, Ci, Co, ld):
    """the AdaIN blocks' 1x1 shortcut on the register-direct block-conv form (STZS_CONV_W_FRAG32, ks 1; the wide form at
    B = 64, the narrow 128-row form last, the 64-row form between) vs the same weights on the K-step path (the LDS-DMA GEMM where the rows
    are wide enough, else the generic conv): the same bits, and within 1e-2 of max|ref| of the fp32 product."""
    g = torch.Generator().manual_seed(Ci + T)
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, 1, generator=g) / math.sqrt(Ci)
    ref = torch.einsum("btc,oc->bto", x, w[:, :, 0])
    xd = _act(_dev_ntc(x, ld), Ci)
    outs = []
    for frag in (False, True):
        cw, _A = _pack(w, None, frag32=frag)
        yd = _act(torch.zeros(B, T, Co, dtype=torch.bfloat16, device="cuda:0"))
        eng.conv(cw, xd, yd)
        torch.cuda.synchronize()
        outs.append(yd.t.float().cpu())
    assert torch.equal(outs[0], outs[1])
    assert max_rel(outs[1], ref) < 1e-2


@pytest.mark.parametrize("B,T,Ci,Co,k", [(2, 3001, 128, 22, 7), (1, 300, 256, 32, 3), (3, 257, 128, 8, 7)])
def test_narrow_conv(eng, B, T, Ci, Co, k):
    """narrow conv (conv_post form: LeakyReLU(0.01) prologue, Co <= 32, fp32 out, csrc/mrf.hip
    narrow_conv) vs the fp32 reference; tolerance 2e-3 of max|ref| (fp32 output, bf16 operands)."""
    g = torch.Generator().manual_seed(T + Co)
    pad = (k - 1) // 2
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    ref = conv_ref(x, w, b, pad=pad, pro_act="leaky", slope=0.01)
    cw, _A = _pack(w, b, narrow32=True)
    from stzs import _lib as L
    yd = _act(torch.zeros(B, T, (Co + 7) // 8 * 8, device="cuda:0"), Co)
    eng.conv(cw, _act(x.to(torch.bfloat16).cuda()), yd, pad=pad, pro_act=L.ACT_LEAKY, pro_slope=0.01)
    got = yd.t[:, :, :Co].cpu()
    e = max_rel(got, ref)
    print(B, T, Ci, Co, k, e)
    assert e < 2e-3


def test_row_layernorm(eng):
    g = torch.Generator().manual_seed(4)
    R, Lr, C = 4, 50, 512
    x = torch.randn(R * Lr, C, generator=g) * 3 + 1
    G = torch.randn(R, 3 * C, generator=g)
    ref = F.layer_norm(x, (C,)).view(R, Lr, C) * G[:, None, C:2 * C] + G[:, None, :C]
    from stzs.engine import Act
    xd = Act(x.view(R, Lr, C).cuda())
    yd = Act(torch.zeros(R, Lr, C, device="cuda:0"))
    Gd = G.cuda()
    eng.rowln(xd, yd, G=Gd.data_ptr() + C * 4, gs=3 * C, Bt=Gd.data_ptr(), bs=3 * C, gdiv=Lr, gadd=0.0)
    assert max_rel(yd.t.cpu(), ref) < 1e-5


@pytest.mark.parametrize("Lk", [50, 130, 530])
def test_attention(eng, Lk):
    """online-softmax MHA (fp32 math, bf16 I/O); tolerance 1e-2 of max|ref|."""
    S = eng.spec
    g = torch.Generator().manual_seed(Lk)
    R, Lq, D = 3, 50, S.dn_d
    H, dh = S.dn_heads, S.dn_head_dim
    q = bf(torch.randn(R, Lq, D, generator=g))
    k = bf(torch.randn(R, Lk, 2 * D, generator=g))
    qh = q.view(R, Lq, H, dh).transpose(1, 2)
    kh = k[..., :D].reshape(R, Lk, H, dh).transpose(1, 2)
    vh = k[..., D:].reshape(R, Lk, H, dh).transpose(1, 2)
    ref = (torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(dh), -1) @ vh).transpose(1, 2).reshape(R, Lq, D)
    from stzs.engine import Act
    kd = Act(k.to(torch.bfloat16).cuda())
    od = Act(torch.zeros(R, Lq, D, dtype=torch.bfloat16, device="cuda:0"))
    eng.attention(Act(q.to(torch.bfloat16).cuda()), kd.sl(0, D), kd.sl(D, D), od)
    assert max_rel(od.t.float().cpu(), ref) < 1e-2


def test_lstm(eng, tiny_params):
    """bidirectional LSTM (GEMM input projection + recurrent kernel) vs torch.nn.LSTM."""
    from oracle.stzs_ref import bilstm
    from stzs.engine import Act
    P = tiny_params
    g = torch.Generator().manual_seed(5)
    B, T = 3, 37
    x = bf(torch.randn(B, T, eng.spec.pr_in, generator=g))
    ref = bilstm(x, P, "pr.de0")
    y = Act(torch.zeros(B, T, eng.spec.pr_hid, dtype=torch.bfloat16, device="cuda:0"))
    eng.lstm(eng.W.pr_de[0], Act(x.to(torch.bfloat16).cuda()), y, "t.lstm")
    e = max_rel(y.t.float().cpu(), ref)
    print("lstm", e)
    assert e < 2e-2


def _v0_lstm(In=640, H=256, seed=9):
    """random LSTM parameters at the v0 predictor width (pr_in 640 -> 2 x 256) and their packing."""
    from stzs.weights import Arena, pack_lstm
    g = torch.Generator().manual_seed(seed)
    k = 1.0 / math.sqrt(H)
    P = {}
    for sfx in ("", "_rev"):
        P["t.w_ih" + sfx] = (torch.rand(4 * H, In, generator=g) * 2 - 1) * k
        P["t.w_hh" + sfx] = (torch.rand(4 * H, H, generator=g) * 2 - 1) * k
        P["t.b_ih" + sfx] = (torch.rand(4 * H, generator=g) * 2 - 1) * k
        P["t.b_hh" + sfx] = (torch.rand(4 * H, generator=g) * 2 - 1) * k
    A = Arena()
    lw = pack_lstm(A, "t", P)
    A.finalize("cuda:0")
    lw.ih.w, lw.ih.b, lw.whhT = A[lw.ih.w], A[lw.ih.b], A[lw.whhT]
    return P, lw, A


@pytest.mark.parametrize("B,T", [(64, 80), (40, 23), (1, 80), (2, 50), (65, 7)])
def test_lstm_v0_width(eng, B, T):
    """the benchmarked LSTM shape: H = 256 (8 exchanging workgroups per direction), 16-64 utterances per
    group (1-4 MFMA row tiles, multi-row exchange loads) vs torch.nn.LSTM on identical bf16 inputs; B = 1 / 2 and
    the 1-row last group of B = 65 hand h over as tagged granules (csrc/lstm.hip TAG_ROWS), run twice: the second
    call must not see the first call's tags (bit-identical).
    tolerance: max-abs error <= 2e-2 of max|ref| (bf16 h exchanged every step, fp32 cell state)."""
    from oracle.stzs_ref import bilstm
    from stzs.engine import Act
    P, lw, _A = _v0_lstm()
    g = torch.Generator().manual_seed(B * 1000 + T)
    x = bf(torch.randn(B, T, 640, generator=g))
    ref = bilstm(x, P, "t")
    y = Act(torch.zeros(B, T, 512, dtype=torch.bfloat16, device="cuda:0"))
    eng.lstm(lw, Act(x.to(torch.bfloat16).cuda()), y, f"t.lstm{B}")
    assert eng.check_status() == 0
    y0 = y.t.clone()
    y.t.zero_()
    eng.lstm(lw, Act(x.to(torch.bfloat16).cuda()), y, f"t.lstm{B}")
    assert eng.check_status() == 0
    assert torch.equal(y.t, y0)
    e = max_rel(y.t.float().cpu(), ref)
    print("lstm v0", B, T, e, rel_err(y.t.float().cpu(), ref))
    assert e < 2e-2


def test_lstm_group_rows_invariant(eng):
    """B = 64 runs as four 16-utterance groups (csrc/lstm.hip lstm_group_rows: 64 workgroups, one MFMA row tile of
    work per group and step), B = 32 as two, B = 16 as one group, B = 1 on the tagged granules: every utterance's h
    must be the same bits in all four (the per-row gate chain and cell update do not depend on the group)."""
    from stzs.engine import Act
    _P, lw, _A = _v0_lstm()
    g = torch.Generator().manual_seed(77)
    x = torch.randn(64, 60, 640, generator=g).to(torch.bfloat16).cuda()
    outs = {}
    for B in (64, 32, 16, 1):
        y = Act(torch.zeros(B, 60, 512, dtype=torch.bfloat16, device="cuda:0"))
        eng.lstm(lw, Act(x[:B].contiguous()), y, f"t.lstmg{B}")
        assert eng.check_status() == 0
        outs[B] = y.t.clone()
    assert torch.equal(outs[64][:32], outs[32])
    assert torch.equal(outs[64][:16], outs[16])
    assert torch.equal(outs[64][:1], outs[1])


@pytest.mark.parametrize("B", [1, 2, 16, 64, 65, 129, 192])
def test_lstm_pair_bit_identical(eng, B):
    """stzs_lstm_pair (engine.lstm_pair): two independent recurrences of different lengths in one launch -- the first
    over T = 60, the second over T = 23 -- each the same bits as its own stzs_lstm call (tagged granules at B = 1 / 2,
    16-row counter groups above), run twice (each pair leaves its own exchange state zeroed).  B = 129 / 192: the two
    grids together exceed one workgroup per CU, so the library runs them as two launches (same bits, no error)."""
    from stzs.engine import Act
    _P, lw, _A = _v0_lstm()
    g = torch.Generator().manual_seed(500 + B)
    xa = Act(torch.randn(B, 60, 640, generator=g).to(torch.bfloat16).cuda())
    xb = Act(torch.randn(B, 23, 640, generator=g).to(torch.bfloat16).cuda())
    ya, yb = (Act(torch.zeros(B, t, 512, dtype=torch.bfloat16, device="cuda:0")) for t in (60, 23))
    eng.lstm(lw, xa, ya, "t.pa")
    eng.lstm(lw, xb, yb, "t.pb")
    assert eng.check_status() == 0
    ra, rb = ya.t.clone(), yb.t.clone()
    for _ in range(2):
        ya.t.zero_()
        yb.t.zero_()
        eng.lstm_pair((lw, xa, ya, "t.pa"), (lw, xb, yb, "t.pb"))
        assert eng.check_status() == 0
        assert torch.equal(ya.t, ra) and torch.equal(yb.t, rb)


def test_lstm_timeout_tagged_never_hangs(eng):
    """B = 1 (tagged-granule sweep) under a 1-poll spin limit: the tagged hand-off seldom waits past two polls, so
    a timeout cannot be forced deterministically; every run must either report STZS_STATUS_LSTM_TIMEOUT (and then
    check_status raises) or match the normal run bit for bit -- never hang, never return silently wrong h."""
    from stzs.engine import Act
    _P, lw, _A = _v0_lstm()
    x = Act(torch.randn(1, 200, 640).to(torch.bfloat16).cuda())
    y = Act(torch.zeros(1, 200, 512, dtype=torch.bfloat16, device="cuda:0"))
    eng.check_status()
    eng.lstm(lw, x, y, "t.lstm_to1")
    assert eng.check_status() == 0
    good = y.t.clone()
    fired = 0
    for _ in range(10):
        eng.lstm_spin_limit = 1
        try:
            eng.lstm(lw, x, y, "t.lstm_to1")
        finally:
            eng.lstm_spin_limit = 0
        try:
            eng.check_status()
            assert torch.equal(y.t, good)
        except RuntimeError as e:
            assert "spin timed out" in str(e)
            fired += 1
    print("tagged forced timeouts fired:", fired, "of 10")
    eng.lstm(lw, x, y, "t.lstm_to1")
    assert eng.check_status() == 0 and torch.equal(y.t, good)


@pytest.mark.parametrize("B", [8])
def test_lstm_timeout_surfaces(eng, B):
    """a spin that times out (forced: spin limit 1 poll) ORs STZS_STATUS_LSTM_TIMEOUT into the engine's
    status word; check_status() raises on it and clears it, and a normal run afterwards is clean."""
    from stzs.engine import Act
    _P, lw, _A = _v0_lstm()
    x = Act(torch.randn(B, 200, 640).to(torch.bfloat16).cuda())
    y = Act(torch.zeros(B, 200, 512, dtype=torch.bfloat16, device="cuda:0"))
    eng.check_status()
    eng.lstm_spin_limit = 1
    try:
        for _ in range(3):  # 8 workgroups per direction x 199 hand-offs: some consumer always waits > 1 poll
            eng.lstm(lw, x, y, "t.lstm_to")
    finally:
        eng.lstm_spin_limit = 0
    with pytest.raises(RuntimeError, match="spin timed out"):
        eng.check_status()
    assert eng.check_status() == 0  # cleared by the raising check
    eng.lstm(lw, x, y, "t.lstm_to")
    assert eng.check_status() == 0


def test_durations_alignment_gather_exact(eng):
    """integer path is bit-exact: round(serial sum sigmoid) clamp>=1, scan, row gather."""
    from oracle.stzs_ref import alignment_index, durations_from_logits
    from stzs import _lib as L
    g = torch.Generator().manual_seed(6)
    B, T, nb = 4, 33, 50
    logits = torch.randn(B, T, nb, generator=g) * 2 - 1
    dur_ref, dsum = durations_from_logits(logits)
    ld = torch.zeros(B, T, nb, device="cuda:0")
    ld.copy_(logits)
    dur = torch.zeros(B, T, dtype=torch.int32, device="cuda:0")
    ds = torch.zeros(B, T, device="cuda:0")
    a = L.DurArgs()
    a.logits, a.override_dur, a.dur, a.dsum = ld.data_ptr(), None, dur.data_ptr(), ds.data_ptr()
    a.ldl, a.bsl, a.B, a.T, a.nbins = nb, T * nb, B, T, nb
    eng._call(eng.lib.stzs_durations, a, "dur")
    tie = ((dsum - dsum.floor() - 0.5).abs() < 1e-4)
    ok = (dur.cpu() == dur_ref) | tie
    assert bool(ok.all())
    # alignment on equal-total durations
    dd = torch.tensor([[3, 2] * 8 + [1]] * B, dtype=torch.int32)
    dd[:, -1] = 0
    dd[:, 0] += 1
    idx_ref = alignment_index(dd)
    T40 = idx_ref.shape[1]
    idx = torch.zeros(B, T40, dtype=torch.int32, device="cuda:0")
    tot = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    a = L.AlignArgs()
    ddd = dd.cuda()
    a.dur, a.idx, a.total, a.B, a.T, a.T40 = ddd.data_ptr(), idx.data_ptr(), tot.data_ptr(), B, dd.shape[1], T40
    eng._call(eng.lib.stzs_alignment, a, "align")
    assert torch.equal(idx.cpu(), idx_ref)
    assert torch.equal(tot.cpu(), dd.sum(1).int())
    src = torch.randn(B, dd.shape[1], 64, generator=g).to(torch.bfloat16)
    from stzs.engine import Act
    y = Act(torch.zeros(B, T40, 72, dtype=torch.bfloat16, device="cuda:0"), 8, 64)
    eng.gather(Act(src.cuda()), idx, y, 64)
    ref = torch.stack([src[b, idx_ref[b].long()] for b in range(B)])
    assert torch.equal(y.t[:, :, 8:].cpu(), ref)


def test_harmonic_source_vs_oracle(eng, tiny_params):
    """SineGen + counter-RNG noise + merge + STFT (real|imag) vs the oracle; bf16 output."""
    from oracle.stzs_ref import source_features
    S = eng.spec
    g = torch.Generator().manual_seed(8)
    B, T80 = 2, 40
    F0 = 120 + 80 * torch.rand(B, T80, generator=g)
    F0[:, 5:9] = 0.0  # unvoiced stretch
    seeds = [11, 12345]
    ref, _ = source_features(tiny_params, S, F0, seeds)   # [B, 22, Tf]
    from stzs.engine import Act
    pre = eng.buf("t.pref", (B, S.harmonic_num + 1, T80), torch.float32)
    Fd = F0.cuda()
    from stzs import _lib as L
    Tf = T80 * S.hop // S.istft_hop + 1
    h = Act(torch.zeros(B, Tf, 24, dtype=torch.bfloat16, device="cuda:0"))
    sd = torch.tensor(seeds, dtype=torch.int32, device="cuda:0")
    a = L.SourceArgs()
    a.f0, a.seeds, a.merge_w, a.prefix, a.har = Fd.data_ptr(), sd.data_ptr(), eng.W.t(eng.W.src_merge).data_ptr(), \
        pre.data_ptr(), h.ptr
    a.ldf, a.ldh, a.bsh = T80, 24, Tf * 24
    a.B, a.T80, a.hop, a.n_fft, a.hop_s, a.nh = B, T80, S.hop, S.n_fft, S.istft_hop, S.harmonic_num + 1
    a.sr, a.sine_amp, a.noise_std, a.voiced_thr = float(S.sr), S.sine_amp, S.noise_std, S.voiced_threshold
    a.har_dtype = L.BF16
    eng._call(eng.lib.stzs_harmonic_source, a, "src")
    har = h.t[:, :, :22].float().cpu().transpose(1, 2)
    e = max_rel(har, ref)
    print("source", e, rel_err(har, ref))
    assert e < 1e-2
    # the per-frame phase prefix: the same IEEE fp64 recurrence (acc = frac(acc + hop * (f0 (h + 1) / sr)), one
    # rounding per operation, fp32 store before each add) restated in numpy -> bit-exact
    f = F0.double().numpy()
    want = np.zeros((B, S.harmonic_num + 1, T80), dtype=np.float32)
    for b in range(B):
        for hh in range(S.harmonic_num + 1):
            acc = np.float64(0.0)
            for k in range(T80):
                want[b, hh, k] = np.float32(acc)
                inc = np.float64(f[b, k] * np.float64(hh + 1)) / np.float64(S.sr)
                acc = acc + np.float64(S.hop) * inc
                acc = acc - np.floor(acc)
    assert np.array_equal(pre.cpu().numpy(), want)


def test_istft(eng):
    """exp/sin spectrum + irfft + Hann OLA + envelope vs torch.istft; fp32, 1e-5."""
    from stzs import _lib as L
    g = torch.Generator().manual_seed(9)
    B, Tf = 2, 2401
    post = torch.randn(B, Tf, 24, generator=g) * 0.5
    spec = torch.exp(post[:, :, :11]) * torch.exp(1j * torch.sin(post[:, :, 11:22]))
    ref = torch.istft(spec.transpose(1, 2), 20, hop_length=5, win_length=20, window=torch.hann_window(20))
    pd = post.cuda()
    wav = torch.zeros(B, (Tf - 1) * 5, device="cuda:0")
    a = L.IstftArgs()
    a.post, a.wav, a.ldp, a.bsp, a.bsw = pd.data_ptr(), wav.data_ptr(), 24, Tf * 24, (Tf - 1) * 5
    a.B, a.Tf, a.n_fft, a.hop_s = B, Tf, 20, 5
    eng._call(eng.lib.stzs_istft, a, "istft")
    assert max_rel(wav.cpu(), ref) < 1e-5


def test_abi_rejects_bad_shapes(eng):
    """invalid arguments return a negative code before any launch (no fault)."""
    from stzs import _lib as L
    import ctypes as C
    a = L.ConvArgs()
    assert eng.lib.stzs_conv1d(C.byref(a), None) == -1  # null pointers
    t = torch.zeros(64, device="cuda:0", dtype=torch.bfloat16)
    a.x = a.w = a.y = t.data_ptr()
    a.cic = 64
    a.B, a.T_in, a.T_out, a.Ci, a.Co, a.ks, a.dil, a.stride = 1, 4, 4, 8, 8, 1, 1, 1
    a.ci_pad, a.co_pad, a.ldx, a.bsx = 64, 64, 7, 28  # ld not a multiple of 8
    assert eng.lib.stzs_conv1d(C.byref(a), None) == -2
    # fused statistics are refused on the ConvTranspose (ups) form and on the flat linear form
    a.ldx, a.bsx, a.ci_pad, a.co_pad = 8, 32, 64, 128
    a.Ci, a.Co, a.cic, a.ldy, a.bsy = 8, 8, 64, 8, 40
    a.stat_part, a.stat_ld = t.data_ptr(), 8
    a.ups, a.ks, a.pad, a.T_out, a.T_final = 2, 2, 1, 5, 8
    assert eng.lib.stzs_conv1d(C.byref(a), None) == -1
    a.ups, a.ks, a.pad, a.T_out, a.T_final = 0, 1, 0, 4, 0
    assert eng.lib.stzs_conv1d(C.byref(a), None) == -1


@pytest.mark.parametrize("B,T,C,dil,res,trio", [(1, 1000, 256, 1, False, True), (1, 1000, 256, 5, True, True),
                                               (1, 3001, 128, 3, False, True), (2, 700, 128, 5, True, True),
                                               (1, 77, 128, 1, True, True), (48, 1400, 128, 1, False, False)])
def test_mrf_trio_group_bit_identical(eng, B, T, C, dil, res, trio):
    """stzs_conv1d_group on the k3 / k7 / k11 convs of one MRF layer (Snake AdaIN prologue, fused statistics, with and
    without the residual; stage-0 256-channel and stage-1 128-channel inputs) vs three stzs_conv1d calls: outputs, the
    statistics partials and their grouped finalisation (stzs_chan_stats_final_group) bit-identical.  Small batches run
    as ONE launch (mrfv_trio; the library returns 1); at 48 utterances the 64-row form does not apply and the group
    runs the three convs one after the other (returns 3), same bits."""
    from stzs import _lib as L
    g = torch.Generator().manual_seed(T + C + dil)
    x = _act(torch.randn(B, T, C, generator=g).to("cuda:0", torch.bfloat16))
    mean = (torch.randn(B, C, generator=g) * 0.1).cuda()
    rstd = (torch.rand(B, C, generator=g) + 0.5).cuda()
    gb = (torch.randn(B, 2 * C, generator=g) * 0.2).cuda()
    al = (torch.rand(C, generator=g) + 0.5).cuda()
    keep, convs = [], []
    for k in (3, 7, 11):
        w = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
        cw, A = _pack(w, torch.randn(C, generator=g) * 0.1, frag32=True)
        keep.append(A)
        convs.append((cw, k))

    def run(group):
        ys, grp, sts = [], [], []
        for cw, k in convs:
            y = _act(torch.zeros(B, T, C, device="cuda:0", dtype=torch.bfloat16))
            _, st = eng.conv(cw, x, y, pad=dil * (k - 1) // 2, dil=dil, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C),
                             pro_act=L.ACT_SNAKE, pro_alpha=al, res=x if res else None,
                             stats_key=f"trio.{group}.{k}", collect=grp if group else None)
            ys.append(y)
            sts.append(st)
        if group:
            arr = (L.ConvArgs * 3)(*grp)
            n = eng.lib.stzs_conv1d_group(arr, 3, eng.stream())
            assert n == (1 if trio else 3), n
            eng._finalize_group([st[0].ref for st in sts])
        torch.cuda.synchronize()
        tens = lambda v: (v.tensor() if hasattr(v, "tensor") else v).clone()
        return [y.t.clone() for y in ys], [(tens(st[0]), tens(st[1])) for st in sts]

    y0, s0 = run(False)
    y1, s1 = run(True)
    for a, b in zip(y0, y1):
        assert torch.equal(a, b)
    for (m0, r0), (m1, r1) in zip(s0, s1):
        assert torch.equal(m0, m1) and torch.equal(r0, r1)


@pytest.mark.parametrize("B,T,Ci,Co,res,pair", [(1, 100, 512, 512, False, True), (1, 200, 512, 256, True, True),
                                               (2, 130, 256, 512, True, True), (1, 100, 512, 512, False, False)])
def test_conv_pair_group_bit_identical(eng, B, T, Ci, Co, res, pair):
    """stzs_conv1d_group on two independent DEEP split-K convs (AdaIN + LeakyReLU prologue, k 3, fused statistics,
    with and without the residual; the prosody predictor's F0 / N block convs at batch 1) vs two stzs_conv1d calls:
    outputs and statistics bit-identical.  One conv_mfma_pair + one splitk_epi_pair launch (the library returns 1);
    with different slice counts (last case: 4 vs 2 slices) the two run one after the other (returns 2), same bits."""
    from stzs import _lib as L
    g = torch.Generator().manual_seed(T + Ci + Co)
    xs = [_act(torch.randn(B, T, Ci, generator=g).to("cuda:0", torch.bfloat16)) for _ in range(2)]
    rs = [_act(torch.randn(B, T, Co, generator=g).to("cuda:0", torch.bfloat16)) if res else None for _ in range(2)]
    pros = []
    for _ in range(2):
        mean = (torch.randn(B, Ci, generator=g) * 0.1).cuda()
        rstd = (torch.rand(B, Ci, generator=g) + 0.5).cuda()
        gb = (torch.randn(B, 2 * Ci, generator=g) * 0.2).cuda()
        pros.append((mean, rstd, gb))
    keep, convs = [], []
    for _ in range(2):
        w = torch.randn(Co, Ci, 3, generator=g) / math.sqrt(Ci * 3)
        cw, A = _pack(w, torch.randn(Co, generator=g) * 0.1)
        keep.append(A)
        convs.append(cw)
    sks = (16, 16) if pair else (16, 2)

    def run(group):
        ys, grp, sts = [], [], []
        for i in range(2):
            mean, rstd, gb = pros[i]
            y = _act(torch.zeros(B, T, Co, device="cuda:0", dtype=torch.bfloat16))
            _, st = eng.conv(convs[i], xs[i], y, pad=1, pro=(mean, rstd, Ci, gb.data_ptr(), 2 * Ci, Ci),
                             pro_act=L.ACT_LEAKY, pro_slope=0.2, res=rs[i], alpha=0.7, stats_key=f"pair.{group}.{i}",
                             splitk=sks[i], collect=grp if group else None)
            ys.append(y)
            sts.append(st)
        if group:
            arr = (L.ConvArgs * 2)(*grp)
            n = eng.lib.stzs_conv1d_group(arr, 2, eng.stream())
            assert n == (1 if pair else 2), n
            eng._finalize_group([st[0].ref for st in sts])
        torch.cuda.synchronize()
        tens = lambda v: (v.tensor() if hasattr(v, "tensor") else v).clone()
        return [y.t.clone() for y in ys], [(tens(st[0]), tens(st[1])) for st in sts]

    y0, s0 = run(False)
    y1, s1 = run(True)
    for a, b in zip(y0, y1):
        assert torch.equal(a, b)
    for (m0, r0), (m1, r1) in zip(s0, s1):
        assert torch.equal(m0, m1) and torch.equal(r0, r1)
