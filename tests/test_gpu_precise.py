"""Precise (parity) mode vs the fp32 oracle: the north-star "mel-L1 <= 1e-3 vs CPU reference".

bf16 storage cannot meet that bound (rounding the decoder weights to bf16 ALONE moves the oracle's own
log-mel by 1.3e-2 L1).  Precise mode keeps fp32 activations and computes every conv / linear on
split bf16 operands (hi*hi + hi*lo + lo*hi, csrc/conv.hip conv_x3, STZS_CONV_W_X3), the LSTM recurrences the
same way (csrc/lstm.hip, stzs_lstm_args.precise) and the attention the same way (csrc/attn.hip attn_x3):
StyleTTSZS(precise_decoder=True) for the decoder, StyleTTSZS(precise=True) for the whole pipeline.
tools/precision_probe.py emulates exactly this arithmetic on the oracle: end-to-end log-mel L1 2.2e-4.
Stated tolerances: conv_f32 / conv_x3 kernels max-abs 2e-5 / 4e-5 of max|ref| vs fp64 (accumulation order; the
split drops al*bl, ~2^-16 relative per product); precise LSTM 1e-5 rel-L2 (measured 5e-6), split-operand attention 1.2e-5 rel-L2 (measured 6e-6) vs fp64;
teacher-forced decoder log-mel L1 <= 1e-3 (north star) and waveform rel-L2 <= 1e-3; END TO END (configs[1]
inputs at v0, and a 4-utterance 2-step batch) log-mel L1 <= 1e-3 (north star), prompt codes teacher-forced
(the bf16 front end's output is a discrete decision, as durations elsewhere).
"""
import ctypes as C
import math

import pytest
import torch
import torch.nn.functional as F

from refops import max_rel, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,T,Ci,Co,k,dil,stride,ups", [(2, 300, 96, 80, 3, 1, 1, 0), (1, 1000, 128, 128, 11, 5, 1, 0),
                                                       (2, 2401, 22, 32, 12, 1, 6, 0), (1, 257, 1090, 256, 3, 1, 1, 0),
                                                       (2, 100, 256, 128, 0, 1, 1, 6)])
def test_conv_f32_kernel(gpu_device, B, T, Ci, Co, k, dil, stride, ups):
    from stzs import _lib as L
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import Arena, pack_conv
    eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(B * T + Ci)
    x = torch.randn(B, T, Ci, generator=g)
    A = Arena()
    if ups:
        w = torch.randn(Ci, Co, 2 * ups, generator=g) / math.sqrt(Ci * 2)
        b = torch.randn(Co, generator=g) * 0.1
        cw = pack_conv(A, "t", w, b, ups=ups, f32=True)
        ref = F.conv_transpose1d(F.leaky_relu(x.transpose(1, 2), 0.1), w, b, stride=ups,
                                 padding=(2 * ups - ups) // 2).transpose(1, 2)
    else:
        w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
        b = torch.randn(Co, generator=g) * 0.1
        pad = dil * (k - 1) // 2 if stride == 1 else (stride + 1) // 2
        cw = pack_conv(A, "t", w, b, f32=True)
        ref = F.conv1d(F.leaky_relu(x.transpose(1, 2), 0.1), w, b, stride=stride, padding=pad,
                       dilation=dil).transpose(1, 2)
    A.finalize(gpu_device)
    cw.w, cw.w32 = A[cw.w], A[cw.w32]
    cw.b = A[cw.b]
    ld = (Ci + 7) // 8 * 8
    xt = torch.zeros(B, T, ld, device=gpu_device)
    xt[:, :, :Ci] = x.to(gpu_device)
    To = ref.shape[1]
    y = Act(torch.zeros(B, To, (Co + 7) // 8 * 8, device=gpu_device), 0, Co)
    if ups:
        eng.conv(cw, Act(xt, 0, Ci), y, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=(2 * ups - ups) // 2,
                 T_final=T * ups, what="f32")
    else:
        eng.conv(cw, Act(xt, 0, Ci), y, pad=pad, dil=dil, stride=stride, pro_act=L.ACT_LEAKY, pro_slope=0.1,
                 what="f32")
    out = y.t[:, :, :Co].cpu()
    e = max_rel(out, ref)
    print("conv_f32", B, T, Ci, Co, k, dil, stride, ups, e)
    assert e < 2e-5


def _decode_tf_precise(eng, S, P, B, T40, seed=5):
    from oracle import stzs_ref as R
    g = torch.Generator().manual_seed(seed)
    asr = torch.randn(B, T40, S.d_txt, generator=g)
    F0 = 100 + 150 * torch.rand(B, 2 * T40, generator=g)
    F0[:, :4] = 0.0
    Nn = torch.randn(B, 2 * T40, generator=g)
    codes = torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3
    seeds = list(range(100, 100 + B))
    wav_ref = R.decode(P, S, asr, F0, Nn, codes, seeds)
    enc_in = eng.act("dec.enc_in", B, T40, S.d_txt + 2, eng.dec_dt)
    enc_in.t[:, :, :S.d_txt] = asr.to(eng.device)
    pro = dict(asr_buf=enc_in, F0=F0.to(eng.device), N=Nn.to(eng.device), T40=T40)
    wav = eng.decode(pro, codes.to(eng.device), seeds).cpu()
    return wav, wav_ref


@pytest.mark.parametrize("spec,B,T40", [("tiny", 2, 20), ("v0", 2, 40)])
def test_precise_decoder_mel_l1(gpu_device, spec, B, T40):
    from stzs.engine import StyleTTSZS
    from stzs.frontend import log_mel
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY, SPEC_V0
    S = SPEC_TINY if spec == "tiny" else SPEC_V0
    P = init_params(S, seed=0)
    eng = StyleTTSZS(S, P, device=gpu_device, precise_decoder=True)
    wav, ref = _decode_tf_precise(eng, S, P, B, T40)
    ml = (log_mel(wav, S) - log_mel(ref, S)).abs().mean().item()
    e = rel_err(wav, ref)
    print(f"precise decoder {spec}: log-mel L1 {ml:.3e}, waveform rel-L2 {e:.3e}")
    assert torch.isfinite(wav).all()
    assert ml <= 1e-3
    assert e <= 1e-3


@pytest.mark.parametrize("B,T,Ci,Co,k,dil,stride,ups,act", [
    (2, 300, 96, 80, 3, 1, 1, 0, "leaky"), (1, 1000, 128, 128, 11, 5, 1, 0, "snake"),
    (2, 2401, 22, 32, 12, 1, 6, 0, "leaky"), (1, 257, 1090, 256, 3, 1, 1, 0, "none"),
    (2, 100, 256, 128, 0, 1, 1, 6, "leaky"), (3, 50, 512, 1536, 1, 1, 1, 0, "none")])
def test_conv_x3_kernel(gpu_device, B, T, Ci, Co, k, dil, stride, ups, act):
    """split-operand conv vs an fp64 torch reference of the same conv (prologue in fp64 too)."""
    from stzs import _lib as L
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import Arena, pack_conv
    eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(B * T + Ci + 7)
    x = torch.randn(B, T, Ci, generator=g)
    alpha = 0.5 + torch.rand(Ci, generator=g)
    xd = x.double().transpose(1, 2)
    if act == "leaky":
        xa = F.leaky_relu(xd, 0.1)
    elif act == "snake":
        a_ = alpha.double()[None, :, None]
        xa = xd + torch.sin(a_ * xd) ** 2 / a_
    else:
        xa = xd
    A = Arena()
    if ups:
        w = torch.randn(Ci, Co, 2 * ups, generator=g) / math.sqrt(Ci * 2)
        b = torch.randn(Co, generator=g) * 0.1
        cw = pack_conv(A, "t", w, b, ups=ups, x3=True)
        ref = F.conv_transpose1d(xa, w.double(), b.double(), stride=ups, padding=(2 * ups - ups) // 2).transpose(1, 2)
    else:
        w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
        b = torch.randn(Co, generator=g) * 0.1
        pad = dil * (k - 1) // 2 if stride == 1 else (stride + 1) // 2
        cw = pack_conv(A, "t", w, b, x3=True)
        ref = F.conv1d(xa, w.double(), b.double(), stride=stride, padding=pad, dilation=dil).transpose(1, 2)
    A.add("alpha", alpha)
    A.finalize(gpu_device)
    cw.w, cw.wx3, cw.b = A[cw.w], A[cw.wx3], A[cw.b]
    cw.fx3 = None  # (this test is the LDS-ring conv_x3 form; the register-direct one: test_mrfx_*)
    ld = (Ci + 7) // 8 * 8
    xt = torch.zeros(B, T, ld, device=gpu_device)
    xt[:, :, :Ci] = x.to(gpu_device)
    To = ref.shape[1]
    y = Act(torch.zeros(B, To, (Co + 7) // 8 * 8, device=gpu_device), 0, Co)
    pa = {"leaky": L.ACT_LEAKY, "snake": L.ACT_SNAKE, "none": L.ACT_NONE}[act]
    kw = dict(pro_act=pa, pro_slope=0.1, pro_alpha=A["alpha"] if act == "snake" else None, what="x3")
    if ups:
        eng.conv(cw, Act(xt, 0, Ci), y, ups_pad=(2 * ups - ups) // 2, T_final=T * ups, **kw)
    else:
        eng.conv(cw, Act(xt, 0, Ci), y, pad=pad, dil=dil, stride=stride, **kw)
    out = y.t[:, :, :Co].cpu().double()
    e = max_rel(out, ref)
    print("conv_x3", B, T, Ci, Co, k, dil, stride, ups, act, f"{e:.2e}")
    assert e < 4e-5


# the precise register-direct conv (csrc/mrfx.hip, STZS_CONV_W_FRAG32X3): B, T, Ci, Co, k, dil, act, residual,
# accumulate, statistics, res_tdiv -- stage-1 shapes (one 128-channel chunk; 128-row tiles up to a 146-row halo, 64-row
# tiles beyond: k7 d5, k11 d3 / d5), stage-0 shapes (two chunks), the AdaIN-block k3 forms (LeakyReLU / identity,
# Ci 1090 = 9 chunks with Ci < ci_pad, x2 shortcut residual), ragged last tiles, Co < co_pad
MRFX_CASES = [
    (3, 1000, 128, 128, 3, 1, "snake", False, False, True, 1),
    (2, 777, 128, 128, 7, 3, "snake", True, False, True, 1),     # 146-row halo: the largest 128-row tile
    (2, 1001, 128, 128, 7, 5, "snake", True, True, False, 1),    # 64-row tiles, residual + accumulate
    (2, 500, 128, 128, 11, 5, "snake", False, False, True, 1),   # 64-row tiles, 178-row halo -> 114
    (3, 333, 128, 128, 11, 1, "snake", True, True, True, 1),
    (2, 400, 256, 256, 11, 3, "snake", True, False, True, 1),    # stage-0 width: 2 chunks, 64-row tiles
    (2, 400, 256, 256, 3, 1, "snake", True, True, True, 1),
    (1, 129, 256, 176, 7, 1, "snake", False, False, True, 1),    # ragged: 1 valid row in the 2nd tile; Co < co_pad
    (3, 400, 1090, 256, 3, 1, "leaky", True, False, True, 2),    # decoder block conv2: 9 chunks, x2 shortcut
    (2, 300, 130, 64, 3, 1, "none", False, False, True, 1),      # up-block conv1 after the dw-ConvT: no prologue
]


@pytest.mark.parametrize("case", MRFX_CASES)
def test_mrfx_kernel(gpu_device, case):
    """the precise register-direct conv (csrc/mrfx.hip) with the AdaIN + Snake / LeakyReLU / identity prologue,
    residual (at t / res_tdiv) / alpha / accumulate epilogue and fused statistics vs an fp64 torch reference of the
    same conv (prologue in fp64 too): max-abs 4e-5 of max|ref| (the conv_x3 bound: split products drop al*bl, ~2^-16
    relative each; the Snake's hardware sine is fp32-level); statistics of the stored fp32 output 1e-5.  Also against
    conv_x3 on the same operands (same arithmetic, another K order): 4e-5."""
    from stzs import _lib as L
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import Arena, pack_conv
    B, T, Ci, Co, k, dil, act, hr, ha, st, tdiv = case
    eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(B * T + Ci + k + dil)
    pad = dil * (k - 1) // 2
    x = torch.randn(B, T, Ci, generator=g)
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    mean = torch.randn(B, Ci, generator=g) * 0.1
    rstd = torch.rand(B, Ci, generator=g) + 0.5
    gb = torch.randn(B, 2 * Ci, generator=g) * 0.2
    alpha = torch.rand(Ci, generator=g) + 0.5
    res = torch.randn(B, (T + tdiv - 1) // tdiv, Co, generator=g) if hr else None
    acc = torch.randn(B, T, Co, generator=g) if ha else None
    osc = 1 / 3 if ha else (0.7071 if hr else 1.0)
    xd = x.double().transpose(1, 2)
    if act != "none":
        sc = ((1 + gb[:, :Ci].double()) * rstd.double())[:, :, None]
        xd = xd * sc + (gb[:, Ci:].double()[:, :, None] - mean.double()[:, :, None] * sc)
    if act == "snake":
        a_ = alpha.double()[None, :, None]
        xd = xd + torch.sin(a_ * xd) ** 2 / a_
    elif act == "leaky":
        xd = F.leaky_relu(xd, 0.2)
    ref = F.conv1d(xd, w.double(), b.double(), padding=pad, dilation=dil).transpose(1, 2)
    if hr:
        ref = ref + res.double().repeat_interleave(tdiv, 1)[:, :T]
    ref = ref * osc
    if ha:
        ref = ref + acc.double()
    A = Arena()
    cw = pack_conv(A, "t", w, b, frag32=True, x3=True)
    A.finalize(gpu_device)
    cw.w, cw.wx3, cw.fx3, cw.b = A[cw.w], A[cw.wx3], A[cw.fx3], A[cw.b]
    ld = (Ci + 7) // 8 * 8
    xt = torch.zeros(B, T, ld, device=gpu_device)
    xt[:, :, :Ci] = x.to(gpu_device)
    keep = [mean.to(gpu_device), rstd.to(gpu_device), gb.to(gpu_device), alpha.to(gpu_device)]
    pro = None if act == "none" else (keep[0], keep[1], Ci, keep[2].data_ptr(), 2 * Ci, Ci)
    pa = {"snake": L.ACT_SNAKE, "leaky": L.ACT_LEAKY, "none": L.ACT_NONE}[act]
    outs = []
    for mrfx in (True, False):
        eng.mrfx = mrfx
        y = Act(torch.zeros(B, T, Co, device=gpu_device))
        rd = Act(res.to(gpu_device)) if hr else None
        ad = Act(acc.to(gpu_device)) if ha else None
        n0 = eng.launches
        o = eng.conv(cw, Act(xt, 0, Ci), y, pad=pad, dil=dil, pro=pro, pro_act=pa, pro_slope=0.2,
                     pro_alpha=keep[3] if act == "snake" else None, res=rd, res_tdiv=tdiv, alpha=osc, acc_in=ad,
                     beta=1.0, stats_key="t.mrfx" if st else None, what="mrfx")
        torch.cuda.synchronize()
        outs.append((y.t.double().cpu(), (o[1][0].clone().cpu(), o[1][1].clone().cpu()) if st else None))
    got, stats = outs[0]
    e = max_rel(got, ref)
    e_x3 = max_rel(got, outs[1][0])
    print("mrfx", case, f"max-rel vs fp64 {e:.2e}, vs conv_x3 {e_x3:.2e}")
    assert e < 4e-5 and e_x3 < 4e-5
    if st:
        m, r = stats
        mr, vr = got.mean(1), got.var(1, unbiased=False)
        assert float(((m.double() - mr).abs() / (mr.abs() + vr.sqrt())).max()) < 1e-5
        assert max_rel(r.double(), 1 / torch.sqrt(vr + 1e-5)) < 1e-5


@pytest.mark.parametrize("B,T", [(2, 3001), (1, 24001), (3, 130)])
def test_mrfx_conv_post(gpu_device, B, T):
    """conv_post (LeakyReLU(0.01), 128 -> 22, k7, fp32 out) on the narrow precise form (csrc/mrfx.hip NW: waves split
    the rows, masked stores past Co = 22 -- the two padding columns of the row pitch 24 stay untouched) vs fp64 and vs
    conv_x3: max-abs 4e-5 of max|ref|."""
    from stzs import _lib as L
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import Arena, pack_conv
    eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(B * T)
    Ci, Co, k = 128, 22, 7
    x = torch.randn(B, T, Ci, generator=g)
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv1d(F.leaky_relu(x.double().transpose(1, 2), 0.01), w.double(), b.double(), padding=3).transpose(1, 2)
    A = Arena()
    cw = pack_conv(A, "t", w, b, narrow32=True, x3=True)
    A.finalize(gpu_device)
    cw.w, cw.wx3, cw.fx3, cw.b = A[cw.w], A[cw.wx3], A[cw.fx3], A[cw.b]
    outs = []
    for mrfx in (True, False):
        eng.mrfx = mrfx
        yb = torch.full((B, T, 24), 7.0, device=gpu_device)
        eng.conv(cw, Act(x.to(gpu_device)), Act(yb, 0, Co), pad=3, pro_act=L.ACT_LEAKY, pro_slope=0.01,
                 what="conv_post")
        torch.cuda.synchronize()
        assert bool((yb[:, :, Co:] == 7.0).all()), "columns past Co written"
        outs.append(yb[:, :, :Co].double().cpu())
    e, e_x3 = max_rel(outs[0], ref), max_rel(outs[0], outs[1])
    print("mrfx conv_post", B, T, f"max-rel vs fp64 {e:.2e}, vs conv_x3 {e_x3:.2e}")
    assert e < 4e-5 and e_x3 < 4e-5


# FLAT linears of the precise pipeline (csrc/mrfx.hip mrfx_lin): rows, T per utterance, K, N, epilogue act, gate,
# residual (broadcast over utterances = the positional table), accumulate, cscale
MRFX_LIN_CASES = [
    (6400, 50, 512, 1536, "none", False, False, False, 1.0),   # qkv at batch 64 (CFG-doubled)
    (6400, 50, 2048, 512, "none", True, True, False, 1.0),     # ff2: K 2048 (16 chunks), gate + residual
    (300, 50, 512, 2048, "gelu", False, False, False, 1.0),    # ff1 (300 rows: a ragged last tile)
    (100, 50, 256, 512, "none", False, "bcast", False, 0.37),  # dn.in: cscale = c_in, the positional rows as residual
    (250, 50, 512, 256, "none", False, False, True, 1.0),      # dn.out: alpha c_out, beta c_skip accumulate
    (173, 173, 640, 2048, "none", False, False, False, 1.0),   # an LSTM input projection (In 640 = 5 chunks), T 173
    (64, 1, 128, 600, "silu", False, False, False, 1.0),       # a per-utterance linear (one row each), Co % 128 != 0
]


@pytest.mark.parametrize("case", MRFX_LIN_CASES)
def test_mrfx_linear(gpu_device, case):
    """the precise FLAT linear (csrc/mrfx.hip mrfx_lin: split bf16 operands, fp32 rows in and out, the next chunk's rows
    in flight during the K loop) vs an fp64 torch reference: max-abs 4e-5 of max|ref| (the conv_x3 bound)."""
    from stzs import _lib as L
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    from stzs.weights import Arena, pack_conv
    R, T, K, N, act, gated, res, acc, cs = case
    B = R // T
    eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, seed=0), device=gpu_device)
    g = torch.Generator().manual_seed(R + K + N)
    x = torch.randn(B, T, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g) * 0.1
    gate = torch.rand(B, N, generator=g) + 0.5
    rv = torch.randn(1 if res == "bcast" else B, T, N, generator=g) if res else None
    av = torch.randn(B, T, N, generator=g) if acc else None
    ref = (x.double() * cs) @ w.double().t() + b.double()
    if act == "gelu":
        ref = F.gelu(ref)
    elif act == "silu":
        ref = F.silu(ref)
    if gated:
        ref = ref * gate.double()[:, None, :]
    if res:
        ref = ref + rv.double()
    alpha, beta = (0.75, 1.25) if acc else (1.0, 0.0)
    ref = ref * alpha
    if acc:
        ref = ref + beta * av.double()
    A = Arena()
    cw = pack_conv(A, "t", w, b, x3=True)
    A.finalize(gpu_device)
    cw.w, cw.wx3, cw.fx3, cw.b = A[cw.w], A[cw.wx3], A[cw.fx3], A[cw.b]
    outs = []
    for mrfx in (True, False):
        eng.mrfx = mrfx
        y = Act(torch.zeros(B, T, (N + 7) // 8 * 8, device=gpu_device), 0, N)
        gd = gate.to(gpu_device)
        eng.conv(cw, Act(x.to(gpu_device)), y, cscale=cs,
                 epi_act={"none": L.ACT_NONE, "gelu": L.ACT_GELU, "silu": L.ACT_SILU}[act],
                 gate=gd.data_ptr() if gated else None, gate_bs=N, res=Act(rv.to(gpu_device)) if res else None,
                 acc_in=Act(av.to(gpu_device)) if acc else None, alpha=alpha, beta=beta, what="mrfx_lin")
        torch.cuda.synchronize()
        outs.append(y.t[:, :, :N].double().cpu())
    e, e_x3 = max_rel(outs[0], ref), max_rel(outs[0], outs[1])
    print("mrfx_lin", case, f"max-rel vs fp64 {e:.2e}, vs conv_x3 {e_x3:.2e}")
    assert e < 4e-5 and e_x3 < 4e-5


def test_mrfx_is_the_precise_path(gpu_device):
    """the precise engine routes its FRAG32 convs to the register-direct split-operand kernel: a stage-1 MRF conv shape
    returns STZS_OK through STZS_CONV_W_FRAG32X3, and the form refuses bf16 operands (ESHAPE before any launch)."""
    from stzs import _lib as L
    lib = L.load()
    a = L.ConvArgs()
    x = torch.zeros(1, 300, 128, device=gpu_device)
    y = torch.zeros(1, 300, 128, device=gpu_device)
    wt = torch.zeros(3 * 4 * 1024 * 8, dtype=torch.bfloat16, device=gpu_device)
    a.x, a.w, a.y = x.data_ptr(), wt.data_ptr(), y.data_ptr()
    a.ldx, a.bsx, a.ldy, a.bsy = 128, 300 * 128, 128, 300 * 128
    a.B, a.T_in, a.T_out, a.Ci, a.Co, a.ks, a.dil, a.stride, a.pad = 1, 300, 300, 128, 128, 3, 1, 1, 1
    a.ci_pad, a.co_pad, a.cic, a.in_dtype, a.out_dtype = 128, 128, 128, L.F32, L.F32
    a.pro_act, a.pro_cscale, a.alpha, a.flags = L.ACT_NONE, 1.0, 1.0, L.CONV_W_FRAG32X3
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.stzs_conv1d(C.byref(a), s) == L.OK
    torch.cuda.synchronize()
    a.in_dtype = L.BF16
    assert lib.stzs_conv1d(C.byref(a), s) == L.ESHAPE


def _lstm_ref64(x, P, name):
    """fp64 torch BiLSTM with the named parameters (the oracle's nn.LSTM, in double)."""
    H = P[name + ".w_hh"].shape[1]
    m = torch.nn.LSTM(x.shape[-1], H, num_layers=1, batch_first=True, bidirectional=True).double()
    with torch.no_grad():
        for a_, b_ in (("weight_ih_l0", ".w_ih"), ("weight_hh_l0", ".w_hh"), ("bias_ih_l0", ".b_ih"),
                       ("bias_hh_l0", ".b_hh"), ("weight_ih_l0_reverse", ".w_ih_rev"),
                       ("weight_hh_l0_reverse", ".w_hh_rev"), ("bias_ih_l0_reverse", ".b_ih_rev"),
                       ("bias_hh_l0_reverse", ".b_hh_rev")):
            getattr(m, a_).copy_(P[name + b_].double())
        return m(x.double())[0]


@pytest.fixture(scope="module")
def v0_precise(gpu_device):
    from stzs.engine import StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    torch.set_num_threads(16)
    P = init_params(SPEC_V0, seed=0)
    return SPEC_V0, P, StyleTTSZS(SPEC_V0, P, device=gpu_device, precise=True)


@pytest.mark.parametrize("name,B,T", [("pr.shared", 3, 120), ("te.lstm", 1, 80)])
def test_lstm_precise(v0_precise, name, B, T):
    from stzs.engine import Act
    S, P, eng = v0_precise
    lw = eng.W.pr_shared if name == "pr.shared" else eng.W.te_lstm
    In = P[name + ".w_ih"].shape[1]
    g = torch.Generator().manual_seed(T)
    x = torch.randn(B, T, In, generator=g)
    xt = torch.zeros(B, T, (In + 7) // 8 * 8, device=eng.device)
    xt[:, :, :In] = x.to(eng.device)
    y = eng.act("t.lstm.y", B, T, 2 * lw.H, torch.float32)
    eng.lstm(lw, Act(xt, 0, In), y, "t.lstm")
    out = y.t[:, :, :2 * lw.H].cpu().double()
    ref = _lstm_ref64(x, P, name)
    e = rel_err(out, ref)
    print(f"precise LSTM {name} B {B} T {T}: rel-L2 {e:.2e}, status {eng.check_status()}")
    assert e < 1e-5


def test_attention_precise(gpu_device):
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    eng = object.__new__(StyleTTSZS)  # only .spec / .lib / launch plumbing are used by attention()
    eng.spec, eng.device, eng.launches = S, torch.device(gpu_device), 0
    from stzs import _lib as L
    eng.lib = L.load()
    R, Lq, Lk, D = 4, 50, 173, S.dn_heads * S.dn_head_dim
    g = torch.Generator().manual_seed(11)
    q, k, v = (torch.randn(R, n, D, generator=g) for n in (Lq, Lk, Lk))
    o = torch.zeros(R, Lq, D, device=gpu_device)
    eng.attention(Act(q.to(gpu_device)), Act(k.to(gpu_device)), Act(v.to(gpu_device)), Act(o))
    h = S.dn_heads
    qd, kd, vd = (t.double().view(R, -1, h, D // h).transpose(1, 2) for t in (q, k, v))
    ref = (torch.softmax(qd @ kd.transpose(-1, -2) / math.sqrt(D // h), -1) @ vd).transpose(1, 2).reshape(R, Lq, D)
    e = rel_err(o.cpu().double(), ref)
    print(f"split-operand attention: rel-L2 {e:.2e}")
    assert e < 1.2e-5


def _logmel_l1(a, b, S):
    from oracle import stzs_ref as R
    return (R.log_mel(a, S) - R.log_mel(b, S)).abs().mean().item()


@pytest.mark.parametrize("case", ["configs1", "batch4"])
def test_precise_end_to_end_mel_l1(v0_precise, case):
    """the north-star bound END TO END: a whole precise synth() vs the fp32 oracle (prompt codes teacher-forced)."""
    import bench
    from oracle import stzs_ref as R
    S, P, eng = v0_precise
    if case == "configs1":
        tok, ref, eps, dur = bench.make_inputs(S, 1, seed=1000)
        steps, seeds = bench.STEPS_LATENCY, [7]
    else:
        tok, ref, eps, dur, seeds = bench.rank_inputs(S, 4, 0)
        steps = bench.STEPS_THROUGHPUT
    out = eng.synth(tok, ref, steps=steps, cfg_scale=bench.CFG, noise=eps, durations=dur, seeds=seeds)
    eng.check_status()
    o = R.synth(P, S, tok, ref, steps, bench.CFG, eps, dur, seeds=seeds, prompt_idx=out["prompt_idx"].cpu())
    e_h = rel_err(out["h_txt"].t[:, :, :S.d_txt].cpu(), o["h_txt"])
    e_c, e_f0 = rel_err(out["codes"].cpu(), o["codes"]), rel_err(out["F0"].cpu(), o["F0"])
    e_w, m_w = rel_err(out["wav"].cpu(), o["wav"]), _logmel_l1(out["wav"].cpu(), o["wav"], S)
    print(f"precise e2e {case}: text {e_h:.2e} codes {e_c:.2e} F0 {e_f0:.2e} wav {e_w:.2e} log-mel L1 {m_w:.3e}")
    assert torch.equal(out["dur"].cpu(), o["dur"].to(out["dur"].dtype))
    assert m_w <= 1e-3


def test_precise_batch64_rows(v0_precise):
    """the bench's precise leg exactly (bench.precise_mode: B = 64, make_inputs(S, 64, 7), 2-step CFG 5, seeds 0..63):
    rows 0 / 31 / 63 of the 64-utterance batch are BIT-IDENTICAL to the same utterances synthesized alone (the
    multi-row hi | lo LSTM exchange, the flat-row split-operand GEMM tiles and the per-utterance statistics keep rows
    independent), and rows 0, 31 and 63 each meet the north-star log-mel L1 <= 1e-3 against the fp32 oracle."""
    import bench
    from oracle import stzs_ref as R
    S, P, eng = v0_precise
    Bb = 64
    tok, ref, eps, dur = bench.make_inputs(S, Bb, 7)
    out = eng.synth(tok, ref, steps=bench.STEPS_THROUGHPUT, cfg_scale=bench.CFG, noise=eps, durations=dur,
                    seeds=list(range(Bb)))
    keep = {k: out[k].detach().clone().cpu() for k in ("wav", "codes", "F0", "prompt_idx")}
    for r in (0, 31, 63):
        o1 = eng.synth(tok[r:r + 1], ref[r:r + 1], steps=bench.STEPS_THROUGHPUT, cfg_scale=bench.CFG,
                       noise=eps[r:r + 1], durations=dur[r:r + 1], seeds=[r])
        for k in ("prompt_idx", "codes", "F0", "wav"):
            assert torch.equal(o1[k].cpu(), keep[k][r:r + 1]), (r, k)
    for r in (0, 31, 63):
        o = R.synth(P, S, tok[r:r + 1], ref[r:r + 1], bench.STEPS_THROUGHPUT, bench.CFG, eps[r:r + 1], dur[r:r + 1],
                    seeds=[r], prompt_idx=keep["prompt_idx"][r:r + 1])
        m_w = _logmel_l1(keep["wav"][r:r + 1], o["wav"], S)
        print(f"precise B=64 row {r}: codes {rel_err(keep['codes'][r:r + 1], o['codes']):.2e} log-mel L1 {m_w:.3e}")
        assert m_w <= 1e-3, r
