"""XCD-aware tile order of the LDS-DMA linear GEMM (csrc/conv.hip gemm_glds): the remapped launch is bit-identical to
the dispatcher's linear order (STZS_CONV_LINEAR_IDS) and matches a plain-torch fp32 restatement, at the batch-64
row counts of the denoiser (3 200 / 6 400 CFG rows, 64- and 128-row tiles, grids not a multiple of 8) and with
in-launch split-K."""
import math

import pytest
import torch
import torch.nn.functional as F

from refops import bf, max_rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    return StyleTTSZS(tiny, tiny_params, device=gpu_device)


def _pack(w, b):
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "t", w, b)
    A.finalize("cuda:0")
    cw.w = A[cw.w]
    cw.b = A[cw.b] if cw.b is not None else None
    return cw, A


def _act(t):
    from stzs.engine import Act
    return Act(t, 0, t.shape[-1])


@pytest.mark.parametrize("R,Ci,Co,splitk", [(64, 512, 2048, 0), (128, 512, 1536, 0), (64, 2048, 512, 0),
                                            (128, 512, 512, 0), (83, 512, 1024, 0), (64, 2048, 512, 4),
                                            (2, 512, 2048, 2)])
def test_gemm_xcd_order_bit_identical(eng, R, Ci, Co, splitk):
    from stzs import _lib as L
    g = torch.Generator().manual_seed(R * 7 + Ci + Co + splitk)
    Lr = 50
    x = bf(torch.randn(R, Lr, Ci, generator=g))
    w = torch.randn(Co, Ci, generator=g) / math.sqrt(Ci)
    b = torch.randn(Co, generator=g) * 0.1
    cw, _A = _pack(w, b)
    xd = x.to(torch.bfloat16).cuda()
    ys = []
    for flags in (0, L.CONV_LINEAR_IDS):
        y = torch.zeros(R, Lr, Co, dtype=torch.bfloat16, device="cuda:0")
        eng.conv(cw, _act(xd), _act(y), epi_act=L.ACT_GELU, splitk=splitk, flags=flags)
        torch.cuda.synchronize()
        ys.append(y)
    assert torch.equal(ys[0], ys[1])
    ref = F.gelu(x @ bf(w).t() + b)
    e = max_rel(ys[0].float().cpu(), ref)
    print("xcd gemm", R, Ci, Co, splitk, e)
    assert e < 1e-2


@pytest.mark.parametrize("R,T,Ci,Co,k", [(32, 200, 1090, 1024, 3), (8, 400, 256, 256, 3), (16, 80, 512, 512, 5),
                                         (3, 130, 80, 384, 1)])
def test_conv_mfma_xcd_order_bit_identical(eng, R, T, Ci, Co, k):
    """conv_mfma (k > 1 convs with a LeakyReLU prologue, and a 1x1 conv off the LDS-DMA path): the XCD-aware tile
    order is bit-identical to the linear order, and matches F.conv1d on the same bf16 operands."""
    from stzs import _lib as L
    from stzs.engine import Act
    g = torch.Generator().manual_seed(R + T + Ci + Co + k)
    x = bf(torch.randn(R, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "t", w, b)
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    ld = (Ci + 7) // 8 * 8
    xd = torch.zeros(R, T, ld, dtype=torch.bfloat16, device="cuda:0")
    xd[..., :Ci] = x.to(torch.bfloat16).cuda()
    ys = []
    for flags in (0, L.CONV_LINEAR_IDS):
        y = torch.zeros(R, T, Co, dtype=torch.bfloat16, device="cuda:0")
        pro = {} if k == 1 else dict(pro_act=L.ACT_LEAKY, pro_slope=0.2)
        eng.conv(cw, Act(xd, 0, Ci), _act(y), pad=k // 2, flags=flags, **pro)
        torch.cuda.synchronize()
        ys.append(y)
    assert torch.equal(ys[0], ys[1])
    xin = x if k == 1 else bf(F.leaky_relu(x, 0.2))
    ref = F.conv1d(xin.transpose(1, 2), bf(w), b, padding=k // 2).transpose(1, 2)
    e = max_rel(ys[0].float().cpu(), ref)
    print("xcd conv", R, T, Ci, Co, k, e)
    assert e < 1e-2


SPLITK_CASES = [  # (B, T, Ci, Co, k, epilogue): the text-encoder shape, then T_out > 128 (several row tiles per
    # utterance) with a residual, fused statistics, accumulate into a separate buffer and in place, a 1x1 conv
    (3, 80, 512, 512, 5, "plain"),
    (3, 300, 512, 256, 3, "res"),
    (3, 300, 512, 256, 3, "stats"),
    (3, 300, 512, 256, 3, "acc"),
    (3, 300, 512, 256, 3, "acc_inplace"),
    (2, 200, 512, 384, 1, "leaky"),  # 1x1 with a prologue: conv_mfma, not the LDS-DMA GEMM
    # the decoder conv1 input width (1090 -> 9 chunks: uneven slices 4 | 5 and 2 | 2 | 2 | 3), statistics + prologue
    (2, 200, 1090, 256, 3, "stats"),
    (1, 200, 1090, 256, 3, "leaky"),
]


@pytest.mark.parametrize("splitk", [2, 4, 16])
@pytest.mark.parametrize("case", SPLITK_CASES, ids=lambda c: f"B{c[0]}-T{c[1]}-k{c[4]}-{c[5]}")
def test_conv_mfma_splitk(eng, splitk, case):
    """conv_mfma in-launch split-K over input-channel chunks (the latency engine's text-encoder k5 convs,
    LATENCY_TE_SPLITK) through the last arriver's full epilogue (residual, alpha / beta accumulate incl. y == acc_in,
    fused InstanceNorm statistics partials), T_out > 128 and a 1x1 conv: matches F.conv1d on the same bf16 operands,
    utterance 0 of a B-utterance launch is bit-identical to the 1-utterance launch (per-utterance tiles:
    batch-invariant), a re-run is bit-identical (the self-resetting tile tickets), and the result is within fp32
    re-association of the unsplit conv (statistics included).  splitk 16 = one chunk per slice (the engine clamps to
    the chunk count): the DEEP form where the slice's K-steps fit LDS, its partials combined by the second launch
    splitk_epi -- outputs bit-identical to the 3-slot ring form (STZS_CONV_RING) and to the last-arriver combine
    (STZS_CONV_SK_TICKET) at the same slice count."""
    from stzs import _lib as L
    from stzs.engine import Act
    from stzs.weights import Arena, pack_conv
    B, T, Ci, Co, k, epi = case
    g = torch.Generator().manual_seed(100 + splitk + T + k)
    x = bf(torch.randn(B, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    r = bf(torch.randn(B, T, Co, generator=g))
    acc = bf(torch.randn(B, T, Co, generator=g))
    A = Arena()
    cw = pack_conv(A, "t", w, b)
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    xd = torch.zeros(B, T, (Ci + 7) // 8 * 8, dtype=torch.bfloat16, device="cuda:0")  # rows 16-B aligned
    xd[:, :, :Ci] = x.to(torch.bfloat16).cuda()
    rd = r.to(torch.bfloat16).cuda()
    accd = acc.to(torch.bfloat16).cuda()
    alpha, beta = (0.7, 0.5) if epi.startswith("acc") else (1.0, 0.0)

    def run(n, sk, flags=0):
        xb = xd[:n].contiguous()
        a0 = accd[:n].clone()
        y = a0 if epi == "acc_inplace" else torch.zeros(n, T, Co, dtype=torch.bfloat16, device="cuda:0")
        kw = dict(pad=k // 2, splitk=sk, flags=flags)
        if epi == "leaky":
            kw.update(pro_act=L.ACT_LEAKY, pro_slope=0.2)
        if epi == "res":
            kw["res"] = _act(rd[:n].contiguous())
        if epi.startswith("acc"):
            kw.update(acc_in=_act(a0), alpha=alpha, beta=beta)
        if epi == "stats":
            kw["stats_key"] = f"t.sk{sk}.{n}"
        out = eng.conv(cw, Act(xb, 0, Ci), _act(y), **kw)
        torch.cuda.synchronize()
        st = None
        if epi == "stats":
            st = (out[1][0].clone(), out[1][1].clone())
        return y.clone(), st

    y3, s3 = run(B, splitk)
    y3b, s3b = run(B, splitk)
    y1, s1 = run(1, splitk)
    y0, s0 = run(B, 0)
    assert torch.equal(y3, y3b)
    assert torch.equal(y3[:1], y1)
    if splitk == 16:  # DEEP (where it fits) vs the ring form and vs the last-arriver combine: same slices, same K order,
        # same slice-order sum -> bit-identical outputs; statistics partials reduced in another order (fp32 association)
        for fl in (L.CONV_RING, L.CONV_SK_TICKET):
            yr, sr = run(B, splitk, fl)
            assert torch.equal(y3, yr), fl
            if epi == "stats":
                assert (s3[0] - sr[0]).abs().max().item() <= 1e-6 * (1 + s3[0].abs().max().item())
                assert max_rel(s3[1].cpu(), sr[1].cpu()) < 1e-5
    xin = bf(F.leaky_relu(x, 0.2)) if epi == "leaky" else x
    ref = F.conv1d(xin.transpose(1, 2), bf(w), b, padding=k // 2).transpose(1, 2)
    if epi == "res":
        ref = ref + r
    if epi.startswith("acc"):
        ref = ref * alpha + beta * acc
    e = max_rel(y3.float().cpu(), ref)
    e0 = max_rel(y3.float().cpu(), y0.float().cpu())
    print("conv split-K", case, splitk, e, "vs unsplit", e0)
    assert e < 1e-2 and e0 < 1e-2
    if epi == "stats":
        assert torch.equal(s3[0], s3b[0]) and torch.equal(s3[1], s3b[1])
        assert torch.equal(s3[0][:1], s1[0]) and torch.equal(s3[1][:1], s1[1])
        yf = y3.double().cpu()  # the statistics of the STORED bf16 output, in fp64
        m_ref = yf.mean(1)
        r_ref = 1.0 / torch.sqrt(yf.var(1, unbiased=False) + 1e-5)
        em = (s3[0].cpu().double() - m_ref).abs().max().item()
        er = max_rel(s3[1].cpu().double(), r_ref)
        eu = (s3[0] - s0[0]).abs().max().item(), max_rel(s3[1].cpu(), s0[1].cpu())
        print("   stats: mean abs err", em, "rstd rel err", er, "vs unsplit", eu)
        assert em < 1e-4 and er < 3e-4
        assert eu[0] < 1e-4 and eu[1] < 3e-4  # the unsplit conv's bf16 output differs by re-association roundings


@pytest.mark.parametrize("splitk", [1, 4, 16])
def test_conv_rejects_epilogue_act_as_prologue(eng, splitk):
    """the prologue activation is NONE / LEAKY / SNAKE; an epilogue-only activation (GELU, SILU) passed as
    pro_act is rejected with STZS_EINVAL before any launch (the DEEP / splitk_epi forms used to route it to the Snake
    template, which reads pro_alpha -- a null pointer here)."""
    from stzs import _lib as L
    from stzs.engine import Act
    from stzs.weights import Arena, pack_conv
    B, T, Ci, Co = 1, 80, 512, 512
    w = torch.randn(Co, Ci, 5) / math.sqrt(Ci * 5)
    A = Arena()
    cw = pack_conv(A, "t", w, torch.zeros(Co))
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    x = Act(torch.randn(B, T, Ci, device="cuda:0").to(torch.bfloat16))
    y = Act(torch.zeros(B, T, Co, dtype=torch.bfloat16, device="cuda:0"))
    for act in (L.ACT_GELU, L.ACT_SILU):
        with pytest.raises(L.StzsError, match="rc=-?[0-9]+"):
            eng.conv(cw, x, y, pad=2, splitk=splitk, pro_act=act)
    torch.cuda.synchronize()
