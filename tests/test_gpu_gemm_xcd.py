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


@pytest.mark.parametrize("splitk", [2, 4])
def test_conv_mfma_splitk(eng, splitk):
    """conv_mfma in-launch split-K over input-channel chunks (the latency engine's text-encoder k5 convs,
    LATENCY_TE_SPLITK): matches F.conv1d on the same bf16 operands, utterance 0 of a 3-utterance launch is
    bit-identical to the 1-utterance launch (per-utterance tiles: batch-invariant), a re-run is bit-identical (the
    self-resetting tile tickets), and the result is within fp32 re-association of the unsplit conv."""
    from stzs import _lib as L
    from stzs.engine import Act
    from stzs.weights import Arena, pack_conv
    T, Ci, Co, k = 80, 512, 512, 5
    g = torch.Generator().manual_seed(100 + splitk)
    x = bf(torch.randn(3, T, Ci, generator=g))
    w = torch.randn(Co, Ci, k, generator=g) / math.sqrt(Ci * k)
    b = torch.randn(Co, generator=g) * 0.1
    A = Arena()
    cw = pack_conv(A, "t", w, b)
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    xd = x.to(torch.bfloat16).cuda()

    def run(xb, sk):
        y = torch.zeros(xb.shape[0], T, Co, dtype=torch.bfloat16, device="cuda:0")
        eng.conv(cw, Act(xb, 0, Ci), _act(y), pad=k // 2, splitk=sk)
        torch.cuda.synchronize()
        return y

    y3 = run(xd, splitk)
    y3b = run(xd, splitk)
    y1 = run(xd[:1].contiguous(), splitk)
    y0 = run(xd, 0)
    assert torch.equal(y3, y3b)
    assert torch.equal(y3[:1], y1)
    ref = F.conv1d(x.transpose(1, 2), bf(w), b, padding=k // 2).transpose(1, 2)
    e = max_rel(y3.float().cpu(), ref)
    e0 = max_rel(y3.float().cpu(), y0.float().cpu())
    print("conv split-K", splitk, e, "vs unsplit", e0)
    assert e < 1e-2 and e0 < 1e-2
