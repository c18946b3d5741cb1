"""configs[4] fp8 denoiser linears (SURVEY.md §8 "Numerics": fp8 e4m3 denoiser linears): kernel parity.

  * stzs_quant_rows vs torch's e4m3fn conversion: codes and row scales BIT-exact;
  * stzs_row_layernorm with fp8 output vs torch LayerNorm + the same quantiser: scales within 1e-6,
    dequantised rows within 1 e4m3 step (rel 2^-3) of the fp32 LayerNorm;
  * gemm_glds<F8> (v_mfma_f32_16x16x32_fp8_fp8) vs a torch fp32 GEMM over the SAME dequantised
    operands: max-abs error <= 5e-5 of max|ref| (fp32 accumulation order only), bf16 output 8e-3;
  * the fp8 denoiser sampler vs the fp32 CPU oracle (quantisation error, stated bounds below).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from refops import max_rel, rel_err

pytestmark = pytest.mark.gpu
E4 = torch.float8_e4m3fn


def quant_ref(x):
    """the documented quantiser (include/stzs.h stzs_quant_rows), fp32 on the host: power-of-two row
    scale 2^k, the smallest with amax / 2^k <= 448, then RNE e4m3fn codes of x / 2^k."""
    amax = x.abs().amax(-1)
    m, e = torch.frexp(amax)
    k = torch.where(m <= 0.875, e - 9, e - 8)
    k = torch.where(amax > 0, k, torch.zeros_like(k))
    scale = torch.ldexp(torch.ones_like(amax), k)
    return (x / scale[..., None]).to(E4), scale


@pytest.mark.parametrize("R,C", [(100, 512), (6400, 2048), (37, 64)])
def test_quant_rows_exact(gpu_device, R, C):
    from stzs import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(R + C)
    x = (torch.randn(R, C, generator=g) * torch.rand(R, 1, generator=g) * 10).to(torch.bfloat16)
    x[3] = 0
    xd = x.to(gpu_device)
    y = torch.zeros(R, C, dtype=E4, device=gpu_device)
    s = torch.zeros(R, device=gpu_device)
    a = L.QuantArgs()
    a.x, a.y, a.scale, a.ldx, a.ldy, a.R, a.C = xd.data_ptr(), y.data_ptr(), s.data_ptr(), C, C, R, C
    L.check(lib.stzs_quant_rows(a, None), "quant")
    q, sc = quant_ref(x.float())
    yc = y.cpu().view(torch.uint8)
    bad = (yc != q.view(torch.uint8)).nonzero()
    if len(bad):
        r, c = bad[0].tolist()
        v = x[r, c].float().item() / sc[r].item()
        print(f"quant mismatches {len(bad)} / {R * C}; first ({r},{c}) scaled {v!r} gpu {yc[r, c].item():#04x} "
              f"ref {q.view(torch.uint8)[r, c].item():#04x}; scale gpu {s[r].item()!r} ref {sc[r].item()!r}; "
              f"scale mismatches {(s.cpu() != sc).sum().item()}")
    assert torch.equal(s.cpu(), sc)
    assert len(bad) == 0


def test_rowln_fp8(gpu_device):
    from stzs import _lib as L
    lib = L.load()
    R, C = 300, 512
    g = torch.Generator().manual_seed(9)
    x = torch.randn(R, C, generator=g) * 3 + 1
    G = torch.randn(R // 50, C, generator=g) * 0.3
    Bt = torch.randn(R // 50, C, generator=g) * 0.3
    xd, Gd, Bd = x.to(gpu_device), G.to(gpu_device), Bt.to(gpu_device)
    y = torch.zeros(R, C, dtype=E4, device=gpu_device)
    s = torch.zeros(R, device=gpu_device)
    a = L.RowLNArgs()
    a.x, a.y, a.G, a.Bt, a.y_scale = xd.data_ptr(), y.data_ptr(), Gd.data_ptr(), Bd.data_ptr(), s.data_ptr()
    a.ldx, a.ldy, a.gs, a.bs, a.R, a.C, a.gdiv = C, C, C, C, R, C, 50
    a.in_dtype, a.out_dtype, a.act, a.gadd, a.eps = L.F32, L.F8, L.ACT_NONE, 1.0, 1e-5
    L.check(lib.stzs_row_layernorm(a, None), "rowln f8")
    ref = F.layer_norm(x, (C,), eps=1e-5) * (1 + G.repeat_interleave(50, 0)) + Bt.repeat_interleave(50, 0)
    _, sref = quant_ref(ref)
    assert max_rel(s.cpu(), sref) < 1e-6
    deq = y.cpu().float() * s.cpu()[:, None]
    err = ((deq - ref).abs() / (ref.abs() + s.cpu()[:, None] * 2 ** -6)).max().item()
    print("rowln fp8 max rel (per element, subnormal floor)", err, "rel-L2", rel_err(deq, ref))
    assert err <= 2 ** -3 + 1e-6
    assert rel_err(deq, ref) < 4e-2


def _pack_f8(w, b):
    from stzs.weights import Arena, pack_conv_f8
    A = Arena()
    cw = pack_conv_f8(A, "t", w, b)
    A.finalize("cuda:0")
    cw.w, cw.wscale = A[cw.w], A[cw.wscale]
    cw.b = A[cw.b] if cw.b is not None else None
    return cw, A


@pytest.fixture(scope="module")
def eng(gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    return StyleTTSZS(tiny, tiny_params, device=gpu_device)


@pytest.mark.parametrize("M,K,N,dt_out,gelu", [(100, 512, 1536, torch.float32, False),
                                                (6400, 512, 2048, torch.bfloat16, True),
                                                (100, 2048, 512, torch.float32, False),
                                                (6400, 2048, 512, torch.float32, False),
                                                (50, 64, 192, torch.float32, False)])
def test_gemm_f8(eng, M, K, N, dt_out, gelu):
    from stzs.engine import Act
    from stzs import _lib as L
    from stzs.weights import quantize_f8_cols
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g) * torch.rand(M, 1, generator=g) * 4
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g) * 0.1
    qx, sx = quant_ref(x)
    cw, _A = _pack_f8(w, b)
    xd = Act(qx.to(eng.device)[None])
    y = Act(torch.zeros(1, M, N, dtype=dt_out, device=eng.device))
    eng.conv(cw, xd, y, x_scale=sx.to(eng.device), epi_act=L.ACT_GELU if gelu else L.ACT_NONE, what="f8")
    qw, sw = quantize_f8_cols(w)
    ref = (qx.float() * sx[:, None]) @ (qw.float() * sw[:, None]).t() + b
    if gelu:
        ref = F.gelu(ref)
    out = y.t[0].float().cpu()
    e = max_rel(out, ref)
    print("gemm f8", M, K, N, dt_out, e)
    assert e < (8e-3 if dt_out == torch.bfloat16 else 5e-5)


def _style_inputs(S, B, T, seed=1234):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(1, S.n_symbols, (B, T), generator=g)
    ref = torch.randn(B, S.sr, generator=g) * 0.1
    eps = torch.randn(B, S.L_s, S.code_dim, generator=g)
    return tok, ref, eps


@pytest.mark.parametrize("spec", ["tiny", "v0"])
def test_sample_style_fp8_vs_oracle(gpu_device, spec):
    """fp8 e4m3 denoiser (6 linears per layer) vs the fp32 oracle.  Stated tolerance: 1 NFE rel-L2
    <= 6e-2 (e4m3 has a 3-bit mantissa: ~2.5% rms per quantised operand); 2-step CFG-5 <= 1.5e-1.
    Measured (r01): tiny 7.1e-3 / 2.5e-2, v0 9.6e-3 / 3.9e-2."""
    from oracle import stzs_ref as R
    from stzs.engine import Act, StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY, SPEC_V0
    S = SPEC_TINY if spec == "tiny" else SPEC_V0
    P = init_params(S, seed=0)
    e8 = StyleTTSZS(S, P, device=gpu_device, fp8_denoiser=True)
    tok, ref, eps = _style_inputs(S, 2, 12 if spec == "tiny" else 80)
    h = R.text_encoder(P, S, tok).to(torch.bfloat16).float()
    prompt = R.prompt_encoder(P, S, ref)[0]
    for steps, cfg, tol in ((1, 1.0, 6e-2), (2, 5.0, 1.5e-1)):
        want = R.sample_style(P, S, h, prompt, eps, steps, cfg)
        ht = torch.zeros(*h.shape, dtype=torch.bfloat16, device=gpu_device)
        ht.copy_(h.to(torch.bfloat16))
        got = e8.sample_style(Act(ht), prompt.to(gpu_device), eps.to(gpu_device), steps, cfg).cpu()
        e = rel_err(got, want)
        print(f"fp8 sampler {spec} steps={steps} cfg={cfg}: rel-L2 {e:.3e}")
        assert torch.isfinite(got).all()
        assert e < tol

