"""The small-M linear (csrc/rows.hip, STZS_CONV_ROWS): the batch-1 denoiser linears on the whole chip.

Against torch fp32 on the same bf16 operands (max-rel over the outputs: fp32 accumulation in a different order,
bf16 output rounding -> 1e-2 for bf16 outputs, 1e-5 for fp32 outputs), for every denoiser linear shape and epilogue
(GELU ffn1, gated residual o / ffn2 in fp32, c_out / c_skip dn.out with accumulate-input, fp32-input dn.in with
cscale) and every K split Z; batch invariance (rows of a 100-row launch == the same rows inside a 6 400-row launch,
bit for bit); re-runs bit-identical (the split-K tickets are left zeroed).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_device):
    from stzs.engine import StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    return StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=gpu_device)


CASES = [  # name, K, N, in dtype, out dtype, act, gated residual, acc_in, cscale
    ("qkv", 512, 1536, torch.bfloat16, torch.bfloat16, "none", False, False, 1.0),
    ("ff1", 512, 2048, torch.bfloat16, torch.bfloat16, "gelu", False, False, 1.0),
    ("o", 512, 512, torch.bfloat16, torch.float32, "none", True, False, 1.0),
    ("ff2", 2048, 512, torch.bfloat16, torch.float32, "none", True, False, 1.0),
    ("out", 512, 256, torch.bfloat16, torch.float32, "none", False, True, 1.0),
    ("in", 256, 512, torch.float32, torch.float32, "none", False, False, 0.37),
]


def _setup(eng, K, N, idt, odt, gated, acc, M, seed):
    from stzs.engine import Act
    from stzs.weights import Arena, pack_conv
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g) * 0.1
    A = Arena()
    cw = pack_conv(A, "g", w, b)
    A.finalize(eng.device)
    cw.w, cw.b = A[cw.w], A[cw.b]
    B = M // 50
    x = torch.randn(B, 50, K, generator=g).to(idt)
    res = torch.randn(B, 50, N, generator=g).to(odt) if gated else None
    ai = torch.randn(B, 50, N, generator=g).to(odt) if acc else None
    gate = torch.rand(B, N, generator=g) + 0.5
    return w, b, cw, x, res, ai, gate


def _run(eng, cw, x, res, ai, gate, N, odt, act, cs, rows):
    from stzs import _lib as L
    from stzs.engine import Act
    dev = eng.device
    B = x.shape[0]
    y = Act(torch.zeros(B, 50, N, device=dev, dtype=odt))
    gd = gate.to(dev)
    eng.conv(cw, Act(x.to(dev)), y, epi_act=L.ACT_GELU if act == "gelu" else L.ACT_NONE,
             res=Act(res.to(dev)) if res is not None else None, gate=gd.data_ptr() if res is not None else None,
             gate_bs=N, acc_in=Act(ai.to(dev)) if ai is not None else None, alpha=0.75 if ai is not None else 1.0,
             beta=1.25 if ai is not None else 0.0, cscale=cs, rows=rows, what="rows")
    torch.cuda.synchronize()
    return y.t.clone()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("Z", [1, 2, 4])
def test_rows_vs_torch(eng, case, Z):
    name, K, N, idt, odt, act, gated, acc, cs = case
    if (K // 32) % (4 * Z):
        pytest.skip("K split must give every wave the same K-step count")
    w, b, cw, x, res, ai, gate = _setup(eng, K, N, idt, odt, gated, acc, 100, K + N + Z)
    y = _run(eng, cw, x, res, ai, gate, N, odt, act, cs, Z).float().cpu()
    xa = (x.float() * cs).to(torch.bfloat16).float()
    ref = xa @ w.to(torch.bfloat16).float().t() + b
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    if gated:
        ref = ref * gate[:, None, :] + res.float()
    if acc:
        ref = 0.75 * ref + 1.25 * ai.float()
    e = ((y - ref).abs().max() / ref.abs().max()).item()
    print(f"rows {name} Z={Z}: max-rel {e:.2e}")
    assert e < (1e-2 if odt == torch.bfloat16 else 1e-5)
    y2 = _run(eng, cw, x, res, ai, gate, N, odt, act, cs, Z).float().cpu()
    assert torch.equal(y, y2)


@pytest.mark.parametrize("case", [CASES[0], CASES[3], CASES[5]], ids=["qkv", "ff2", "in"])
def test_rows_batch_invariant(eng, case):
    """the per-element summation order depends on K and Z only: rows of a 100-row launch are bit-identical to the
    same rows inside a 6 400-row (and a 250-row) launch."""
    name, K, N, idt, odt, act, gated, acc, cs = case
    Z = 4 if K == 2048 else 1
    w, b, cw, x, res, ai, gate = _setup(eng, K, N, idt, odt, gated, acc, 6400, 9)
    big = _run(eng, cw, x, res, ai, gate, N, odt, act, cs, Z)
    for lo, hi in ((0, 2), (61, 66)):
        sl = slice(lo, hi)
        small = _run(eng, cw, x[sl], res[sl] if res is not None else None, ai[sl] if ai is not None else None,
                     gate[sl], N, odt, act, cs, Z)
        assert torch.equal(small, big[sl]), (name, lo, hi)


# ---- fused consumers (include/stzs_fused.h): bit-identical to the linear + the separate LayerNorm / attention ----
FUSE_LN_CASES = [  # name, K, N, in dtype, gated residual, cscale, Z
    ("o", 512, 512, torch.bfloat16, True, 1.0, 1),
    ("ff2", 2048, 512, torch.bfloat16, True, 1.0, 4),
    ("in", 256, 512, torch.float32, False, 0.37, 1),
]


def _with_fuse(eng, on, fn):
    old = eng.fuse_rows
    eng.fuse_rows = on
    try:
        n0 = eng.launches
        out = fn()
        torch.cuda.synchronize()
        return out, eng.launches - n0
    finally:
        eng.fuse_rows = old


@pytest.mark.parametrize("case", FUSE_LN_CASES, ids=[c[0] for c in FUSE_LN_CASES])
@pytest.mark.parametrize("B", [1, 2, 5])
def test_rows_fused_layernorm_bit_identical(eng, case, B):
    """STZS_FUSE_LN: the residual linear's output rows and the modulated LayerNorm of them (per-utterance gamma /
    beta rows, gadd 1: the adaLN modulate) from ONE launch equal the linear + stzs_row_layernorm bit for bit
    (tolerance 0); 16-row blocks straddle utterances at B = 5 (250 rows, ragged last block); re-run identical and
    the hand-off counters left zero."""
    from stzs.engine import Act
    name, K, N, idt, gated, cs, Z = case
    dev = eng.device
    w, b, cw, x, res, ai, gate = _setup(eng, K, N, idt, torch.float32, gated, False, 50 * B, K + B)
    g = torch.Generator().manual_seed(B)
    G = (torch.randn(B, N, generator=g) * 0.3).to(dev)
    Bt = (torch.randn(B, N, generator=g) * 0.3).to(dev)
    xd, gd = Act(x.to(dev)), gate.to(dev)
    resd = res.to(dev) if gated else None

    def run():
        y = Act(resd.clone() if gated else torch.zeros(B, 50, N, device=dev))
        an = Act(torch.zeros(B, 50, N, device=dev, dtype=torch.bfloat16))
        ln = eng._ln_args(y, an, G=G.data_ptr(), gs=N, Bt=Bt.data_ptr(), bs=N, gdiv=50, gadd=1.0)
        eng.conv(cw, xd, y, res=y if gated else None, gate=gd.data_ptr() if gated else None, gate_bs=N,
                 cscale=cs, rows=Z, post_ln=ln, what="fz")
        return y.t.clone(), an.t.clone()

    (y0, a0), n0 = _with_fuse(eng, False, run)
    (y1, a1), n1 = _with_fuse(eng, True, run)
    (y2, a2), _ = _with_fuse(eng, True, run)
    assert (n0, n1) == (2, 1)
    assert torch.equal(y0, y1) and torch.equal(a0, a1), (name, B)
    assert torch.equal(y1, y2) and torch.equal(a1, a2)
    assert int(eng._counters("fuse_ctr", 1).abs().sum()) == 0
    ref = torch.nn.functional.layer_norm(y0.float(), (N,), eps=1e-5).cpu() * (1 + G.cpu()[:, None]) + Bt.cpu()[:, None]
    assert ((a0.float().cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("kind", ["self", "cross"])
@pytest.mark.parametrize("B", [1, 2, 3])
def test_rows_fused_attention_bit_identical(eng, kind, B):
    """STZS_FUSE_ATTN: the qkv linear + self-attention (q / k / v inside the linear's output) and the query linear +
    cross-attention (k / v of a 130-key context written earlier) from ONE launch equal the linear + stzs_attention
    bit for bit (tolerance 0); 8 heads x 64; re-run identical, counters left zero."""
    from stzs.engine import Act
    dev = eng.device
    d, H = 512, 8
    N = 3 * d if kind == "self" else d
    w, b, cw, x, res, ai, gate = _setup(eng, 512, N, torch.bfloat16, torch.bfloat16, False, False, 50 * B, N + B)
    g = torch.Generator().manual_seed(7 + B)
    kv = Act(torch.randn(B, 130, 2 * d, generator=g).to(dev, torch.bfloat16))
    xd = Act(x.to(dev))
    saved = eng.spec

    def run():
        y = Act(torch.zeros(B, 50, N, device=dev, dtype=torch.bfloat16))
        o = Act(torch.zeros(B, 50, d, device=dev, dtype=torch.bfloat16))
        at = (y.sl(0, d), y.sl(d, d), y.sl(2 * d, d), o) if kind == "self" else (y, kv.sl(0, d), kv.sl(d, d), o)
        eng.conv(cw, xd, y, rows=1, attn=at, what="fz")
        return y.t.clone(), o.t.clone()

    import dataclasses
    eng.spec = dataclasses.replace(saved, dn_d=d, dn_heads=H)  # the attention shape of the v0 denoiser
    try:
        assert eng.spec.dn_head_dim == 64
        (y0, o0), n0 = _with_fuse(eng, False, run)
        (y1, o1), n1 = _with_fuse(eng, True, run)
        (y2, o2), _ = _with_fuse(eng, True, run)
    finally:
        eng.spec = saved
    assert (n0, n1) == (2, 1)
    assert torch.equal(y0, y1) and torch.equal(o0, o1), (kind, B)
    assert torch.equal(o1, o2)
    assert int(eng._counters("fuse_ctr", 1).abs().sum()) == 0
    assert float(o0.float().abs().max()) > 0


@pytest.mark.parametrize("B,cfg", [(1, 1), (2, 1), (3, 0)])
def test_rows_fused_cfg_euler_bit_identical(eng, B, cfg):
    """STZS_FUSE_CFG: the denoiser output projection D = c_out F + c_skip x and the sampler's CFG + Euler update of x
    from ONE launch equal the linear + stzs_cfg_euler bit for bit (state and D; tolerance 0), counters left zero."""
    from stzs import _lib as L
    from stzs.engine import Act
    dev = eng.device
    R = 2 * B if cfg else B
    K, N = 512, 256
    g = torch.Generator().manual_seed(R)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "g", w, torch.randn(N, generator=g) * 0.1)
    A.finalize(dev)
    cw.w, cw.b = A[cw.w], A[cw.b]
    an = Act(torch.randn(R, 50, K, generator=g).to(dev, torch.bfloat16))
    x0 = torch.randn(R, 50, N, generator=g).to(dev)
    eu = (B, cfg, 5.0, 0.8, -0.3)

    def run(on):
        x = x0.clone()
        D = Act(torch.zeros(R, 50, N, device=dev))
        old, eng.fuse_rows = eng.fuse_rows, on
        try:
            fused = eng.conv(cw, an, D, alpha=0.6, acc_in=Act(x), beta=0.4, rows=1, cfg=eu, what="fz") is not D
        finally:
            eng.fuse_rows = old
        if not fused:
            L.check(eng.lib.stzs_cfg_euler(x.data_ptr(), D.t.data_ptr(), B, 50 * N, cfg, 5.0, 0.8, -0.3,
                                           eng.stream()), "cfg_euler")
        torch.cuda.synchronize()
        return fused, x.cpu(), D.t.cpu()

    f0, xa, Da = run(False)
    f1, xb, Db = run(True)
    assert (f0, f1) == (False, True)
    assert torch.equal(Da, Db) and torch.equal(xa, xb)
    assert not torch.equal(xa, x0.cpu())
    assert int(eng._counters("fuse_ctr", 1).abs().sum()) == 0
