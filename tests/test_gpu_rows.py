"""The small-M linear (csrc/rows.hip, STZS_CONV_ROWS): the batch-1 denoiser linears on the whole chip.

Against torch fp32 on the same bf16 operands (max-rel over the outputs: fp32 accumulation in a different order,
bf16 output rounding -> 1e-2 for bf16 outputs, 1e-5 for fp32 outputs), for every denoiser linear shape and epilogue
(GELU ffn1, gated residual o / ffn2 in fp32, c_out / c_skip dn.out with accumulate-input, fp32-input dn.in with
cscale) and every K split Z, on both small-M forms (rows.hip, lnrows.hip rows16); batch invariance (rows of a
100-row launch == the same rows inside a 6 400-row launch, bit for bit); re-runs bit-identical (the split-K tickets
are left zeroed).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["rows", "rows16"])
def eng(request, gpu_device):
    """both small-M forms: csrc/rows.hip (K slices Z) and the 16-row register-direct csrc/lnrows.hip rows16 (which
    the engine takes for K <= rows16_maxk, ignoring Z)"""
    from stzs.engine import StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_TINY
    e = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=gpu_device)
    e.rows16 = request.param == "rows16"
    return e


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


# partial column tiles (N not a multiple of 64): the inactive waves of a 64-column rows16 K-slice tile still load
# tile 0's weights and meet the barriers, and the `ct * 16 >= Co` returns after the hand-off run
PARTIAL = [
    ("p80", 512, 80, torch.bfloat16, torch.bfloat16, "none", False, False, 1.0),
    ("p200", 512, 200, torch.bfloat16, torch.float32, "none", True, False, 1.0),
    ("p16", 2048, 16, torch.bfloat16, torch.float32, "none", True, False, 1.0),
]
# (K split must give every wave the same K-step count: (K / 32) % (4 Z) == 0)
RZ = [(c, Z) for c in CASES + PARTIAL for Z in (1, 2, 4) if (c[1] // 32) % (4 * Z) == 0]


@pytest.mark.parametrize("case,Z", RZ, ids=[f"{c[0]}-{Z}" for c, Z in RZ])
def test_rows_vs_torch(eng, case, Z):
    name, K, N, idt, odt, act, gated, acc, cs = case
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


@pytest.mark.parametrize("N,M", [(16, 50), (16, 100), (80, 100), (200, 50)])
def test_rows_split_workspace_exact(eng, N, M):
    """a C-ABI caller that sizes splitk_ws by stzs_conv_rows_workspace(M, Co, Z) exactly: both K-slice forms
    (csrc/rows.hip and the rows16 split form of csrc/lnrows.hip) stay inside it (a guard region behind the
    workspace is untouched) for Co % 64 in (0, 48], where rows16's 4-KB-per-(16 x 64 tile) slabs outgrow rows.hip's
    layout (the header promised this size, the engine was only safe by its 4-MB minimum scratch)."""
    K, Z = 512, 2
    w, b, cw, x, res, ai, gate = _setup(eng, K, N, torch.bfloat16, torch.float32, True, False, M, N + M)
    nb = eng.lib.stzs_conv_rows_workspace(M, N, Z)
    assert nb > 0 and nb % 4 == 0
    guard = 1 << 16
    store = torch.full((nb // 4 + guard,), 12345.0, device=eng.device)
    orig = eng._scratch
    eng._scratch = lambda name, n: store if name.startswith("rows_ws") else orig(name, n)
    try:
        y = _run(eng, cw, x, res, ai, gate, N, torch.float32, "none", 1.0, Z).float().cpu()
    finally:
        eng._scratch = orig
    assert bool((store[nb // 4:] == 12345.0).all()), "slab writes past stzs_conv_rows_workspace bytes"
    ref = (x.float() @ w.to(torch.bfloat16).float().t() + b) * gate[:, None, :] + res.float()
    assert ((y - ref).abs().max() / ref.abs().max()).item() < 1e-5
