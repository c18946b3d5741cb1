"""Reference-prompt front end on HIP (csrc/frontend.hip) vs the oracle.

Stated tolerances: log-mel mean-abs (L1) <= 3e-3 vs oracle log_mel (torch.stft fp32): the DFT runs as a bf16
MFMA GEMM, whose operand rounding alone costs 1.2e-3 on the CPU emulation (an fp32 emulation of the same
framing/basis matches torch.stft to 1.7e-7); adaptive pooling vs F.adaptive_avg_pool1d max-rel 1e-6 (fp32);
continuous prompt features vs oracle prompt_features rel-L2 <= 3e-2 (bf16 storage, as the text encoder);
discrete prompt codes (stzs_code_quantize) bit-exact on the oracle's fp32 inputs, and end to end wherever the
oracle's decision margin exceeds the bound the front end's measured error can move a distance by."""
import pytest
import torch
import torch.nn.functional as F

from refops import max_rel, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def v0eng(gpu_device):
    from stzs.engine import StyleTTSZS
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    P = init_params(SPEC_V0, seed=0)
    return StyleTTSZS(SPEC_V0, P, device=gpu_device), SPEC_V0, P


@pytest.mark.parametrize("N", [72000, 24000, 30001])
def test_log_mel(v0eng, N):
    from stzs.frontend import log_mel
    eng, S, _ = v0eng
    g = torch.Generator().manual_seed(N)
    wav = torch.randn(3, N, generator=g) * 0.1
    wav[1] *= torch.linspace(0, 3, N)  # non-stationary level
    ref = log_mel(wav, S).transpose(1, 2)
    got = eng.log_mel(wav.to(eng.device), torch.float32).t[:, :, :S.n_mels].cpu()  # fp32 out: the bf16
    # the encoder consumes adds one output rounding (~4e-3 mean at |log-mel| ~ 2), covered by the codes test
    assert got.shape == ref.shape
    l1 = (got - ref).abs().mean().item()
    print("log-mel L1", N, l1, "max", (got - ref).abs().max().item())
    assert l1 <= 3e-3


@pytest.mark.parametrize("T,L", [(241, 50), (50, 50), (37, 50), (1001, 8)])
def test_pool_rows(gpu_device, T, L):
    from stzs import _lib as L_
    lib = L_.load()
    g = torch.Generator().manual_seed(T)
    x = torch.randn(2, T, 64, generator=g)
    xd = x.to(gpu_device)
    y = torch.zeros(2, L, 64, device=gpu_device)
    a = L_.PoolArgs()
    a.x, a.y, a.ldx, a.bsx, a.ldy, a.bsy = xd.data_ptr(), y.data_ptr(), 64, T * 64, 64, L * 64
    a.B, a.T, a.L, a.C, a.in_dtype, a.out_dtype = 2, T, L, 64, L_.F32, L_.F32
    L_.check(lib.stzs_pool_rows(a, None), "pool")
    ref = F.adaptive_avg_pool1d(x.transpose(1, 2), L).transpose(1, 2)
    assert max_rel(y.cpu(), ref) < 1e-6


@pytest.mark.parametrize("spec", ["tiny", "v0"])
def test_prompt_encoder(gpu_device, v0eng, spec, tiny, tiny_params):
    from oracle import stzs_ref as R
    from stzs.engine import StyleTTSZS
    if spec == "v0":
        eng, S, P = v0eng
    else:
        S, P = tiny, tiny_params
        eng = StyleTTSZS(S, P, device=gpu_device)
    g = torch.Generator().manual_seed(11)
    ref = torch.randn(2, 3 * S.sr, generator=g) * 0.1
    z_want = R.prompt_features(P, S, ref)
    z = eng.prompt_features(ref.to(gpu_device)).cpu()
    e = rel_err(z, z_want)
    # discrete codes end to end: the GPU's indices equal the oracle's wherever the oracle's decision margin
    # (second-best minus best distance) exceeds what the bf16 front end's error can move (guard below)
    _, idx_want, margin = R.prompt_encoder(P, S, ref)
    got = eng.prompt_encode(ref.to(gpu_device)).cpu()
    idx = eng.prompt_idx.cpu()
    # |d_k(z) - d_k(z')| <= 2 dg max|z - z'| (max|z| + max|c|) per distance, and the margin is a difference of two
    guard = 4 * S.vq_group * (z - z_want).abs().max().item() * (z_want.abs().max().item() + P["pe.vq"].abs().max().item())
    clear = margin > guard
    agree = (idx == idx_want)
    print("prompt features", spec, e, "guard", guard, "clear", clear.float().mean().item(),
          "agree", agree.float().mean().item())
    assert e <= 3e-2
    assert bool(agree[clear].all())
    torch.testing.assert_close(got, R.lookup_codes(P, S, idx), atol=0, rtol=0)


@pytest.mark.parametrize("spec", ["tiny", "v0"])
def test_code_quantize_bit_exact(gpu_device, spec, tiny, tiny_params, v0eng):
    """stzs_code_quantize on the oracle's own fp32 inputs: indices and dequantised rows bit-exact, including
    exact ties (duplicated codebook rows: the first index wins) and the lookup (teacher-forced) mode."""
    from oracle import stzs_ref as R
    from stzs.engine import StyleTTSZS
    if spec == "v0":
        eng, S, P = v0eng
    else:
        S, P = tiny, tiny_params
        eng = StyleTTSZS(S, P, device=gpu_device)
    G = S.code_dim // S.vq_group
    B = 5
    z = torch.randn(B, S.L_s, S.code_dim, generator=torch.Generator().manual_seed(31)) * 0.2
    z[0, 0] = P["pe.vq"][torch.arange(G), 3].reshape(-1)   # exactly on codebook rows
    idx_w, q_w, _ = R.quantize_codes(P, S, z)
    idx = torch.zeros(B, S.L_s, G, dtype=torch.int32, device=gpu_device)
    out = torch.zeros(B, S.L_s, S.code_dim, device=gpu_device)
    eng.code_quantize(z.to(gpu_device), idx, out)
    assert torch.equal(idx.cpu(), idx_w)
    assert torch.equal(out.cpu(), q_w)
    assert (idx_w[0, 0] == 3).all()
    out2 = torch.zeros_like(out)
    eng.code_quantize(None, idx, out2, lookup=True)
    assert torch.equal(out2, out)


def test_code_quantize_first_minimum_on_ties(gpu_device, tiny, tiny_params):
    """a codebook with duplicated rows: every tie resolves to the lower index (torch.argmin's rule)."""
    from oracle import stzs_ref as R
    from stzs.engine import StyleTTSZS
    S = tiny
    P = dict(tiny_params)
    cb = P["pe.vq"].clone()
    cb[:, 1::2] = cb[:, 0::2]            # row 2i+1 duplicates row 2i
    P["pe.vq"] = cb
    eng = StyleTTSZS(S, P, device=gpu_device)
    z = torch.randn(3, S.L_s, S.code_dim, generator=torch.Generator().manual_seed(32)) * 0.2
    idx_w, q_w, _ = R.quantize_codes(P, S, z)
    assert (idx_w % 2 == 0).all()
    G = S.code_dim // S.vq_group
    idx = torch.zeros(3, S.L_s, G, dtype=torch.int32, device=gpu_device)
    out = torch.zeros(3, S.L_s, S.code_dim, device=gpu_device)
    eng.code_quantize(z.to(gpu_device), idx, out)
    assert torch.equal(idx.cpu(), idx_w) and torch.equal(out.cpu(), q_w)
