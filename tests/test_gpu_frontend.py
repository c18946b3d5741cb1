"""Reference-prompt front end on HIP (csrc/frontend.hip) vs the oracle.

Stated tolerances: log-mel mean-abs (L1) <= 3e-3 vs oracle log_mel (torch.stft fp32): the DFT runs as a bf16
MFMA GEMM, whose operand rounding alone costs 1.2e-3 on the CPU emulation (an fp32 emulation of the same
framing/basis matches torch.stft to 1.7e-7); adaptive pooling vs F.adaptive_avg_pool1d max-rel 1e-6 (fp32);
prompt codes vs oracle prompt_encoder rel-L2 <= 3e-2 (bf16 storage, as the text encoder)."""
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
    want = R.prompt_encoder(P, S, ref)
    got = eng.prompt_encode(ref.to(gpu_device)).cpu()
    e = rel_err(got, want)
    print("prompt codes", spec, e)
    assert e <= 3e-2
