import pytest
"""Weight-packing layouts (CPU): the fp8 K-step stream un-swizzles back to the quantised matrix, and the
quantiser matches its documented formula (stzs/weights.py, include/stzs.h stzs_conv_args.w_scale)."""
import torch

from stzs.weights import _GSWZ, kstep_stream_f8, quantize_f8_cols


def test_quantize_f8_cols():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(70, 96, generator=g)
    w[5] = 0
    q, s = quantize_f8_cols(w)
    assert s[5] == 1 and (q[5].float() == 0).all()
    assert torch.allclose(s[:5], w[:5].abs().amax(1) / 448)
    assert q.float().abs().max() <= 448
    rel = ((q.float() * s[:, None] - w).abs() / w.abs().clamp_min(1e-3)).max()
    assert rel < 2 ** -3


def test_kstep_stream_f8_roundtrip():
    g = torch.Generator().manual_seed(1)
    qp = torch.randint(0, 256, (256, 192), generator=g, dtype=torch.uint8)
    st = kstep_stream_f8(qp)
    assert st.shape == (2, 3, 128, 64)
    for cot in range(2):
        for k in range(3):
            for r in range(128):
                gz = _GSWZ[(r >> 2) & 3]
                for pos in range(4):
                    c = pos ^ gz
                    assert torch.equal(st[cot, k, r, pos * 16:(pos + 1) * 16],
                                       qp[cot * 128 + r, k * 64 + c * 16:k * 64 + (c + 1) * 16])


@pytest.mark.parametrize("s,Ch,T", [(6, 22, 40), (4, 20, 17), (3, 7, 9)])
def test_noise_super_weights_restatement(s, Ch, T):
    """the strided noise conv (k 2s, stride s, pad (s+1)//2) == a k3 stride-1 conv with padding 1 over super-rows of s
    zero-padded 32-channel rows (weights.noise_super_weights; engine.upsample), up to fp32 re-association"""
    import torch.nn.functional as F
    from stzs.weights import noise_super_weights
    g = torch.Generator().manual_seed(s + Ch + T)
    Co = 8
    wn = torch.randn(Co, Ch, 2 * s, generator=g, dtype=torch.float64)
    har = torch.randn(2, s * T + 1, Ch, generator=g, dtype=torch.float64)
    ref = F.conv1d(har.transpose(1, 2), wn, stride=s, padding=(s + 1) // 2)
    assert ref.shape[2] >= T
    rows = -(-(s * T + 1) // s) * s
    hp = torch.zeros(2, rows, 32, dtype=torch.float64)
    hp[:, :s * T + 1, :Ch] = har
    sup = hp.view(2, rows // s, s * 32)
    out = F.conv1d(sup.transpose(1, 2), noise_super_weights(wn.float(), s, 32).double(), padding=1)
    assert torch.allclose(out[:, :, :T], ref[:, :, :T], atol=1e-5)
