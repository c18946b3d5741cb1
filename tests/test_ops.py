"""torch.ops.stzs without a GPU: every operator is registered, its fake (meta)
implementation gives the documented output shapes, and a CPU tensor raises (HIP-only, no fallback)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode


def test_registered():
    from stzs import ops
    for name in ops.OPS:
        assert hasattr(torch.ops.stzs, name), name


def test_fake_shapes():
    from stzs import ops  # noqa: F401
    with FakeTensorMode():
        post = torch.empty(2, 24001, 24)
        assert torch.ops.stzs.istft(post, 20, 5).shape == (2, 120000)
        w, t = torch.ops.stzs.istft_stream(torch.empty(2, 4800, 24), torch.empty(2, 3, 24), 4800, False, 20, 5)
        assert w.shape == (2, 24000) and t.shape == (2, 3, 24)
        d, s = torch.ops.stzs.duration_head(torch.empty(3, 80, 50))
        assert d.shape == (3, 80) and d.dtype == torch.int32 and s.dtype == torch.float32
        assert torch.ops.stzs.length_regulate(torch.empty(3, 80, dtype=torch.int32), 200).shape == (3, 200)
        assert torch.ops.stzs.cfg_euler_step(torch.empty(4, 50, 256), torch.empty(4, 50, 256), True, 5.0, 3.0,
                                             0.5).shape == (4, 50, 256)
        assert torch.ops.stzs.decode(1, torch.empty(2, 200, 512), torch.empty(2, 400), torch.empty(2, 400),
                                     torch.empty(2, 50, 256), [0, 1]).shape == (2, 120000)
        assert torch.ops.stzs.sample_style(1, torch.empty(2, 80, 512), torch.empty(2, 50, 256),
                                           torch.empty(2, 50, 256), 2, 5.0).shape == (2, 50, 256)


def test_fake_shapes_model_bound(tiny, tiny_params):
    """the model-bound per-row operators' fakes read the registered engine's spec (host metadata, no GPU)."""
    from stzs import ops
    from stzs.engine import StyleTTSZS
    S = tiny
    eng = object.__new__(StyleTTSZS)  # metadata-only stand-in: the fakes only read .spec
    eng.spec = S
    h = ops.register(eng)
    with FakeTensorMode():
        assert torch.ops.stzs.bilstm(h, "pr.de0", torch.empty(2, 9, S.pr_in)).shape == (2, 9, S.pr_hid)
        assert torch.ops.stzs.denoiser_fwd(h, torch.empty(2, 9, S.d_txt), torch.empty(2, S.L_s, S.code_dim),
                                           torch.empty(4, S.L_s, S.code_dim), 3.0, True).shape == (4, S.L_s, S.code_dim)
        F0, N = torch.ops.stzs.f0n_predictor(h, torch.empty(2, 20, S.pr_in), torch.empty(2, S.L_s, S.code_dim))
        assert F0.shape == N.shape == (2, 40)
        assert torch.ops.stzs.decoder_pre(h, torch.empty(2, 20, S.d_txt), torch.empty(2, 40), torch.empty(2, 40),
                                          torch.empty(2, S.L_s, S.code_dim)).shape == (2, 40, S.dec_out)
        har = torch.ops.stzs.sine_gen(h, torch.empty(2, 40), [0, 1])
        assert har.shape == (2, 40 * S.hop // S.istft_hop + 1, S.har_ch)
        assert torch.ops.stzs.conv_transpose_up(h, torch.empty(2, 40, S.dec_out), har, 0).shape == \
            (2, 40 * S.up_rates[0], S.gen_ch[0])
        assert torch.ops.stzs.conv_transpose_up(h, torch.empty(2, 400, S.gen_ch[0]), har, 1).shape == \
            (2, 400 * S.up_rates[1] + 1, S.gen_ch[1])
        assert torch.ops.stzs.mrf_resblock(h, torch.empty(2, 400, S.gen_ch[0]), torch.empty(2, S.L_s, S.code_dim),
                                           0).shape == (2, 400, S.gen_ch[0])
        assert torch.ops.stzs.conv_post_istft(h, torch.empty(2, 2401, S.gen_ch[1])).shape == (2, 2400 * S.istft_hop)
        i, q = torch.ops.stzs.code_quantize(h, torch.empty(2, S.L_s, S.code_dim))
        assert i.shape == (2, S.L_s, S.code_dim // S.vq_group) and i.dtype == torch.int32 and q.shape == (2, S.L_s, S.code_dim)


def test_cpu_tensor_raises():
    from stzs import ops  # noqa: F401
    with pytest.raises(NotImplementedError):
        torch.ops.stzs.istft(torch.zeros(1, 10, 24), 20, 5)
    with pytest.raises(NotImplementedError):
        torch.ops.stzs.duration_head(torch.zeros(1, 4, 50))
