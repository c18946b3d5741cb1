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


def test_cpu_tensor_raises():
    from stzs import ops  # noqa: F401
    with pytest.raises(NotImplementedError):
        torch.ops.stzs.istft(torch.zeros(1, 10, 24), 20, 5)
    with pytest.raises(NotImplementedError):
        torch.ops.stzs.duration_head(torch.zeros(1, 4, 50))
