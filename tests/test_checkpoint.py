"""safetensors parameter checkpoints (stzs/checkpoint.py), CPU only."""
import pytest
import torch
from safetensors.torch import save_file

from stzs.checkpoint import load_params, save_params
from stzs.params import init_params, param_checksum, param_shapes


def test_param_shapes_match_init(tiny, tiny_params):
    sh = param_shapes(tiny)
    assert list(sh) == list(tiny_params)
    assert all(sh[k] == v.shape for k, v in tiny_params.items())


def test_roundtrip(tmp_path, tiny, tiny_params):
    p = str(tmp_path / "tiny.safetensors")
    ck = save_params(p, tiny_params, tiny)
    params, spec = load_params(p)
    assert spec == tiny
    assert list(params) == list(tiny_params)
    assert param_checksum(params) == ck == param_checksum(tiny_params)
    assert all(torch.equal(params[k], v) for k, v in tiny_params.items())


def test_rejects_mismatches(tmp_path, tiny, tiny_params):
    from stzs.spec import SPEC_V0
    p = str(tmp_path / "tiny.safetensors")
    save_params(p, tiny_params, tiny)
    with pytest.raises(ValueError, match="differs"):
        load_params(p, SPEC_V0)
    bad = dict(tiny_params)
    bad["te.emb"] = torch.zeros(3, 3)
    with pytest.raises(ValueError, match="do not match"):
        save_params(str(tmp_path / "bad.safetensors"), bad, tiny)
    foreign = str(tmp_path / "foreign.safetensors")
    save_file({"x": torch.zeros(2)}, foreign)
    with pytest.raises(ValueError, match="not a"):
        load_params(foreign)
