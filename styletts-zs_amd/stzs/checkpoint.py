"""safetensors checkpoints of the model parameters (checkpoint loader).

No StyleTTS-ZS checkpoint is published (`/root/reference/README.md:15-16`), so the format is this
framework's own: one safetensors file holding the torch-native parameter tensors of `stzs.params`
(Conv1d [Co, Ci, k], Linear [out, in], LSTM gate order i, f, g, o, ...) under their declaration names,
with the `Spec` and a content checksum in the metadata.  Loading goes through safetensors only (no
pickle), validates every name and shape against the spec, and checks the checksum; the packed
device layouts are then rebuilt by `stzs.weights.PackedModel` exactly as for random-init weights.

    save_params("model.safetensors", params, SPEC_V0)
    params, spec = load_params("model.safetensors")
    eng = StyleTTSZS.from_checkpoint("model.safetensors", device="cuda:0")   # engine.py
"""
from __future__ import annotations

import dataclasses
import json
from collections import OrderedDict

import torch
from safetensors import safe_open
from safetensors.torch import save_file

from .params import param_checksum, param_shapes
from .spec import Spec

FORMAT = "stzs-params-v0"


def _spec_json(spec: Spec) -> str:
    return json.dumps(dataclasses.asdict(spec), sort_keys=True)


def _spec_from_json(s: str) -> Spec:
    d = json.loads(s)
    return Spec(**{k: tuple(v) if isinstance(v, list) else v for k, v in d.items()})


def save_params(path: str, params, spec: Spec) -> str:
    """write `params` (name -> tensor, validated against `spec`) to a safetensors file; -> checksum"""
    _validate(params, spec)
    ck = param_checksum(params)
    save_file({k: v.detach().contiguous().cpu() for k, v in params.items()}, path,
              metadata={"format": FORMAT, "spec": _spec_json(spec), "checksum": ck})
    return ck


def load_params(path: str, spec: Spec = None):
    """-> (params OrderedDict in declaration order, spec).  `spec` defaults to the one stored in the file;
    a given spec must equal it.  Raises ValueError on a foreign format, a spec / name / shape mismatch or a
    checksum mismatch."""
    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} checkpoint (format={meta.get('format')!r})")
        stored = _spec_from_json(meta["spec"])
        if spec is not None and spec != stored:
            raise ValueError(f"{path}: checkpoint spec {stored.name!r} differs from the requested spec {spec.name!r}")
        spec = stored
        names = list(f.keys())
        expected = param_shapes(spec)
        missing = [k for k in expected if k not in names]
        unexpected = [k for k in names if k not in expected]
        if missing or unexpected:
            raise ValueError(f"{path}: missing {missing[:8]} unexpected {unexpected[:8]}")
        params = OrderedDict((k, f.get_tensor(k)) for k in expected)
    _validate(params, spec)
    ck = param_checksum(params)
    if meta.get("checksum") and meta["checksum"] != ck:
        raise ValueError(f"{path}: checksum {ck} != stored {meta['checksum']}")
    return params, spec


def _validate(params, spec: Spec):
    expected = param_shapes(spec)
    bad = [(k, tuple(params[k].shape), tuple(s)) for k, s in expected.items() if k in params and params[k].shape != s]
    missing = [k for k in expected if k not in params]
    if bad or missing:
        raise ValueError(f"parameters do not match spec {spec.name!r}: shape {bad[:6]} missing {missing[:6]}")
    for k, v in params.items():
        if v.dtype != torch.float32:
            raise ValueError(f"{k}: expected float32 parameters, got {v.dtype}")
