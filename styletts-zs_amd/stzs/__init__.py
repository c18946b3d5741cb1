"""stzs — MI355X-native StyleTTS-ZS synthesis hot path (host side).

Importing the package is cheap and does not touch the GPU; `StyleTTSZS` loads libstzs_hip.so and
fails loudly if it is missing (there is no CPU fallback on the product path).
"""
from .spec import SPEC_TINY, SPEC_V0, Spec  # noqa: F401
from .params import init_params, param_checksum, param_count  # noqa: F401

__all__ = ["Spec", "SPEC_V0", "SPEC_TINY", "init_params", "param_checksum", "param_count", "StyleTTSZS"]


def __getattr__(name):
    if name == "StyleTTSZS":
        from .engine import StyleTTSZS
        return StyleTTSZS
    raise AttributeError(name)
