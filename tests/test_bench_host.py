"""bench.py host logic without a GPU: the kernel-family map of the per-stage roofline (roofline.stages) and the
whole-chip small-M routing rule of the per-utterance linears (a function of the weight's K only, shared with the
native composite operators: csrc/abi_ops.hip rows_ok)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def test_kernel_families():
    import bench
    assert bench._family("rb.c1", (3, 1, 24001, 128)) == "mrf k3 stage 1"
    assert bench._family("rb.c2", (11, 1, 4000, 256)) == "mrf k11 stage 0"
    assert bench._family("ups1", (2, 1, 4001, 128)) == "ConvT ups1"
    assert bench._family("te.lstm.rec", None) == "lstm recurrence"
    assert bench._family("sa_o.ln", None) == "row LayerNorm"
    assert bench._family("te.ln0", None) == "row LayerNorm"
    assert bench._family("ln1", None) == "row LayerNorm"
    assert bench._family("attention", None) == "attention"
    assert bench._family("qkv", (1, 1, 50, 1536)) == "linears (ks=1: gemm_glds / rows)"
    assert bench._family("dec.encode.conv1", (3, 1, 200, 1024)) == "other convs (k>1)"
    assert bench._family("istft", None) == "istft"


def test_small_rows_rule():
    from types import SimpleNamespace

    from stzs.engine import StyleTTSZS
    e = object.__new__(StyleTTSZS)
    e.small_rows = True
    z = lambda ci_pad: StyleTTSZS._rows_z(e, SimpleNamespace(ci_pad=ci_pad))
    # K = 128 .. 512: one K-step per wave .. four; K = 96 / 384: the waves would differ (the tiled path)
    assert [z(k) for k in (128, 256, 512, 1024, 2048)] == [1, 1, 1, 1, 1]
    assert z(96) == 0 and z(384) == 0 and z(4096) == 0
    e.small_rows = False
    assert z(256) == 0
