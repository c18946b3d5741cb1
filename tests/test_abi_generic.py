"""The generic tensor-descriptor C-ABI (include/stzs.h, csrc/abi.hip) without a GPU: the C++ weight packers are
bit-identical to the Python ones the engine uses (stzs/weights.py), the workspace queries are consistent, and every
generic entry point rejects bad calls before touching the device."""
import ctypes as C
import math

import numpy as np
import pytest
import torch

from stzs import _lib as L


def _py_pack(w, b=None, **kw):
    from stzs.weights import Arena, pack_conv
    A = Arena()
    cw = pack_conv(A, "t", w, b, **kw)
    A.finalize("cpu")
    return A[cw.w].contiguous().view(torch.uint8).numpy().tobytes(), cw


@pytest.mark.parametrize("Co,Ci,ks,ups,form", [
    (128, 128, 3, 0, L.PACK_FRAG32), (128, 128, 11, 0, L.PACK_FRAG32), (256, 256, 7, 0, L.PACK_FRAG32),
    (128, 128, 3, 0, L.PACK_LANE16), (1024, 1090, 3, 0, L.PACK_LANE16), (64, 200, 3, 0, L.PACK_KSTEP),
    (3072, 512, 1, 0, L.PACK_KSTEP), (96, 20, 5, 0, L.PACK_KSTEP), (22, 128, 7, 0, L.PACK_NARROW32),
    (256, 512, 20, 10, L.PACK_LANE16), (32, 64, 12, 6, L.PACK_KSTEP),
])
def test_pack_conv_matches_python(Co, Ci, ks, ups, form):
    lib = L.load()
    g = torch.Generator().manual_seed(Co + Ci + ks)
    shape = (Ci, Co, 2 * ups) if ups else (Co, Ci, ks)
    w = torch.randn(shape, generator=g) / math.sqrt(Ci * ks)
    kw = {L.PACK_LANE16: dict(lane16=True), L.PACK_FRAG32: dict(frag32=True), L.PACK_NARROW32: dict(narrow32=True),
          L.PACK_KSTEP: {}}[form]
    want, cw = _py_pack(w, ups=ups, **kw)
    n = lib.stzs_pack_conv_size(Co, Ci, ks, ups, form)
    assert n == len(want)
    out = np.zeros(n, dtype=np.uint8)
    wc = np.ascontiguousarray(w.numpy(), dtype=np.float32)
    assert lib.stzs_pack_conv(wc.ctypes.data, Co, Ci, ks, ups, form, out.ctypes.data) == L.OK
    assert out.tobytes() == want


@pytest.mark.parametrize("Co,Ci,ks,ups", [(128, 128, 3, 0), (80, 96, 3, 0), (1536, 512, 1, 0), (22, 128, 7, 0),
                                          (256, 512, 20, 10)])
def test_pack_conv_x3_matches_python(Co, Ci, ks, ups):
    """the precise-mode split streams (hi | lo, 32-channel K-steps) bit-identical to stzs/weights.py."""
    from stzs.weights import Arena, pack_conv
    lib = L.load()
    g = torch.Generator().manual_seed(Co + 3 * Ci + ks)
    shape = (Ci, Co, 2 * ups) if ups else (Co, Ci, ks)
    w = torch.randn(shape, generator=g) / math.sqrt(Ci * ks)
    A = Arena()
    cw = pack_conv(A, "t", w, None, ups=ups, x3=True)
    A.finalize("cpu")
    want = A[cw.wx3].contiguous().view(torch.uint8).numpy().tobytes()
    n = lib.stzs_pack_conv_size(Co, Ci, ks, ups, L.PACK_X3)
    assert n == len(want)
    out = np.zeros(n, dtype=np.uint8)
    wc = np.ascontiguousarray(w.numpy(), dtype=np.float32)
    assert lib.stzs_pack_conv(wc.ctypes.data, Co, Ci, ks, ups, L.PACK_X3, out.ctypes.data) == L.OK
    assert out.tobytes() == want


@pytest.mark.parametrize("Co,Ci,ks", [(128, 128, 3), (256, 256, 11), (176, 256, 7), (64, 130, 3), (1536, 512, 1),
                                      (2048, 640, 1)])
def test_pack_conv_frag32x3_matches_python(Co, Ci, ks):
    """the precise register-direct split stream (hi | lo FRAG32 blocks per K-step, csrc/mrfx.hip) bit-identical to
    stzs/weights.py frag32x3_stream."""
    from stzs.weights import Arena, pack_conv
    lib = L.load()
    g = torch.Generator().manual_seed(Co + 5 * Ci + ks)
    w = torch.randn(Co, Ci, ks, generator=g) / math.sqrt(Ci * ks)
    A = Arena()
    cw = pack_conv(A, "t", w[:, :, 0] if ks == 1 else w, None, frag32=ks > 1, x3=True)
    A.finalize("cpu")
    want = A[cw.fx3].contiguous().view(torch.uint8).numpy().tobytes()
    n = lib.stzs_pack_conv_size(Co, Ci, ks, 0, L.PACK_FRAG32X3)
    assert n == len(want)
    out = np.zeros(n, dtype=np.uint8)
    wc = np.ascontiguousarray(w.numpy(), dtype=np.float32)
    assert lib.stzs_pack_conv(wc.ctypes.data, Co, Ci, ks, 0, L.PACK_FRAG32X3, out.ctypes.data) == L.OK
    assert out.tobytes() == want
    assert lib.stzs_pack_conv_size(22, 128, 7, 0, L.PACK_FRAG32X3) == 0  # Co % 8


def test_pack_lstm_x3_matches_python(tiny_params):
    from stzs.weights import Arena, pack_lstm
    lib = L.load()
    P = tiny_params
    A = Arena()
    lw = pack_lstm(A, "pr.de0", P, x3=True)
    A.finalize("cpu")
    ih_want = A[lw.ih.wx3].contiguous().view(torch.uint8).numpy().tobytes()
    f_want = A[lw.whx3].contiguous().view(torch.uint8).numpy().tobytes()
    H, In = lw.H, P["pr.de0.w_ih"].shape[1]
    ih = np.zeros(lib.stzs_pack_conv_size(8 * H, In, 1, 0, L.PACK_X3), np.uint8)
    bias = np.zeros(8 * H, np.float32)
    fr = np.zeros(2 * 2 * 4 * H * H * 2, np.uint8)
    arrs = [np.ascontiguousarray(P["pr.de0." + n].numpy(), dtype=np.float32)
            for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w_ih_rev", "w_hh_rev", "b_ih_rev", "b_hh_rev")]
    assert lib.stzs_pack_lstm_x3(*[a.ctypes.data for a in arrs], In, H, ih.ctypes.data, bias.ctypes.data,
                                 fr.ctypes.data) == L.OK
    assert ih.tobytes() == ih_want
    assert fr.tobytes() == f_want


def test_pack_conv_rejects_inapplicable_forms():
    lib = L.load()
    assert lib.stzs_pack_conv_size(22, 128, 7, 0, L.PACK_FRAG32) == 0   # Co % 8
    assert lib.stzs_pack_conv_size(128, 64, 3, 0, L.PACK_LANE16) == 0   # one 128-channel chunk needed
    assert lib.stzs_pack_conv_size(64, 128, 7, 0, L.PACK_NARROW32) == 0  # Co <= 32
    buf = np.zeros(16, np.uint8)
    w = np.zeros(16, np.float32)
    assert lib.stzs_pack_conv(w.ctypes.data, 22, 128, 7, 0, L.PACK_FRAG32, buf.ctypes.data) == L.ESHAPE
    assert lib.stzs_pack_conv(None, 22, 128, 7, 0, L.PACK_NARROW32, buf.ctypes.data) == L.EINVAL


def test_pack_lstm_matches_python(tiny_params):
    from stzs.weights import Arena, pack_lstm
    lib = L.load()
    P = tiny_params
    A = Arena()
    lw = pack_lstm(A, "pr.de0", P)
    A.finalize("cpu")
    ih_want = A[lw.ih.w].contiguous().view(torch.uint8).numpy().tobytes()
    b_want = A[lw.ih.b].numpy()
    f_want = A[lw.whhT].contiguous().view(torch.uint8).numpy().tobytes()
    H, In = lw.H, P["pr.de0.w_ih"].shape[1]
    ih = np.zeros(lib.stzs_pack_conv_size(8 * H, In, 1, 0, L.PACK_KSTEP), np.uint8)
    bias = np.zeros(8 * H, np.float32)
    fr = np.zeros(2 * 4 * H * H * 2, np.uint8)
    arrs = [np.ascontiguousarray(P["pr.de0." + n].numpy(), dtype=np.float32)
            for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w_ih_rev", "w_hh_rev", "b_ih_rev", "b_hh_rev")]
    assert lib.stzs_pack_lstm(*[a.ctypes.data for a in arrs], In, H, ih.ctypes.data, bias.ctypes.data,
                              fr.ctypes.data) == L.OK
    assert ih.tobytes() == ih_want
    assert np.array_equal(bias, b_want)
    assert fr.tobytes() == f_want


def _desc(shape, dtype=L.BF16, data=0x1000):
    d = L.Tensor()
    d.data, d.dtype, d.ndim = data, dtype, len(shape)
    st = 1
    for k in range(len(shape) - 1, -1, -1):
        d.shape[k] = shape[k]
        d.stride[k] = st
        st *= shape[k]
    return d


def test_workspace_queries_scale_with_shapes():
    lib = L.load()
    x = _desc((64, 24001, 128))
    p = L.params([128, 3, 7, 11, 1, 3, 5, 3, 3, L.PACK_FRAG32])
    ws = lib.stzs_mrf_resblock_workspace(C.byref(x), 56, C.byref(p))
    act = 64 * 24001 * 128 * 2
    assert 3 * act <= ws <= 3 * act + 64 * 376 * 128 * 8 + 8 * 64 * 128 * 4 + 64 * 376 * 128 * 8 + 16 * 256
    xl = _desc((4, 80, 640))
    assert lib.stzs_bilstm_workspace(C.byref(xl), 4, C.byref(L.params([256]))) >= 4 * 80 * 8 * 256 * 4 + 4096
    F0 = _desc((2, 400), L.F32)
    assert lib.stzs_sine_gen_workspace(C.byref(F0), 3, C.byref(L.params([300, 20, 5, 9]))) >= 2 * 9 * 400 * 4
    assert lib.stzs_cfg_euler_step_workspace(None, 0, None) == 0


@pytest.mark.parametrize("op", L.GENERIC_OPS)
def test_generic_ops_reject_before_launch(op):
    """NULL descriptor arrays / params / required data pointers -> STZS_EINVAL, nothing dereferenced on the device."""
    lib = L.load()
    fn = getattr(lib, f"stzs_{op}")
    p = L.params()
    assert fn(None, 0, None, 0, None, None, 0, None) == L.EINVAL
    ins = (L.Tensor * 60)()   # all data pointers NULL
    outs = (L.Tensor * 2)()
    assert fn(ins, 60 if op == "mrf_resblock" else 6, outs, 2, C.byref(p), C.c_void_p(0x1000), 1 << 30, None) in (
        L.EINVAL, L.ESHAPE)
