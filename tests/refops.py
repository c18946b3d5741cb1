"""Plain-torch fp32 restatements of the C-ABI op semantics (include/stzs.h), used as the numerics
reference for the HIP kernels.  Inputs are pre-rounded to bf16 where the kernel stores bf16, so
the kernel-vs-reference difference is only accumulation order and the output rounding."""
import torch
import torch.nn.functional as F


def bf(x):
    return x.to(torch.bfloat16).float()


def act(x, kind, slope=0.0, alpha=None):
    if kind == "leaky":
        return F.leaky_relu(x, slope)
    if kind == "snake":
        a = alpha[None, :, None]
        return x + torch.sin(a * x) ** 2 / a
    if kind == "gelu":
        return F.gelu(x)
    if kind == "silu":
        return F.silu(x)
    return x


def conv_ref(x_ntc, w, b, *, pad=0, dil=1, stride=1, sc=None, sh=None, pro_act=None, slope=0.0, alpha=None,
             epi_act=None, gate=None, res=None, res_tdiv=1, out_scale=1.0, acc_in=None, beta=0.0):
    """x [B, T, Ci] (fp32 holding bf16 values), w [Co, Ci, k] -> [B, T_out, Co] fp32."""
    x = x_ntc.transpose(1, 2)
    if sc is not None:
        x = x * sc[:, :, None] + sh[:, :, None]
    x = act(x, pro_act, slope, alpha)
    x = bf(x)
    y = F.conv1d(x, bf(w), b, stride=stride, padding=pad, dilation=dil).transpose(1, 2)
    y = act(y, epi_act)
    if gate is not None:
        y = y * gate[:, None, :]
    if res is not None:
        r = res
        if res_tdiv > 1:
            r = r.repeat_interleave(res_tdiv, dim=1)[:, : y.shape[1]]
        y = y + r
    y = y * out_scale
    if acc_in is not None:
        y = y + beta * acc_in
    return y


def convT_ref(x_ntc, w, b, *, stride, pad, refl=0, pro_act=None, slope=0.0, res=None):
    x = bf(act(x_ntc.transpose(1, 2), pro_act, slope))
    y = F.conv_transpose1d(x, bf(w), b, stride=stride, padding=pad)
    if refl:
        y = F.pad(y, (1, 0), mode="reflect")
    y = y.transpose(1, 2)
    if res is not None:
        y = y + res
    return y


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def max_rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
