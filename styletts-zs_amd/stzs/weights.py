"""Weight packing: torch-native parameter dict -> one contiguous device arena of kernel layouts.

Layouts (see include/stzs.h):
  * conv / linear : bf16 [ks][co_pad][ci_pad]  (ci chunk cic = 32|64, co padded to the tile)
  * ConvTranspose1d(k = 2s): polyphase bf16 [2][s*Co][ci_pad]  W'[0][p*Co+co] = W[:, co, p+s],
                             W'[1][p*Co+co] = W[:, co, p]
  * LSTM          : W_ih of both directions as one linear [8H, in] with bias b_ih + b_hh, and
                    W_hh^T fp32 [2][H][4H]
  * AdaIN fcs     : every norm fc of a stage concatenated into ONE linear (style -> sum 2C), so
                    all gamma/beta of a stage come from one GEMM per utterance batch
The arena is a single uint8 tensor (256-B aligned sub-buffers) so that multi-GPU runs move all
weights with ONE RCCL broadcast; its layout depends only on the spec, so every
rank can build the views before receiving the bytes.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass
from typing import Optional

import torch

from .frontend import mel_filterbank
from .spec import Spec

ALIGN = 256


def _rup(x, m):
    return (x + m - 1) // m * m


@dataclass
class ConvW:
    w: object            # name in arena (resolved to a tensor view)
    b: Optional[object]
    Ci: int
    Co: int
    ks: int
    ci_pad: int
    co_pad: int
    cic: int
    ups: int = 0
    lane16: bool = False  # packed with the MRF kernel's channel permutation (STZS_CONV_W_LANE16)
    narrow32: bool = False  # [NK][32][32] narrow packing (STZS_CONV_W_NARROW32)
    wscale: Optional[object] = None  # fp8 linears: per-output-column fp32 scale [co_pad]
    f8: bool = False
    w32: Optional[object] = None  # fp32 K-step stream (STZS_CONV_W_F32, conv_f32), unpermuted
    frag32: bool = False  # fragment-order packing of the register-direct MRF kernel (STZS_CONV_W_FRAG32)
    wx3: Optional[object] = None  # precise mode: hi | lo bf16 K-step streams (STZS_CONV_W_X3, conv_x3), unpermuted
    fx3: Optional[object] = None  # precise mode, register-direct: hi | lo FRAG32 blocks per K-step (STZS_CONV_W_FRAG32X3)
    nz32: Optional[object] = None  # fused noise conv (STZS_CONV_UPS_NOISE): its fp32 weights [Co][32]


class Arena:
    """Collects CPU tensors, lays them out in one buffer, uploads once."""

    def __init__(self):
        self.items: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        self.views = {}
        self.buf = None

    def add(self, name, t: torch.Tensor):
        assert name not in self.items, name
        self.items[name] = t.contiguous()
        return name

    def layout(self):
        off = 0
        lay = OrderedDict()
        for k, t in self.items.items():
            nb = t.numel() * t.element_size()
            lay[k] = (off, nb)
            off = _rup(off + nb, ALIGN)
        return lay, off

    def finalize(self, device, fill=True):
        lay, total = self.layout()
        host = torch.zeros(total, dtype=torch.uint8)
        if fill:
            for k, t in self.items.items():
                o, nb = lay[k]
                host[o:o + nb] = t.reshape(-1).view(torch.uint8)
        self.buf = host.to(device)
        for k, t in self.items.items():
            o, nb = lay[k]
            self.views[k] = self.buf[o:o + nb].view(t.dtype).view(t.shape)
        self.items = OrderedDict((k, None) for k in self.items)  # drop host copies
        return self

    def __getitem__(self, k):
        return self.views[k]


_GSWZ = (0, 2, 3, 1)


def kstep_stream(wp: torch.Tensor, cic: int) -> torch.Tensor:
    """[ks, co_pad, ci_pad] -> [co_pad/128, NK, 128, 32] K-step stream in the kernel's loop order
    (ci chunk, tap, 32-wide k-step), each 8-KB K-step already in its LDS image order: the 16-B
    chunk c of row r sits at position c ^ g((r >> 2) & 3), g = (0, 2, 3, 1) -- the XOR swizzle
    that makes the 16x16x32 B-fragment ds_read_b128 conflict-free (csrc/conv.hip)."""
    ks, co_pad, ci_pad = wp.shape
    ncot, nchunk, kpc = co_pad // 128, ci_pad // cic, cic // 32
    t = wp.view(ks, ncot, 128, nchunk, kpc, 4, 8).permute(1, 3, 0, 4, 2, 5, 6)  # cot, cc, tap, kq, r, c, 8
    r = torch.arange(128)
    g = torch.tensor(_GSWZ)[(r >> 2) & 3]
    p = torch.arange(4)
    src_c = p[None, :] ^ g[:, None]                                            # [128, 4]: position -> chunk
    t = t[:, :, :, :, r[:, None], src_c, :]
    return t.reshape(ncot, nchunk * ks * kpc, 128, 32).contiguous()


def kstep_stream_f32(wp: torch.Tensor) -> torch.Tensor:
    """[ks, co_pad, ci_pad] fp32 -> [co_pad/128, ci_pad/32, ks, 128, 32]: the precise-mode conv's K-steps
    (csrc/conv.hip conv_f32) in its loop order (32-channel chunk, tap), natural row / channel order."""
    ks, co_pad, ci_pad = wp.shape
    t = wp.float().view(ks, co_pad // 128, 128, ci_pad // 32, 32).permute(1, 3, 0, 2, 4)
    return t.contiguous()


def split_bf16(w: torch.Tensor):
    """fp32 -> (hi, lo) bf16 with hi = bf16(w), lo = bf16(w - hi): w = hi + lo to ~2^-17 relative (the
    split-operand precise mode, csrc/conv.hip conv_x3 / csrc/lstm.hip)."""
    w = w.float()
    hi = w.to(torch.bfloat16)
    return hi, (w - hi.float()).to(torch.bfloat16)


def kstep_stream_x3(wp: torch.Tensor) -> torch.Tensor:
    """[ks, co_pad, ci_pad] fp32 -> [2, co_pad/128, ci_pad/32 * ks, 128, 32] bf16: the hi stream, then the lo
    stream, each the 32-channel-chunk K-step layout of kstep_stream (include/stzs.h STZS_CONV_W_X3)."""
    hi, lo = split_bf16(wp)
    return torch.stack([kstep_stream(hi.float(), 32), kstep_stream(lo.float(), 32)]).to(torch.bfloat16)


def lane16_perm() -> torch.Tensor:
    """packed row rr = wc*64 + nt*16 + g*4 + r of a 128-column tile holds output channel
    wc*64 + g*16 + nt*4 + r: the MRF kernel's swapped-operand accumulators then give each lane 16
    consecutive channels of one time step (include/stzs.h STZS_CONV_W_LANE16, csrc/mrf.hip)."""
    rr = torch.arange(128)
    return (rr & 64) + ((rr >> 2) & 3) * 16 + ((rr >> 4) & 3) * 4 + (rr & 3)


def frag32_perm() -> torch.Tensor:
    """packed row rr = w*32 + nt*16 + g*4 + r of a 128-column tile holds output channel w*32 + g*8 + nt*4 + r:
    in the register-direct MRF kernel (csrc/mrfv.hip) wave w owns packed rows [32w, 32w + 32) and its
    swapped-operand accumulators then give lane group g 8 consecutive channels of one time step."""
    rr = torch.arange(128)
    return (rr & 96) + ((rr >> 2) & 3) * 8 + ((rr >> 4) & 1) * 4 + (rr & 3)


def frag32_stream(wp: torch.Tensor) -> torch.Tensor:
    """[ks, co_pad, ci_pad] (rows already frag32-permuted) -> [co_pad/128, ci_pad/128 * ks * 4 * 512, 8]: per
    (co tile, 128-channel chunk, tap, 32-wide k-step) the 16x16x32 A-fragments of the 4 waves x 2 row tiles in
    lane order -- lane l = g*16 + i holds packed row w*32 + nt*16 + i, channels kq*32 + 8g .. + 8 -- so each
    fragment is one coalesced 16-B load per lane (include/stzs.h STZS_CONV_W_FRAG32)."""
    ks, co_pad, ci_pad = wp.shape
    t = wp.reshape(ks, co_pad // 128, 4, 2, 16, ci_pad // 128, 4, 4, 8)  # tap, cot, w, nt, i, chunk, kq, g, e
    t = t.permute(1, 5, 0, 6, 2, 3, 7, 4, 8)                              # cot, chunk, tap, kq, w, nt, g, i, e
    return t.reshape(co_pad // 128, -1, 8).contiguous()


def frag32x3_stream(wp: torch.Tensor) -> torch.Tensor:
    """[ks, co_pad, ci_pad] fp32 (rows already frag32-permuted) -> [co_pad/128, NK * 1024, 8] bf16: per 32-wide
    K-step (the frag32_stream order) the hi fragment block [4 waves][2][64 lanes][8] of bf16(w), then the lo block of
    bf16(w - hi) -- one K-step of both halves adjacent for the precise register-direct kernel (csrc/mrfx.hip,
    include/stzs.h STZS_CONV_W_FRAG32X3)."""
    hi, lo = split_bf16(wp)
    h = frag32_stream(hi.float()).view(wp.shape[1] // 128, -1, 512, 8)
    l = frag32_stream(lo.float()).view(wp.shape[1] // 128, -1, 512, 8)
    return torch.stack([h, l], 2).reshape(wp.shape[1] // 128, -1, 8).to(torch.bfloat16)


def narrow32_stream(wp: torch.Tensor, cic: int) -> torch.Tensor:
    """[ks, 32, ci_pad] -> [NK, 32, 32] K-steps for the narrow conv (csrc/mrf.hip narrow_conv): packed row
    rr = nt*16 + g*4 + r holds output channel g*8 + nt*4 + r; 16-B chunks XOR-swizzled as kstep_stream."""
    ks, _, ci_pad = wp.shape
    rr = torch.arange(32)
    perm = ((rr >> 2) & 3) * 8 + ((rr >> 4) & 1) * 4 + (rr & 3)
    wp = wp[:, perm]
    nchunk, kpc = ci_pad // cic, cic // 32
    t = wp.view(ks, 32, nchunk, kpc, 4, 8).permute(2, 0, 3, 1, 4, 5)  # cc, tap, kq, row, c, 8
    g = torch.tensor(_GSWZ)[(rr >> 2) & 3]
    src_c = torch.arange(4)[None, :] ^ g[:, None]
    t = t[:, :, :, rr[:, None], src_c, :]
    return t.reshape(nchunk * ks * kpc, 32, 32).contiguous()


def pack_conv(A: Arena, name, w, b=None, ups=0, lane16=False, narrow32=False, f32=False, frag32=False,
              x3=False) -> ConvW:
    """w: Conv1d [Co, Ci, k] / Linear [Co, Ci] / ConvTranspose1d [Ci, Co, 2*ups] (ups > 0).
    lane16: the MRF kernel's layout (Ci % 128 == 0, Co % 16 == 0, plain conv).
    f32: also pack the fp32 stream (ConvW.w32, conv_f32); x3: also pack the precise-mode split hi | lo
    streams (ConvW.wx3, conv_x3)."""
    if ups:
        Ci, Co, k = w.shape
        assert k == 2 * ups
        ncol = ups * Co
        wk = torch.empty(2, ncol, Ci)
        for p in range(ups):
            wk[0, p * Co:(p + 1) * Co] = w[:, :, p + ups].t()
            wk[1, p * Co:(p + 1) * Co] = w[:, :, p].t()
        ks = 2
    else:
        if w.dim() == 2:
            w = w[:, :, None]
        Co, Ci, ks = w.shape
        ncol = Co
        wk = w.permute(2, 0, 1)
    cic = 32 if Ci <= 32 else (64 if Ci <= 64 else 128)
    ci_pad = _rup(Ci, cic)
    co_pad = _rup(ncol, 128)
    wp = torch.zeros(ks, co_pad, ci_pad)
    wp[:, :ncol, :Ci] = wk
    w32 = A.add(name + ".w32", kstep_stream_f32(wp)) if f32 else None
    wx3 = A.add(name + ".wx3", kstep_stream_x3(wp)) if x3 else None
    if narrow32:
        assert not ups and cic == 128 and Co <= 32, (name, Ci, Co)
        wn = A.add(name + ".wpk", narrow32_stream(wp[:, :32], cic).to(torch.bfloat16))
        bn = A.add(name + ".bpk", b.float().clone()) if b is not None else None
        fx3 = None  # precise: the narrow register-direct split-operand form (csrc/mrfx.hip, conv_post)
        if x3 and ks in (3, 7, 11):
            wf = wp.view(ks, co_pad // 128, 128, ci_pad)[:, :, frag32_perm()].reshape(ks, co_pad, ci_pad)
            fx3 = A.add(name + ".wfx3", frag32x3_stream(wf))
        return ConvW(wn, bn, Ci, Co, ks, ci_pad, co_pad, cic, ups, False, True, w32=w32, wx3=wx3, fx3=fx3)
    if frag32:  # register-direct MRF convs (csrc/mrfv.hip) and the polyphase ConvTranspose (csrc/ups.hip, ups > 0)
        assert cic == 128 and ((not ups and Co % 8 == 0 and ks in (1, 3, 7, 11)) or (ups and Co % 32 == 0)), \
            (name, Ci, Co, ks, ups)
        wp = wp.view(ks, co_pad // 128, 128, ci_pad)[:, :, frag32_perm()].reshape(ks, co_pad, ci_pad)
        wn = A.add(name + ".wfr", frag32_stream(wp).to(torch.bfloat16))
        bn = A.add(name + ".bpk", b.float().clone()) if b is not None else None
        # the precise register-direct form (csrc/mrfx.hip) of the plain convs
        fx3 = A.add(name + ".wfx3", frag32x3_stream(wp)) if (x3 and not ups) else None
        return ConvW(wn, bn, Ci, Co, ks, ci_pad, co_pad, cic, ups, False, w32=w32, frag32=True, wx3=wx3, fx3=fx3)
    # the precise register-direct FLAT linear (csrc/mrfx.hip mrfx_lin): ks 1, 128-channel chunks
    fx3 = None
    if x3 and ks == 1 and not ups and cic == 128 and Co % 8 == 0:
        wf = wp.view(ks, co_pad // 128, 128, ci_pad)[:, :, frag32_perm()].reshape(ks, co_pad, ci_pad)
        fx3 = A.add(name + ".wfx3", frag32x3_stream(wf))
    if lane16:
        assert cic == 128 and Co % 16 == 0, (name, Ci, Co)
        perm = lane16_perm()
        wp = wp.view(ks, co_pad // 128, 128, ci_pad)[:, :, perm].reshape(ks, co_pad, ci_pad)
    wn = A.add(name + ".wpk", kstep_stream(wp, cic).to(torch.bfloat16))
    bn = A.add(name + ".bpk", b.float().clone()) if b is not None else None
    return ConvW(wn, bn, Ci, Co, ks, ci_pad, co_pad, cic, ups, lane16, w32=w32, wx3=wx3, fx3=fx3)


def noise_super_weights(wn: torch.Tensor, s: int, ld: int) -> torch.Tensor:
    """the strided noise conv of a non-last generator stage -- Conv1d(C_har -> Co, k = 2 s, stride s, pad (s + 1) // 2)
    over the harmonic-source rows -- restated on SUPER-ROWS of s consecutive rows (s ld channels: row pos*ld + c) as a
    k3 stride-1 conv with padding 1: out[t] = sum_tap W'[tap] . super[t + tap - 1], where tap's position pos holds
    the original tap j = s (tap - 1) + pos + pad (zero where j falls outside [0, 2 s), and for c >= C_har).
    -> W' [Co, s ld, 3]"""
    Co, Ch, k = wn.shape
    assert k == 2 * s and Ch <= ld
    pad = (s + 1) // 2
    w = torch.zeros(Co, s * ld, 3)
    for tap in range(3):
        for pos in range(s):
            j = s * (tap - 1) + pos + pad
            if 0 <= j < k:
                w[:, pos * ld:pos * ld + Ch, tap] = wn[:, :, j]
    return w


def pack_ups_noise(A: Arena, name, wu, bu, wn, bn) -> ConvW:
    """the last generator stage's polyphase ConvTranspose1d with its 1x1 noise conv fused (csrc/ups.hip,
    STZS_CONV_UPS_NOISE): wu [Ci, Co, 2 r] / bu [Co] the ConvTranspose, wn [Co, C_har, 1] / bn [Co] the noise conv.
    Weight stream: per 128-column tile the r-phase ConvTranspose K-steps (pack_conv(ups=r, frag32=True)) followed by
    ONE K-step of the noise conv's weights for the tile's channels (C_har <= 32, zero-padded), fragment order; the
    bias is bu + bn; nz32 keeps the (bf16-rounded) noise weights in fp32 [Co][32] (the ReflectionPad(1,0) row's
    correction)."""
    Ci, Co, k = wu.shape
    r = k // 2
    Ch = wn.shape[1]
    assert Co % 128 == 0 and Ch <= 32 and wn.shape[0] == Co, (name, wu.shape, wn.shape)
    ncol = r * Co
    co_pad = _rup(ncol, 128)
    wk = torch.empty(2, ncol, Ci)
    for ph in range(r):
        wk[0, ph * Co:(ph + 1) * Co] = wu[:, :, ph + r].t()
        wk[1, ph * Co:(ph + 1) * Co] = wu[:, :, ph].t()
    ci_pad = _rup(Ci, 128)
    wp = torch.zeros(2, co_pad, ci_pad)
    wp[:, :ncol, :Ci] = wk
    wp = wp.view(2, co_pad // 128, 128, ci_pad)[:, :, frag32_perm()].reshape(2, co_pad, ci_pad)
    su = frag32_stream(wp)                                       # [nct, NK * 512, 8]
    wnp = torch.zeros(1, co_pad, 128)
    for ph in range(r):
        wnp[0, ph * Co:(ph + 1) * Co, :Ch] = wn[:, :, 0]
    wnp = wnp.view(1, co_pad // 128, 128, 128)[:, :, frag32_perm()].reshape(1, co_pad, 128)
    sn = frag32_stream(wnp)[:, :512]                             # k-step 0 (k 0..31) of every tile
    wname = A.add(name + ".wfrn", torch.cat([su, sn], 1).to(torch.bfloat16))
    bname = A.add(name + ".bpkn", (bu.float() + bn.float()).clone())
    w32 = torch.zeros(Co, 32)
    w32[:, :Ch] = wn[:, :, 0].to(torch.bfloat16).float()  # the MFMA K-step's (bf16) weights, in fp32
    nz = A.add(name + ".nz32", w32)
    return ConvW(wname, bname, Ci, Co, 2, ci_pad, co_pad, 128, r, False, frag32=True, nz32=nz)


def quantize_f8_cols(w: torch.Tensor):
    """Linear [Co, Ci] fp32 -> (e4m3fn codes [Co, Ci], per-output-channel scale [Co]):
    scale = max|w_co| / 448 (1 for an all-zero row), codes = e4m3fn(clamp(w / scale, +-448)) (RNE)."""
    amax = w.abs().amax(1)
    scale = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (w / scale[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    return q, scale


def kstep_stream_f8(q: torch.Tensor) -> torch.Tensor:
    """e4m3fn [co_pad, ci_pad] (as uint8) -> [co_pad/128, ci_pad/64, 128, 64]: the 64-k K-steps of the fp8
    GEMM (csrc/conv.hip gemm_glds<F8>), 16-B chunk c of row r at position c ^ g((r >> 2) & 3) exactly as
    kstep_stream (a K-step row is 64 B in both dtypes: 32 bf16 or 64 fp8 values)."""
    co_pad, ci_pad = q.shape
    ncot, nk = co_pad // 128, ci_pad // 64
    t = q.view(ncot, 128, nk, 4, 16).permute(0, 2, 1, 3, 4)  # cot, kstep, r, c, 16
    r = torch.arange(128)
    g = torch.tensor(_GSWZ)[(r >> 2) & 3]
    src_c = torch.arange(4)[None, :] ^ g[:, None]
    t = t[:, :, r[:, None], src_c, :]
    return t.reshape(ncot, nk, 128, 64).contiguous()


def pack_conv_f8(A: Arena, name, w, b=None) -> ConvW:
    """fp8 e4m3fn Linear [Co, Ci] for the configs[4] denoiser (include/stzs.h stzs_conv_args.w_scale)."""
    Co, Ci = w.shape
    ci_pad, co_pad = _rup(Ci, 64), _rup(Co, 128)
    q, sc = quantize_f8_cols(w.float())
    qp = torch.zeros(co_pad, ci_pad, dtype=torch.uint8)
    qp[:Co, :Ci] = q.view(torch.uint8)
    scp = torch.ones(co_pad)
    scp[:Co] = sc
    wn = A.add(name + ".wf8", kstep_stream_f8(qp))
    sn = A.add(name + ".sf8", scp)
    bn = A.add(name + ".bf8", b.float().clone()) if b is not None else None
    return ConvW(wn, bn, Ci, Co, 1, ci_pad, co_pad, 64, wscale=sn, f8=True)


def dft_basis(n_fft: int, win: int) -> torch.Tensor:
    """Linear [2 * nbin, win]: rows k < nbin = cos(2 pi k n / n_fft), rows nbin + k = -sin(...), n = (n_fft - win) / 2
    + m the position of window sample m inside the frame -> (Re | Im) of the n_fft-point DFT of a windowed
    frame (torch.stft's zero-padded centred window; the window itself is applied by stzs_stft_frames)."""
    nbin = n_fft // 2 + 1
    n = torch.arange(win, dtype=torch.float64) + (n_fft - win) // 2
    k = torch.arange(nbin, dtype=torch.float64)[:, None]
    ang = 2.0 * math.pi * ((k * n[None, :]) % n_fft) / n_fft
    return torch.cat([torch.cos(ang), -torch.sin(ang)], 0).float()


@dataclass
class NormGroup:
    """all AdaIN fc layers of one stage, packed as one linear; offsets per norm name."""
    lin: ConvW
    offsets: dict
    total: int


def pack_norm_group(A: Arena, name, P, norm_names, style_dim, x3=False) -> NormGroup:
    ws, bs, offs, off = [], [], {}, 0
    for n in norm_names:
        w, b = P[n + ".w"], P[n + ".b"]
        offs[n] = (off, w.shape[0] // 2)
        off += w.shape[0]
        ws.append(w)
        bs.append(b)
    W = torch.cat(ws, 0)
    Bv = torch.cat(bs, 0)
    return NormGroup(pack_conv(A, name, W, Bv, x3=x3), offs, off)


@dataclass
class LstmW:
    ih: ConvW
    whhT: str
    H: int
    whx3: Optional[str] = None  # precise mode: hi fragments of both directions, then lo (stzs_lstm_args.precise)


def pack_lstm(A: Arena, name, P, x3=False) -> LstmW:
    H = P[name + ".w_hh"].shape[1]
    wih = torch.cat([P[name + ".w_ih"], P[name + ".w_ih_rev"]], 0)
    bias = torch.cat([P[name + ".b_ih"] + P[name + ".b_hh"], P[name + ".b_ih_rev"] + P[name + ".b_hh_rev"]], 0)
    ih = pack_conv(A, name + ".ih", wih, bias, x3=x3)
    frags = torch.stack([lstm_frags(P[name + ".w_hh"]), lstm_frags(P[name + ".w_hh_rev"])], 0)
    whx3 = None
    if x3:
        parts = [split_bf16(P[name + ".w_hh"]), split_bf16(P[name + ".w_hh_rev"])]
        hl = [torch.stack([lstm_frags(parts[d][h].float()) for d in range(2)], 0) for h in range(2)]
        whx3 = A.add(name + ".whhx3", torch.stack(hl, 0).to(torch.bfloat16))
    return LstmW(ih, A.add(name + ".whhT", frags.to(torch.bfloat16)), H, whx3)


def lstm_frags(w_hh: torch.Tensor) -> torch.Tensor:
    """W_hh [4H, H] -> W_hh^T as 16x16x32 B fragments [4H/16][H/32][64 lanes][8]:
    lane l, element j holds W_hh[n = ct*16 + (l & 15)][k = ks*32 + 8*(l >> 4) + j] (csrc/lstm.hip)."""
    G4, H = w_hh.shape
    t = w_hh.reshape(G4 // 16, 16, H // 32, 4, 8).permute(0, 2, 3, 1, 4)
    return t.reshape(G4 // 16, H // 32, 64, 8).contiguous()


def blk_norms(prefix):
    return [prefix + ".norm1", prefix + ".norm2"]


@dataclass
class BlkW:
    """AdainResBlk1d"""
    name: str
    din: int
    dout: int
    up: bool
    conv1: ConvW
    conv2: ConvW
    sc: Optional[ConvW]
    pool_w: Optional[str]
    pool_b: Optional[str]
    # the register-direct (frag32) convs again in the generic conv_mfma layout: the batch-1 engine runs them split-K
    # over input-channel chunks (StyleTTSZS(blk_splitk=...)): a 5-s utterance's decoder conv is 16 tiles otherwise
    conv1s: Optional[ConvW] = None
    conv2s: Optional[ConvW] = None
    scs: Optional[ConvW] = None  # (the shortcut likewise, when it is on the register-direct form)


def _lane16_ok(w) -> bool:
    """conv eligible for the MRF-family kernel (csrc/mrf.hip): 128-channel input chunks, Co % 16 == 0."""
    Co, Ci = w.shape[0], w.shape[1]
    return Ci > 64 and Co % 16 == 0


def _frag32_ok(w) -> bool:
    """AdaIN-block conv eligible for the register-direct kernel (csrc/mrfv.hip, bit-identical to csrc/mrf.hip):
    k3, 128-channel input chunks, Co % 32 == 0.  Faster on every decoder / predictor block shape at the bench batch
    (tools/blk_bench.py, B = 64: dec.encode.conv1 103 -> 83 us, decode conv1 155 -> 143, conv2 135 -> 125, decode3
    conv2 79 -> 65, predictor 45 -> 39 and 28 -> 24).  csrc/abi_ops.hip blk_form applies the same rule."""
    Co, Ci = w.shape[0], w.shape[1]
    return w.shape[2] == 3 and Ci > 64 and Co % 32 == 0


def pack_blk(A: Arena, P, name, up=False, x3=False) -> BlkW:
    w1, w2 = P[name + ".conv1.w"], P[name + ".conv2.w"]
    f1, f2 = _frag32_ok(w1), _frag32_ok(w2)
    c1 = pack_conv(A, name + ".conv1", w1, P[name + ".conv1.b"], lane16=_lane16_ok(w1) and not f1, frag32=f1, x3=x3)
    c2 = pack_conv(A, name + ".conv2", w2, P[name + ".conv2.b"], lane16=_lane16_ok(w2) and not f2, frag32=f2, x3=x3)
    # the 1x1 shortcut on the register-direct form too (r06, tools/sc_bench.py: the decoder's 1090 -> 1024 shortcut
    # 100 us on the generic conv -- its 1090-channel rows are too narrow for the LDS-DMA GEMM -- vs 52 us; the
    # encode block's 514 -> 1024 68 vs 33 us; the same bits as the GEMM forms)
    wsc = P.get(name + ".sc.w")
    fs = wsc is not None and not x3 and wsc.shape[1] > 64 and wsc.shape[0] % 32 == 0
    sc = pack_conv(A, name + ".sc", wsc, x3=x3, frag32=fs) if wsc is not None else None
    scs = pack_conv(A, name + ".scs", wsc) if fs else None
    c1s = pack_conv(A, name + ".conv1s", w1, P[name + ".conv1.b"]) if f1 and not x3 else None
    c2s = pack_conv(A, name + ".conv2s", w2, P[name + ".conv2.b"]) if f2 and not x3 else None
    pw = pb = None
    if up:
        pw = A.add(name + ".poolw", P[name + ".pool.w"].reshape(-1, 3).float())
        pb = A.add(name + ".poolb", P[name + ".pool.b"].float())
    din = P[name + ".conv1.w"].shape[1]
    dout = P[name + ".conv1.w"].shape[0]
    return BlkW(name, din, dout, up, c1, c2, sc, pw, pb, c1s, c2s, scs)


class PackedModel:
    """All hot-path weights of spec v0 in kernel layouts, resident in one device arena."""

    def __init__(self, spec: Spec, P, device, fill=True, precise=False, precise_all=False, lowp_denoiser=False):
        """precise: also pack the split-operand (hi | lo) streams of every decoder conv (StyleTTSZS(
        precise_decoder=True)); precise_all: of every conv, linear and LSTM of the pipeline except the
        reference-prompt front end, whose output is quantised to discrete codes (StyleTTSZS(precise=True)).
        lowp_denoiser (with precise_all): the denoiser's linears without the split streams -- the configs[4]
        long-form mode StyleTTSZS(precise=True, fp8_denoiser=True): fp8 sampler, precise text / prosody / decoder."""
        S = self.spec = spec
        xd = precise or precise_all
        xa = precise_all
        A = self.arena = Arena()
        d = S.dn_d
        # --- text encoder ---
        self.te_emb = A.add("te.emb", P["te.emb"].float())
        self.te_conv = [pack_conv(A, f"te.conv{i}", P[f"te.conv{i}.w"], P[f"te.conv{i}.b"], x3=xa)
                        for i in range(S.te_layers)]
        self.te_ln = [(A.add(f"te.ln{i}.g", P[f"te.ln{i}.g"]), A.add(f"te.ln{i}.b", P[f"te.ln{i}.b"])) for i in range(S.te_layers)]
        self.te_lstm = pack_lstm(A, "te.lstm", P, x3=xa)
        # --- reference-prompt front end (csrc/frontend.hip): DFT basis, window, mel filterbank, encoder ---
        self.fe_dft = pack_conv(A, "fe.dft", dft_basis(S.mel_nfft, S.mel_win))
        self.fe_win = A.add("fe.win", torch.hann_window(S.mel_win).float())
        fb = mel_filterbank(S.n_mels, S.mel_nfft, S.sr)
        nz = fb > 0
        rng = torch.zeros(S.n_mels, 2, dtype=torch.int32)
        for m in range(S.n_mels):
            idx = nz[m].nonzero()
            if len(idx):
                rng[m, 0], rng[m, 1] = int(idx[0]), int(idx[-1]) + 1
        self.fe_fb = A.add("fe.fb", fb.contiguous())
        self.fe_rng = A.add("fe.fbr", rng)
        self.pe_conv0 = pack_conv(A, "pe.conv0", P["pe.conv0.w"], P["pe.conv0.b"])
        self.pe_conv1 = pack_conv(A, "pe.conv1", P["pe.conv1.w"], P["pe.conv1.b"])
        self.pe_proj = pack_conv(A, "pe.proj", P["pe.proj.w"], P["pe.proj.b"])
        self.pe_vq = A.add("pe.vq", P["pe.vq"].float())  # [G][K][dg] codebooks (stzs_code_quantize)
        # --- denoiser ---
        L = lambda n: pack_conv(A, n, P[n + ".w"], P[n + ".b"], x3=xa)
        xdn = xa and not lowp_denoiser
        Ld = lambda n: pack_conv(A, n, P[n + ".w"], P[n + ".b"], x3=xdn)
        self.dn_in = Ld("dn.in_proj")
        self.dn_pos = A.add("dn.pos", P["dn.pos"].float())
        self.dn_t0, self.dn_t1 = Ld("dn.t_mlp0"), Ld("dn.t_mlp1")
        self.dn_pool = Ld("dn.pool_proj")
        self.dn_ctx_txt, self.dn_ctx_prm = Ld("dn.ctx_txt"), Ld("dn.ctx_prm")
        self.dn_ada = Ld("dn.ada")
        self.dn_table = A.add("dn.ada_table", P["dn.ada_table"].float())
        self.dn_final_ada = Ld("dn.final_ada")
        self.dn_out = Ld("dn.out")
        # constant unconditional-branch context: null codes through ctx_prm / pool_proj (fp32, once)
        null = P["dn.null_codes"].float()
        ctx_null = null @ P["dn.ctx_prm.w"].t() + P["dn.ctx_prm.b"]
        pool_null = null.mean(0) @ P["dn.pool_proj.w"].t() + P["dn.pool_proj.b"]
        self.dn_ctx_null = A.add("dn.ctx_null", ctx_null.to(torch.bfloat16))
        self.dn_pool_null = A.add("dn.pool_null", pool_null.float())
        self.dn_ctx_null32 = A.add("dn.ctx_null32", ctx_null.float()) if xdn else None
        self.dn_layers = []
        for l in range(S.dn_layers):
            p = f"dn.l{l}"
            self.dn_layers.append(dict(
                qkv=Ld(p + ".sa_qkv"), o=Ld(p + ".sa_o"), q=Ld(p + ".ca_q"), kv=Ld(p + ".ca_kv"), co=Ld(p + ".ca_o"),
                ff1=Ld(p + ".ff1"), ff2=Ld(p + ".ff2"),
                ln_g=A.add(p + ".ca_ln.g", P[p + ".ca_ln.g"]), ln_b=A.add(p + ".ca_ln.b", P[p + ".ca_ln.b"])))
            # fp8 e4m3fn copies of the per-layer linears (configs[4]: StyleTTSZS(fp8_denoiser=True))
            for key, n in (("qkv", ".sa_qkv"), ("o", ".sa_o"), ("q", ".ca_q"), ("co", ".ca_o"), ("ff1", ".ff1"),
                           ("ff2", ".ff2")):
                self.dn_layers[-1][key + "8"] = pack_conv_f8(A, p + n + ".f8", P[p + n + ".w"], P[p + n + ".b"])
        # (r06) every layer's cross-attention K / V projection of the one shared context as ONE linear: the layers'
        # [2 d, d] weights stacked along the output channels (2 d is a multiple of the 128-column tile, so each tile is
        # the K-step stream of its own layer's linear: the same bits, one launch instead of dn_layers)
        kvw = [P[f"dn.l{l}.ca_kv.w"] for l in range(S.dn_layers)]
        kvb = [P[f"dn.l{l}.ca_kv.b"] for l in range(S.dn_layers)]
        self.dn_kv_all = pack_conv(A, "dn.ca_kv_all", torch.cat(kvw), torch.cat(kvb), x3=xdn) \
            if (2 * d) % 128 == 0 else None
        # --- predictor ---
        self.pr_de = [pack_lstm(A, f"pr.de{i}", P, x3=xa) for i in range(S.pr_layers)]
        self.pr_aln = [L(f"pr.de{i}.aln") for i in range(S.pr_layers)]
        # (r06) the duration encoder's AdaLN projections all read the same style columns: one stacked linear (each
        # 128-column tile its own layer's K-step stream -- same bits, one launch instead of pr_layers)
        self.pr_aln_all = pack_conv(A, "pr.de.aln_all", torch.cat([P[f"pr.de{i}.aln.w"] for i in range(S.pr_layers)]),
                                    torch.cat([P[f"pr.de{i}.aln.b"] for i in range(S.pr_layers)]), x3=xa) \
            if (2 * S.pr_hid) % 128 == 0 else None
        self.pr_dur_lstm = pack_lstm(A, "pr.dur_lstm", P, x3=xa)
        self.pr_dur_proj = L("pr.dur_proj")
        self.pr_shared = pack_lstm(A, "pr.shared", P, x3=xa)
        pr_norms = []
        self.pr_blk = {}
        for br in ("f0", "n"):
            for i in range(3):
                nm = f"pr.{br}{i}"
                self.pr_blk[nm] = pack_blk(A, P, nm, up=(i == 1), x3=xa)
                pr_norms += blk_norms(nm)
            self.pr_blk[f"pr.{br}_proj"] = pack_conv(A, f"pr.{br}_proj", P[f"pr.{br}_proj.w"], P[f"pr.{br}_proj.b"],
                                                     x3=xa)
        self.pr_norm = pack_norm_group(A, "pr.norms", P, pr_norms, S.style_pr, x3=xa)
        # --- decoder ---
        self.dec_f0 = A.add("dec.f0c", torch.cat([P["dec.f0_conv.w"].reshape(-1), P["dec.f0_conv.b"]]).float())
        self.dec_n = A.add("dec.nc", torch.cat([P["dec.n_conv.w"].reshape(-1), P["dec.n_conv.b"]]).float())
        self.dec_asr_res = pack_conv(A, "dec.asr_res", P["dec.asr_res.w"], P["dec.asr_res.b"], x3=xd)
        dec_norms = []
        self.dec_blk = {}
        for nm, up in [("dec.encode", False), ("dec.decode0", False), ("dec.decode1", False),
                       ("dec.decode2", False), ("dec.decode3", True)]:
            self.dec_blk[nm] = pack_blk(A, P, nm, up=up, x3=xd)
            dec_norms += blk_norms(nm)
        self.src_merge = A.add("gen.src_merge", torch.cat([P["gen.src_merge.w"].reshape(-1), P["gen.src_merge.b"]]).float())
        self.noise_conv, self.ups, self.rb, self.ups_nz, self.noise_sup = [], [], [], [], []
        for i, (r, k) in enumerate(zip(S.up_rates, S.up_kernels)):
            self.noise_conv.append(pack_conv(A, f"gen.noise_conv{i}", P[f"gen.noise_conv{i}.w"], P[f"gen.noise_conv{i}.b"],
                                             x3=xd))
            # a strided noise conv restated on super-rows of the harmonic source (k3 stride 1 over s*32 channels, the
            # register-direct kernel; engine.upsample): bf16 engines
            sf0 = math.prod(S.up_rates[i + 1:])
            wn0 = P[f"gen.noise_conv{i}.w"]
            self.noise_sup.append(
                pack_conv(A, f"gen.noise_sup{i}", noise_super_weights(wn0, sf0, 32), P[f"gen.noise_conv{i}.b"],
                          frag32=True)
                if (i < len(S.up_rates) - 1 and not xd and wn0.shape[2] == 2 * sf0 and wn0.shape[1] <= 32 and
                    sf0 * 32 > 128 and wn0.shape[0] % 8 == 0) else None)
            wu = P[f"gen.ups{i}.w"]  # ConvTranspose1d [Ci, Co, 2r]
            # 128-channel input chunks, Co % 32 == 0: the input-staged-once polyphase kernel (csrc/ups.hip)
            self.ups.append(pack_conv(A, f"gen.ups{i}", wu, P[f"gen.ups{i}.b"], ups=r,
                                      frag32=wu.shape[0] > 64 and wu.shape[1] % 32 == 0,
                                      lane16=wu.shape[0] > 64 and wu.shape[1] % 16 == 0 and wu.shape[1] % 32 != 0,
                                      x3=xd))
            # the last stage's ConvTranspose with its 1x1 noise conv fused (the noise conv's 393-MB output and the
            # residual re-read of it at batch 64 never exist): bf16 engines
            wn = P[f"gen.noise_conv{i}.w"]
            last = i == len(S.up_rates) - 1
            self.ups_nz.append(pack_ups_noise(A, f"gen.ups{i}", wu, P[f"gen.ups{i}.b"], wn, P[f"gen.noise_conv{i}.b"])
                               if last and wn.shape[2] == 1 and wn.shape[1] <= 32 and wu.shape[1] % 128 == 0 and
                               wu.shape[0] % 128 == 0 else None)
            stage = []
            for j, kr in enumerate(S.rb_kernels):
                res = []
                for m, dil in enumerate(S.rb_dils):
                    p = f"gen.rb{i}.{j}.{m}"
                    l16 = S.gen_ch[i] % 128 == 0 and (kr - 1) * dil <= 64  # MRF kernel (csrc/mrf.hip)
                    # the register-direct MRF kernel (csrc/mrfv.hip; bit-identical to mrf.hip) for every generator
                    # conv: with one 128-channel input chunk (stage 1: 3 workgroups per CU, 8-18% faster than the
                    # LDS-ring kernel, profiles/r02_mrfv_bench_s.log) and, in its wide form (256 output channels per
                    # workgroup, each staged input row transformed once), with two (stage 0, B = 64,
                    # profiles/r03_r_mrfv_wide.log: k3 c1 131 vs 175 us on the LDS ring, k7 d3 c1 255 vs 279,
                    # k11 d5 c1 352 vs 401, c2 / c2 + accumulate 7-17% faster, k11 c2 level)
                    one = S.gen_ch[i] == 128 and kr in (3, 7, 11) and (kr - 1) * dil <= 64
                    two = S.gen_ch[i] == 256 and kr in (3, 7, 11) and (kr - 1) * dil <= 64
                    fr1 = fr2 = one or two
                    res.append(dict(
                        c1=pack_conv(A, p + ".c1", P[p + ".c1.w"], P[p + ".c1.b"], lane16=l16 and not fr1, frag32=fr1,
                                     x3=xd),
                        c2=pack_conv(A, p + ".c2", P[p + ".c2.w"], P[p + ".c2.b"], lane16=l16 and not fr2, frag32=fr2,
                                     x3=xd),
                        a1=A.add(p + ".a1", P[p + ".alpha1"].float()), a2=A.add(p + ".a2", P[p + ".alpha2"].float()),
                        n1=p + ".n1", n2=p + ".n2", k=kr, dil=dil))
                    dec_norms += [p + ".n1", p + ".n2"]
                stage.append(res)
            self.rb.append(stage)
        wpost = P["gen.conv_post.w"]
        self.conv_post = pack_conv(A, "gen.conv_post", wpost, P["gen.conv_post.b"],
                                   narrow32=wpost.shape[1] > 64 and wpost.shape[0] <= 32, x3=xd)
        self.dec_norm = pack_norm_group(A, "dec.norms", P, dec_norms, S.style_ac, x3=xd)
        A.finalize(device, fill=fill)
        self.device = device
        self.precise = precise
        self.precise_all = precise_all
        self.lowp_denoiser = bool(lowp_denoiser and precise_all)

    def t(self, name):
        return self.arena[name]

    @property
    def nbytes(self):
        return self.arena.buf.numel()
