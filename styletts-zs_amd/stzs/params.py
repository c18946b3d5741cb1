"""Deterministic seeded random-init parameters for HOTPATH spec v0.

No StyleTTS-ZS checkpoint exists (`/root/reference/README.md:15-16`), so every configuration
runs on seeded random weights (`BASELINE.json` configs[0]: "random-init weights").  Parameters
are produced in declaration order from ONE `torch.Generator` so the same (spec, seed) yields
bit-identical tensors on every host; `param_checksum` fingerprints them for the fixtures.

Shapes are the torch-native layouts (Conv1d [Co,Ci,k], ConvTranspose1d [Ci,Co,k],
Linear [out,in], LSTM w_ih [4H,in] / w_hh [4H,H] in gate order i,f,g,o) so the CPU oracle can
use torch.nn.functional directly; `stzs.weights` repacks them for the HIP kernels.
"""
from __future__ import annotations

import hashlib
import math
from collections import OrderedDict

import torch

from .spec import Spec


class _Init:
    def __init__(self, seed: int):
        self.g = torch.Generator().manual_seed(int(seed))
        self.p: "OrderedDict[str, torch.Tensor]" = OrderedDict()

    def uni(self, name, shape, bound):
        t = (torch.rand(shape, generator=self.g, dtype=torch.float64) * 2 - 1) * bound
        self.p[name] = t.float()

    def nrm(self, name, shape, std, mean=0.0):
        t = torch.randn(shape, generator=self.g, dtype=torch.float64) * std + mean
        self.p[name] = t.float()

    def const(self, name, shape, v):
        self.p[name] = torch.full(shape, float(v))

    # torch-default-like fan-in uniform for weights and biases
    def linear(self, name, n_out, n_in, bias=True, gain=1.0):
        b = gain / math.sqrt(n_in)
        self.uni(name + ".w", (n_out, n_in), b)
        if bias:
            self.uni(name + ".b", (n_out,), b)

    def conv(self, name, co, ci, k, bias=True, gain=1.0):
        b = gain / math.sqrt(ci * k)
        self.uni(name + ".w", (co, ci, k), b)
        if bias:
            self.uni(name + ".b", (co,), b)

    def convT(self, name, ci, co, k):
        b = 1.0 / math.sqrt(co * k)
        self.uni(name + ".w", (ci, co, k), b)
        self.uni(name + ".b", (co,), b)

    def lstm(self, name, n_in, h):
        b = 1.0 / math.sqrt(h)
        for sfx in ("", "_rev"):
            self.uni(f"{name}.w_ih{sfx}", (4 * h, n_in), b)
            self.uni(f"{name}.w_hh{sfx}", (4 * h, h), b)
            self.uni(f"{name}.b_ih{sfx}", (4 * h,), b)
            self.uni(f"{name}.b_hh{sfx}", (4 * h,), b)

    def adain_res_blk(self, name, din, dout, style, upsample=False):
        """StyleTTS2 AdainResBlk1d: norm1(fc)->lrelu->[dw ConvT x2]->conv1->norm2->lrelu->conv2,
        shortcut = [nearest x2] -> [conv1x1 if din != dout], out = (res + sc)/sqrt(2)."""
        self.linear(name + ".norm1", 2 * din, style, gain=0.5)
        if upsample:
            self.uni(name + ".pool.w", (din, 1, 3), 1.0 / math.sqrt(3))
            self.uni(name + ".pool.b", (din,), 1.0 / math.sqrt(3))
        self.conv(name + ".conv1", dout, din, 3)
        self.linear(name + ".norm2", 2 * dout, style, gain=0.5)
        self.conv(name + ".conv2", dout, dout, 3)
        if din != dout:
            self.conv(name + ".sc", dout, din, 1, bias=False)


class _Shapes(_Init):
    """declares every parameter as a meta tensor (shape only, no values, no generator draws)"""

    def uni(self, name, shape, bound):
        self.p[name] = torch.empty(shape, device="meta")

    def nrm(self, name, shape, std, mean=0.0):
        self.p[name] = torch.empty(shape, device="meta")

    def const(self, name, shape, v):
        self.p[name] = torch.empty(shape, device="meta")


def init_params(spec: Spec, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    return _declare(_Init(seed), spec)


def param_shapes(spec: Spec) -> "OrderedDict[str, torch.Size]":
    """name -> shape of every parameter of `spec`, in declaration order (checkpoint validation)."""
    return OrderedDict((k, v.shape) for k, v in _declare(_Shapes(0), spec).items())


def _declare(I: _Init, spec: Spec) -> "OrderedDict[str, torch.Tensor]":
    S = spec
    sty = S.style_ac
    # ---- text encoder (front end; StyleTTS2 TextEncoder CNN part; its BiLSTM is declared last) ----
    I.nrm("te.emb", (S.n_symbols, S.d_txt), 1.0)
    for i in range(S.te_layers):
        I.conv(f"te.conv{i}", S.d_txt, S.d_txt, S.te_kernel)
        I.nrm(f"te.ln{i}.g", (S.d_txt,), 0.1, 1.0)
        I.nrm(f"te.ln{i}.b", (S.d_txt,), 0.1)
    # ---- prompt encoder (front end) ----
    I.conv("pe.conv0", S.pe_ch, S.n_mels, 5)
    I.conv("pe.conv1", S.pe_ch, S.pe_ch, 5)
    I.linear("pe.proj", S.code_dim, S.pe_ch, gain=0.5)
    # ---- style denoiser ----
    d = S.dn_d
    I.linear("dn.in_proj", d, S.code_dim)
    I.nrm("dn.pos", (S.L_s, d), 0.1)
    I.linear("dn.t_mlp0", d, S.dn_fourier)
    I.linear("dn.t_mlp1", d, d)
    I.linear("dn.pool_proj", d, S.code_dim)
    I.nrm("dn.null_codes", (S.L_s, S.code_dim), 0.2)
    I.linear("dn.ctx_txt", d, S.d_txt)
    I.linear("dn.ctx_prm", d, S.code_dim)
    I.linear("dn.ada", 6 * d, d, gain=0.5)
    I.nrm("dn.ada_table", (S.dn_layers, 6 * d), 0.05)
    for l in range(S.dn_layers):
        p = f"dn.l{l}"
        I.linear(p + ".sa_qkv", 3 * d, d)
        I.linear(p + ".sa_o", d, d)
        I.nrm(p + ".ca_ln.g", (d,), 0.1, 1.0)
        I.nrm(p + ".ca_ln.b", (d,), 0.1)
        I.linear(p + ".ca_q", d, d)
        I.linear(p + ".ca_kv", 2 * d, d)
        I.linear(p + ".ca_o", d, d)
        I.linear(p + ".ff1", S.dn_ffn, d)
        I.linear(p + ".ff2", d, S.dn_ffn)
    I.linear("dn.final_ada", 2 * d, d, gain=0.5)
    I.linear("dn.out", S.code_dim, d)
    # ---- prosody predictor ----
    H = S.lstm_h
    for i in range(S.pr_layers):
        I.lstm(f"pr.de{i}", S.pr_in, H)
        I.linear(f"pr.de{i}.aln", 2 * S.pr_hid, S.style_pr, gain=0.5)
    I.lstm("pr.dur_lstm", S.pr_in, H)
    I.linear("pr.dur_proj", S.dur_bins, S.pr_hid)
    I.lstm("pr.shared", S.pr_in, H)
    c0, c1, c2 = S.f0n_ch
    for br in ("f0", "n"):
        I.adain_res_blk(f"pr.{br}0", S.pr_hid, c0, S.style_pr)
        I.adain_res_blk(f"pr.{br}1", c0, c1, S.style_pr, upsample=True)
        I.adain_res_blk(f"pr.{br}2", c1, c2, S.style_pr)
        I.conv(f"pr.{br}_proj", 1, c2, 1)
    I.p["pr.f0_proj.b"] = I.p["pr.f0_proj.b"] + S.f0_bias
    # ---- decoder (iSTFTNet shape) ----
    I.conv("dec.f0_conv", 1, 1, 3)
    I.conv("dec.n_conv", 1, 1, 3)
    I.conv("dec.asr_res", S.dec_asr_res, S.d_txt, 1)
    I.adain_res_blk("dec.encode", S.d_txt + 2, S.dec_enc, sty)
    dcat = S.dec_enc + 2 + S.dec_asr_res
    for i in range(3):
        I.adain_res_blk(f"dec.decode{i}", dcat, S.dec_enc, sty)
    I.adain_res_blk("dec.decode3", dcat, S.dec_out, sty, upsample=True)
    I.linear("gen.src_merge", 1, S.harmonic_num + 1)
    cin = S.dec_out
    n_up = len(S.up_rates)
    for i, (r, k) in enumerate(zip(S.up_rates, S.up_kernels)):
        c = S.gen_ch[i]
        if i + 1 < n_up:
            sf0 = 1
            for rr in S.up_rates[i + 1:]:
                sf0 *= rr
            I.conv(f"gen.noise_conv{i}", c, S.har_ch, 2 * sf0)
        else:
            I.conv(f"gen.noise_conv{i}", c, S.har_ch, 1)
        I.convT(f"gen.ups{i}", cin, c, k)
        for j, kr in enumerate(S.rb_kernels):
            for m, _dil in enumerate(S.rb_dils):
                p = f"gen.rb{i}.{j}.{m}"
                I.linear(p + ".n1", 2 * c, sty, gain=0.5)
                I.nrm(p + ".alpha1", (c,), 0.1, 1.0)
                I.conv(p + ".c1", c, c, kr)
                I.linear(p + ".n2", 2 * c, sty, gain=0.5)
                I.nrm(p + ".alpha2", (c,), 0.1, 1.0)
                I.conv(p + ".c2", c, c, kr)
        cin = c
    I.conv("gen.conv_post", S.har_ch, S.gen_ch[-1], 7)
    # ---- round-2 additions, declared last so every earlier parameter keeps its seeded value ----
    # text encoder BiLSTM after the CNN stack (StyleTTS2 TextEncoder: CNN + BiLSTM)
    I.lstm("te.lstm", S.d_txt, S.d_txt // 2)
    # discrete style-code codebooks [groups][entries][group width] (README.md:5)
    I.nrm("pe.vq", (S.code_dim // S.vq_group, S.vq_size, S.vq_group), S.vq_std)
    return I.p


def param_count(params) -> int:
    return sum(int(v.numel()) for v in params.values())


def param_checksum(params) -> str:
    h = hashlib.sha256()
    for k, v in params.items():
        h.update(k.encode())
        h.update(v.detach().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]
