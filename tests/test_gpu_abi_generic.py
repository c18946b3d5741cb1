"""The generic tensor-descriptor C-ABI on the GPU (include/stzs.h, csrc/abi.hip): each operator, fed the C++
packers' weights, against the engine path it restates natively (bit-identical: same kernels, same arguments,
bit-identical packed bytes) or against the oracle formula; the composite operators (denoiser_fwd, decoder_pre,
f0n_predictor) both ways: bit-identical to the engine AND within the stage bounds of the fp32 oracle."""
import ctypes as C

import numpy as np
import pytest
import torch

from refops import rel_err
from stzs import _lib as L

pytestmark = pytest.mark.gpu

# oracle parity of the composite operators (rel-L2, teacher-forced inputs), the stage bounds of
# tests/test_gpu_configs.py: a single NFE against the sampler's bound, F0 / N against the predictor's; decoder_pre
# (the generator input, 5 AdaIN blocks at 1024 channels in bf16) at ~2x its measured error
TOL_SAMPLER = 1e-2
TOL_F0, TOL_N = 1e-4, 4.5e-2
TOL_DEC_PRE = 1.5e-2  # (measured r05_a: v0 6.9e-3, tiny 3.6e-3)


def _call(op, ins, outs, p, ws_bytes=None):
    lib = L.load()
    ti = (L.Tensor * len(ins))(*[L.tensor(t) for t in ins])
    to = (L.Tensor * len(outs))(*[L.tensor(t) for t in outs])
    n = getattr(lib, f"stzs_{op}_workspace")(ti, len(ins), C.byref(p))
    ws = torch.zeros(max(n, 256), dtype=torch.uint8, device=ins[0].device)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = getattr(lib, f"stzs_{op}")(ti, len(ins), to, len(outs), C.byref(p), ws.data_ptr(), n if ws_bytes is None else
                                    ws_bytes, s)
    return rc, ws


def _pack(w, Co, Ci, ks, ups, form, dev):
    lib = L.load()
    n = lib.stzs_pack_conv_size(Co, Ci, ks, ups, form)
    assert n > 0
    out = np.zeros(n, np.uint8)
    wc = np.ascontiguousarray(w.float().numpy())
    assert lib.stzs_pack_conv(wc.ctypes.data, Co, Ci, ks, ups, form, out.ctypes.data) == L.OK
    return torch.from_numpy(out).to(dev)


@pytest.fixture(scope="module")
def eng(gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    return StyleTTSZS(tiny, tiny_params, device=gpu_device)


def test_generic_cfg_euler_duration_length(gpu_device):
    from oracle import stzs_ref as R
    g = torch.Generator().manual_seed(61)
    x0 = torch.randn(2, 50, 16, generator=g)
    x = torch.cat([x0, x0])  # the CFG state is duplicated: both halves hold the same x
    D = torch.randn(4, 50, 16, generator=g)
    y = torch.empty_like(x).to(gpu_device)
    rc, _ = _call("cfg_euler_step", [x.to(gpu_device), D.to(gpu_device)], [y], L.params([1], [5.0, 3.0, 0.5]))
    assert rc == L.OK
    Dg = D[2:] + 5.0 * (D[:2] - D[2:])
    xn = x0 + (0.5 - 3.0) * (x0 - Dg) / 3.0
    want = torch.cat([xn, xn])
    assert (y.cpu() - want).abs().max().item() < 1e-5
    logits = torch.randn(3, 40, 50, generator=g) * 2
    dref, sref = R.durations_from_logits(logits)
    dur = torch.empty(3, 40, dtype=torch.int32, device=gpu_device)
    dsum = torch.empty(3, 40, device=gpu_device)
    assert _call("duration_head", [logits.to(gpu_device)], [dur, dsum], L.params())[0] == L.OK
    tie = (sref - sref.floor() - 0.5).abs() < 1e-4
    assert bool(((dur.cpu() == dref) | tie).all())
    d = torch.randint(1, 4, (3, 30), generator=g, dtype=torch.int32)
    d[:, -1] = 100 - d[:, :-1].sum(1)
    d = d.clamp_min(1)
    d[:, -1] += 100 - d.sum(1)
    idx = torch.empty(3, 100, dtype=torch.int32, device=gpu_device)
    assert _call("length_regulate", [d.to(gpu_device)], [idx], L.params())[0] == L.OK
    assert torch.equal(idx.cpu(), R.alignment_index(d))


def test_generic_sine_gen_and_conv_post_istft(eng, tiny, tiny_params):
    S, P, dev = tiny, tiny_params, eng.device
    g = torch.Generator().manual_seed(62)
    F0 = (100 + 150 * torch.rand(2, 40, generator=g)).to(dev)
    Tf = F0.shape[1] * S.hop // S.istft_hop + 1
    har_e = eng.sine_gen(F0, [3, 4]).t[:, :Tf, :S.har_ch].clone()  # (buffer rows: a multiple of the noise stride)
    har = torch.zeros(2, Tf, 32, dtype=torch.bfloat16, device=dev)
    merge = torch.cat([P["gen.src_merge.w"].reshape(-1), P["gen.src_merge.b"]]).float().to(dev)
    seeds = torch.tensor([3, 4], dtype=torch.int32, device=dev)
    p = L.params([S.hop, S.n_fft, S.istft_hop, S.harmonic_num + 1], [S.sr, S.sine_amp, S.noise_std, S.voiced_threshold])
    assert _call("sine_gen", [F0, merge, seeds], [har], p)[0] == L.OK
    assert torch.equal(har[:, :, :S.har_ch], har_e)
    # conv_post + iSTFT on some generator-width rows, vs the engine's conv_post / istft launches
    Ci = S.gen_ch[-1]
    x = (torch.randn(2, 241, Ci, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    from stzs.engine import Act
    want = eng.istft(eng.conv_post(Act(x))).clone()
    w = _pack(P["gen.conv_post.w"], S.har_ch, Ci, 7, 0, L.PACK_KSTEP, dev)
    wav = torch.empty(2, 240 * S.istft_hop, device=dev)
    rc, _ = _call("conv_post_istft", [x, w, P["gen.conv_post.b"].float().to(dev)], [wav],
                  L.params([S.n_fft, S.istft_hop], [0.01]))
    assert rc == L.OK
    assert torch.equal(wav, want)


@pytest.mark.parametrize("B", [1, 2, 3])
def test_generic_bilstm(eng, tiny, tiny_params, B):
    """B 1 / 2 take the tagged-granule exchange, B 3 the counter form.  The LSTM state lives in the caller's scratch:
    the op resets it on entry, so a workspace dirtied by random bytes and by another operator between calls (the
    reuse the per-op _workspace queries invite) gives the same bits."""
    S, P, dev = tiny, tiny_params, eng.device
    lib = L.load()
    g = torch.Generator().manual_seed(63)
    In, H = S.pr_in, S.lstm_h
    x = torch.randn(B, 13, In, generator=g).to(torch.bfloat16).to(dev)
    from stzs.engine import Act
    y_e = eng.act("t.gen.lstm", B, 13, 2 * H)
    eng.lstm(eng.W.pr_de[0], Act(x), y_e, "t.gen")
    eng.check_status()
    ih = np.zeros(lib.stzs_pack_conv_size(8 * H, In, 1, 0, L.PACK_KSTEP), np.uint8)
    bias = np.zeros(8 * H, np.float32)
    fr = np.zeros(2 * 4 * H * H * 2, np.uint8)
    arrs = [np.ascontiguousarray(P["pr.de0." + n].numpy(), dtype=np.float32)
            for n in ("w_ih", "w_hh", "b_ih", "b_hh", "w_ih_rev", "w_hh_rev", "b_ih_rev", "b_hh_rev")]
    assert lib.stzs_pack_lstm(*[a.ctypes.data for a in arrs], In, H, ih.ctypes.data, bias.ctypes.data,
                              fr.ctypes.data) == L.OK
    y = torch.zeros(B, 13, 2 * H, dtype=torch.bfloat16, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ins = [x, torch.from_numpy(ih).to(dev), torch.from_numpy(bias).to(dev), torch.from_numpy(fr).to(dev)]
    rc, ws = _call("bilstm", ins, [y, status], L.params([H]))
    assert rc == L.OK
    assert torch.equal(y, y_e.t[:, :, :2 * H]) and int(status.item()) == 0
    ti = (L.Tensor * 4)(*[L.tensor(t) for t in ins])
    to = (L.Tensor * 2)(L.tensor(y), L.tensor(status))
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for dirt in ("none", "random", "other_op"):
        if dirt == "random":
            ws.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(5))
        elif dirt == "other_op":  # another operator's scratch use of the same bytes (its alignment totals)
            d = torch.randint(1, 4, (B, 600), dtype=torch.int32, device=dev)
            idx = torch.empty(B, 1200, dtype=torch.int32, device=dev)
            ti2, to2 = (L.Tensor * 1)(L.tensor(d)), (L.Tensor * 1)(L.tensor(idx))
            ws.fill_(0x5A)
            assert lib.stzs_length_regulate(ti2, 1, to2, 1, C.byref(L.params()), ws.data_ptr(), ws.numel(), st) == L.OK
        y.zero_()
        rc = lib.stzs_bilstm(ti, 4, to, 2, C.byref(L.params([H])), ws.data_ptr(), ws.numel(), st)
        assert rc == L.OK and torch.equal(y, y_e.t[:, :, :2 * H]), dirt
        assert int(status.item()) == 0, dirt


@pytest.mark.parametrize("stage", [0, 1])
def test_generic_conv_transpose_up(eng, tiny, tiny_params, stage):
    S, P, dev = tiny, tiny_params, eng.device
    g = torch.Generator().manual_seed(64 + stage)
    from stzs.engine import Act
    cin = S.dec_out if stage == 0 else S.gen_ch[0]
    T80 = 20
    T = T80 * (1 if stage == 0 else S.up_rates[0])
    x = torch.randn(2, T, cin, generator=g).to(torch.bfloat16).to(dev)
    F0 = (100 + 150 * torch.rand(2, T80, generator=g)).to(dev)
    har = eng.sine_gen(F0, [1, 2])
    ns = eng.noise_super  # the generic op computes the stride-6 noise conv: compare with that engine form
    eng.noise_super = False
    want = eng.upsample(Act(x), har, stage).t.clone()
    eng.noise_super = ns
    r, k, Co = S.up_rates[stage], S.up_kernels[stage], S.gen_ch[stage]
    last = stage == len(S.up_rates) - 1
    nk = 1 if last else 2 * int(np.prod(S.up_rates[stage + 1:]))
    nstride = 1 if last else nk // 2
    npad = 0 if last else (nstride + 1) // 2
    form = L.PACK_LANE16 if (cin % 128 == 0 and Co % 16 == 0) else L.PACK_KSTEP
    wu = _pack(P[f"gen.ups{stage}.w"], Co, cin, k, r, form, dev)
    wn = _pack(P[f"gen.noise_conv{stage}.w"], Co, S.har_ch, nk, 0, L.PACK_KSTEP, dev)
    y = torch.zeros_like(want)
    ins = [x, har.t, wu, P[f"gen.ups{stage}.b"].float().to(dev), wn, P[f"gen.noise_conv{stage}.b"].float().to(dev)]
    # har descriptor: the engine's buffer (row pitch 32, channels har_ch)
    hv = har.t[:, :T80 * S.hop // S.istft_hop + 1, :S.har_ch]  # the Tf frames (buffer rows are rounded up)
    ins[1] = hv
    rc, _ = _call("conv_transpose_up", ins, [y[:, :, :Co]], L.params([r, int(last), nk, nstride, npad, S.har_ch, Co],
                                                                       [0.1]))
    assert rc == L.OK
    assert torch.equal(y[:, :, :Co], want[:, :, :Co])


@pytest.mark.parametrize("spec", ["tiny", "v0"])
def test_generic_mrf_resblock(gpu_device, tiny, tiny_params, spec):
    """the MRF of generator stage 1 through the generic entry (C++ orchestration of 18 convs + statistics) vs the
    engine's mrf(): bit-identical (tiny: KSTEP weights; v0: FRAG32 weights, 128 channels)."""
    from stzs.engine import Act, StyleTTSZS
    if spec == "tiny":
        S, P = tiny, tiny_params
    else:
        from stzs.params import init_params
        from stzs.spec import SPEC_V0
        S, P = SPEC_V0, init_params(SPEC_V0, seed=0)
    eng = StyleTTSZS(S, P, device=gpu_device)
    dev = eng.device
    stage, C_ = 1, S.gen_ch[1]
    g = torch.Generator().manual_seed(66)
    B, T = 2, 3001
    x = torch.randn(B, T, C_, generator=g).to(torch.bfloat16).to(dev)
    codes = (torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3).to(dev)
    gbd = eng.dec_style(codes)
    want = eng.mrf(Act(x), stage, gbd, eng.W.dec_norm).t.clone()
    ng = eng.W.dec_norm
    form = L.PACK_FRAG32 if (C_ == 128) else (L.PACK_LANE16 if C_ % 128 == 0 else L.PACK_KSTEP)
    gb_cols, ins = [], []
    nk, nd = len(S.rb_kernels), len(S.rb_dils)
    for j, kr in enumerate(S.rb_kernels):
        for m in range(nd):
            pfx = f"gen.rb{stage}.{j}.{m}"
            for nn in (".n1", ".n2"):
                off, c = ng.offsets[pfx + nn]
                gb_cols.append(gbd[:, off:off + 2 * c])
            for cc, al in ((".c1", ".alpha1"), (".c2", ".alpha2")):
                ins += [_pack(P[pfx + cc + ".w"], C_, C_, kr, 0, form, dev), P[pfx + cc + ".b"].float().to(dev),
                        P[pfx + al].float().to(dev)]
    gb = torch.cat(gb_cols, 1).contiguous()
    y = torch.zeros(B, T, C_, dtype=torch.bfloat16, device=dev)
    p = L.params([C_] + list(S.rb_kernels) + list(S.rb_dils) + [nk, nd, form])
    rc, _ = _call("mrf_resblock", [x, gb] + ins, [y], p)
    assert rc == L.OK
    assert torch.equal(y, want[:, :, :C_])


def test_generic_mrf_resblock_rejects_in_place(gpu_device, tiny, tiny_params):
    """y overlapping x is rejected before any launch (resblocks after the first still read x)."""
    S = tiny
    C_ = S.gen_ch[1]
    x = torch.zeros(1, 64, C_, dtype=torch.bfloat16, device=gpu_device)
    nk, nd = len(S.rb_kernels), len(S.rb_dils)
    gb = torch.zeros(1, nk * nd * 4 * C_, device=gpu_device)
    dummy = torch.zeros(16, device=gpu_device)
    p = L.params([C_] + list(S.rb_kernels) + list(S.rb_dils) + [nk, nd, L.PACK_KSTEP])
    ins = [x, gb] + [dummy] * (6 * nk * nd)
    assert _call("mrf_resblock", ins, [x], p)[0] == L.EINVAL
    assert _call("mrf_resblock", ins, [x[:, 10:]], p)[0] in (L.EINVAL, L.ESHAPE)


def test_generic_rejects_short_workspace(eng):
    x = torch.zeros(2, 30, dtype=torch.int32, device=eng.device)
    idx = torch.zeros(2, 60, dtype=torch.int32, device=eng.device)
    assert _call("length_regulate", [x], [idx], L.params(), ws_bytes=4)[0] == L.ESHAPE


# ---------------------------------------------------------------------------------------------------------------
# composite operators (csrc/abi_ops.hip): a2 denoiser_fwd, a9 decoder_pre, a8 f0n_predictor.  Weights either from the
# C++ packers applied to the torch parameters (tiny spec: the path a non-Python host takes) or from the engine's
# packed arena (v0; the packers are bit-identical to it, tests/test_abi_generic.py).  Both must reproduce the engine
# path BIT FOR BIT (same kernels, same arguments, same order).

def _none_tensor():
    return L.Tensor()  # data NULL: an absent optional tensor (sc / pool of a block)


class _Weights:
    """packed weights by engine-arena view (src="arena") or by the C++ packers from the parameters (src="packer")."""

    def __init__(self, eng, P, src):
        self.eng, self.P, self.src, self.dev = eng, P, src, eng.device
        self.keep = []

    def _t(self, t):
        if t.dim() > 4:  # packed fragment streams are raw bytes to the ABI: a flat view
            t = t.reshape(-1)
        self.keep.append(t)
        return L.tensor(t)

    def conv(self, cw, pname, ks=None, form=L.PACK_KSTEP, w=None, b=None):
        """[w, b] descriptors of a packed conv: cw = the engine's ConvW, pname = its parameter prefix."""
        if self.src == "arena":
            W = self.eng.W
            return [self._t(W.t(cw.w)), self._t(W.t(cw.b)) if cw.b is not None else _none_tensor()]
        w = self.P[pname + ".w"] if w is None else w
        if w.dim() == 2:
            w = w[:, :, None]
        bias = (self.P.get(pname + ".b") if b is None else b)
        pk = _pack(w, w.shape[0], w.shape[1], w.shape[2], 0, form, self.dev)
        return [self._t(pk), self._t(bias.float().to(self.dev)) if bias is not None else _none_tensor()]

    def raw(self, name_or_t):
        W = self.eng.W
        return self._t(W.t(name_or_t) if isinstance(name_or_t, str) else name_or_t)

    def blk(self, bw):
        """the 7 tensors of an AdaIN block (include/stzs.h STZS_DP_BLK0 layout)."""
        n = bw.name
        form = lambda cw: L.PACK_FRAG32 if cw.frag32 else (L.PACK_LANE16 if cw.lane16 else L.PACK_KSTEP)
        f1, f2 = form(bw.conv1), form(bw.conv2)
        out = self.conv(bw.conv1, n + ".conv1", form=f1) + self.conv(bw.conv2, n + ".conv2", form=f2)
        out.append(self.conv(bw.sc, n + ".sc", form=form(bw.sc))[0] if bw.sc is not None else _none_tensor())
        out += [self.raw(bw.pool_w), self.raw(bw.pool_b)] if bw.up else [_none_tensor(), _none_tensor()]
        return out

    def norm_group(self, ng, names):
        if self.src == "arena":
            return self.conv(ng.lin, None)
        w = torch.cat([self.P[n + ".w"] for n in names], 0)
        b = torch.cat([self.P[n + ".b"] for n in names], 0)
        return self.conv(None, None, w=w, b=b)

    def lstm(self, lw, name):
        if self.src == "arena":
            W = self.eng.W
            return [self._t(W.t(lw.ih.w)), self._t(W.t(lw.ih.b)), self._t(W.t(lw.whhT))]
        lib = L.load()
        P = self.P
        In, H = P[name + ".w_ih"].shape[1], P[name + ".w_hh"].shape[1]
        ih = np.zeros(lib.stzs_pack_conv_size(8 * H, In, 1, 0, L.PACK_KSTEP), np.uint8)
        bias = np.zeros(8 * H, np.float32)
        fr = np.zeros(2 * 4 * H * H * 2, np.uint8)
        arrs = [np.ascontiguousarray(P[name + "." + k].numpy(), dtype=np.float32)
                for k in ("w_ih", "w_hh", "b_ih", "b_hh", "w_ih_rev", "w_hh_rev", "b_ih_rev", "b_hh_rev")]
        assert lib.stzs_pack_lstm(*[a.ctypes.data for a in arrs], In, H, ih.ctypes.data, bias.ctypes.data,
                                  fr.ctypes.data) == L.OK
        return [self._t(torch.from_numpy(x).to(self.dev)) for x in (ih, bias, fr)]


def _run_generic(op, ins, outs, p):
    lib = L.load()
    ti = (L.Tensor * len(ins))(*ins)
    to = (L.Tensor * len(outs))(*[L.tensor(t) for t in outs])
    n = getattr(lib, f"stzs_{op}_workspace")(ti, len(ins), C.byref(p))
    assert n > 0, op
    ws = torch.empty(n, dtype=torch.uint8, device=outs[0].device)
    ws.random_(0, 256)  # scratch with no required contents
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = getattr(lib, f"stzs_{op}")(ti, len(ins), to, len(outs), C.byref(p), ws.data_ptr(), n, s)
    short = getattr(lib, f"stzs_{op}")(ti, len(ins), to, len(outs), C.byref(p), ws.data_ptr(), n - 256, s)
    torch.cuda.synchronize()
    return rc, short


def _engine(spec, gpu_device, tiny, tiny_params):
    from stzs.engine import StyleTTSZS
    if spec == "tiny":
        return tiny, tiny_params, StyleTTSZS(tiny, tiny_params, device=gpu_device)
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    P = init_params(SPEC_V0, seed=0)
    return SPEC_V0, P, StyleTTSZS(SPEC_V0, P, device=gpu_device)


CASES_SRC = [("tiny", "packer"), ("v0", "arena")]


@pytest.mark.parametrize("spec,src", CASES_SRC)
@pytest.mark.parametrize("cfg,sigma", [(True, 3.0), (True, 0.5), (False, 0.5)])
def test_generic_denoiser_fwd(gpu_device, tiny, tiny_params, spec, src, cfg, sigma):
    """one full NFE through the C-ABI (context, K/V, sigma conditioning, 6 layers, EDM output) == engine.denoiser_fwd"""
    from stzs.engine import Act
    S, P, eng = _engine(spec, gpu_device, tiny, tiny_params)
    dev = eng.device
    g = torch.Generator().manual_seed(71)
    B, T = 2, 23
    h = (torch.randn(B, T, S.d_txt, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    prompt = (torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3).to(dev)
    R = 2 * B if cfg else B
    x0 = torch.randn(B, S.L_s, S.code_dim, generator=g) * sigma
    x = (torch.cat([x0, x0]) if cfg else x0).to(dev)
    want = eng.denoiser_fwd(Act(h), prompt, x, sigma, cfg).clone()
    W, Wt = eng.W, _Weights(eng, P, src)
    ins = [Wt._t(x), Wt._t(h), Wt._t(prompt)]
    ins += Wt.conv(W.dn_in, "dn.in_proj") + [Wt.raw(W.dn_pos)] + Wt.conv(W.dn_t0, "dn.t_mlp0") + \
        Wt.conv(W.dn_t1, "dn.t_mlp1") + Wt.conv(W.dn_pool, "dn.pool_proj") + Wt.conv(W.dn_ctx_txt, "dn.ctx_txt") + \
        Wt.conv(W.dn_ctx_prm, "dn.ctx_prm") + Wt.conv(W.dn_ada, "dn.ada") + [Wt.raw(W.dn_table)] + \
        Wt.conv(W.dn_final_ada, "dn.final_ada") + Wt.conv(W.dn_out, "dn.out") + [Wt.raw(W.dn_ctx_null),
                                                                                  Wt.raw(W.dn_pool_null)]
    assert len(ins) == L.DN_NIN_BASE
    for l, lw in enumerate(W.dn_layers):
        pf = f"dn.l{l}"
        for k, n in (("qkv", ".sa_qkv"), ("o", ".sa_o"), ("q", ".ca_q"), ("kv", ".ca_kv"), ("co", ".ca_o"),
                     ("ff1", ".ff1"), ("ff2", ".ff2")):
            ins += Wt.conv(lw[k], pf + n)
        ins += [Wt.raw(lw["ln_g"]), Wt.raw(lw["ln_b"])]
    D = torch.full((R, S.L_s, S.code_dim), float("nan"), device=dev)
    p = L.params([int(cfg), S.dn_layers, S.dn_heads, S.dn_d, S.dn_ffn, S.dn_fourier], [sigma, S.sigma_data])
    rc, short = _run_generic("denoiser_fwd", ins, [D], p)
    assert rc == L.OK and short == L.ESHAPE
    assert torch.equal(D, want), (D - want).abs().max().item()
    # ... and against the fp32 oracle directly (same bf16-rounded text rows): one NFE at the sampler's stage bound
    from oracle import stzs_ref as R
    kv, pool = R.denoiser_context(P, S, h.float().cpu(), prompt.cpu(), cfg)
    ref = R.denoiser(P, S, x.cpu(), sigma, kv, pool)
    e = rel_err(D.cpu(), ref)
    print(f"stzs_denoiser_fwd {spec} cfg={cfg} sigma={sigma}: rel-L2 vs oracle {e:.2e}")
    assert e < TOL_SAMPLER


@pytest.mark.parametrize("spec,src", CASES_SRC)
def test_generic_decoder_pre(gpu_device, tiny, tiny_params, spec, src):
    S, P, eng = _engine(spec, gpu_device, tiny, tiny_params)
    dev = eng.device
    g = torch.Generator().manual_seed(72)
    B, T40 = 2, 37
    asr = torch.randn(B, T40, S.d_txt, generator=g).to(torch.bfloat16).to(dev)
    F0 = (100 + 150 * torch.rand(B, 2 * T40, generator=g)).to(dev)
    Nn = torch.randn(B, 2 * T40, generator=g).to(dev)
    codes = (torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3).to(dev)
    enc_in = eng.act("dec.enc_in", B, T40, S.d_txt + 2)
    enc_in.t[:, :, :S.d_txt] = asr
    gen_in, _ = eng.decoder_pre(dict(asr_buf=enc_in, F0=F0, N=Nn, T40=T40), codes)
    want = gen_in.t[:, :, :S.dec_out].clone()
    W, Wt = eng.W, _Weights(eng, P, src)
    names = []
    for nm in ("dec.encode", "dec.decode0", "dec.decode1", "dec.decode2", "dec.decode3"):
        names += [nm + ".norm1", nm + ".norm2"]
    ins = [Wt._t(asr), Wt._t(F0), Wt._t(Nn), Wt._t(codes), Wt.raw(W.dec_f0), Wt.raw(W.dec_n)] + \
        Wt.conv(W.dec_asr_res, "dec.asr_res") + Wt.norm_group(W.dec_norm, names)
    for nm in ("dec.encode", "dec.decode0", "dec.decode1", "dec.decode2", "dec.decode3"):
        ins += Wt.blk(W.dec_blk[nm])
    assert len(ins) == L.DP_NIN
    total = W.dec_norm.total if src == "arena" else sum(P[n + ".w"].shape[0] for n in names)
    out = torch.full((B, 2 * T40, S.dec_out), float("nan"), dtype=torch.bfloat16, device=dev)
    p = L.params([S.dec_enc, S.dec_asr_res, S.dec_out, S.style_ac, total])
    rc, short = _run_generic("decoder_pre", ins, [out], p)
    assert rc == L.OK and short == L.ESHAPE
    assert torch.equal(out, want)
    from oracle import stzs_ref as R
    ref = R.decoder_pre(P, S, asr.float().cpu(), F0.cpu(), Nn.cpu(), codes.cpu()).transpose(1, 2)
    e = rel_err(out.float().cpu(), ref)
    print(f"stzs_decoder_pre {spec}: rel-L2 vs oracle {e:.2e}")
    assert e < TOL_DEC_PRE


@pytest.mark.parametrize("spec,src", CASES_SRC)
@pytest.mark.parametrize("B", [1, 3])
def test_generic_f0n_predictor(gpu_device, tiny, tiny_params, spec, src, B):
    from stzs.engine import Act
    S, P, eng = _engine(spec, gpu_device, tiny, tiny_params)
    dev = eng.device
    g = torch.Generator().manual_seed(73)
    T40 = 41
    en = torch.randn(B, T40, S.pr_in, generator=g).to(torch.bfloat16).to(dev)
    codes = (torch.randn(B, S.L_s, S.code_dim, generator=g) * 0.3).to(dev)
    F0w, Nw = eng.f0n_predictor(Act(en), codes)
    F0w, Nw = F0w.contiguous().clone(), Nw.contiguous().clone()
    eng.check_status()
    W, Wt = eng.W, _Weights(eng, P, src)
    names = []
    for br in ("f0", "n"):
        for i in range(3):
            names += [f"pr.{br}{i}.norm1", f"pr.{br}{i}.norm2"]
    ins = [Wt._t(en), Wt._t(codes)] + Wt.lstm(W.pr_shared, "pr.shared") + Wt.norm_group(W.pr_norm, names)
    for br in ("f0", "n"):
        for i in range(3):
            ins += Wt.blk(W.pr_blk[f"pr.{br}{i}"])
        ins += Wt.conv(W.pr_blk[f"pr.{br}_proj"], f"pr.{br}_proj")
    assert len(ins) == L.FN_NIN
    total = W.pr_norm.total if src == "arena" else sum(P[n + ".w"].shape[0] for n in names)
    F0 = torch.full((B, 2 * T40), float("nan"), device=dev)
    Nn = torch.full((B, 2 * T40), float("nan"), device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    c0, c1, c2 = S.f0n_ch
    p = L.params([S.lstm_h, c0, c1, c2, S.style_ac, S.style_pr, total])
    rc, short = _run_generic("f0n_predictor", ins, [F0, Nn, status], p)
    assert rc == L.OK and short == L.ESHAPE and int(status.item()) == 0
    assert torch.equal(F0, F0w) and torch.equal(Nn, Nw)
    from oracle import stzs_ref as R
    rF, rN = R.f0n_predictor(P, S, en.float().cpu(), codes.cpu())
    eF, eN = rel_err(F0.cpu(), rF), rel_err(Nn.cpu(), rN)
    print(f"stzs_f0n_predictor {spec} B={B}: F0 rel-L2 vs oracle {eF:.2e}, N {eN:.2e}")
    assert eF < TOL_F0 and eN < TOL_N
