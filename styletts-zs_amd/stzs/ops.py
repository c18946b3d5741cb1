"""torch operators over the HIP hot path (SURVEY.md §8(b) "torch ops (L1)"): `torch.ops.stzs.<op>`.

The upstream inference API is "Under construction" (`/root/reference/README.md:15-16`), so these
operators pin the L1 surface SURVEY §8(b) lists, one per hot-path row of §8(a):

  stzs::synth            a1-a13  tokens + reference wav -> waveform (whole pipeline)
  stzs::sample_style     a1-a4   style diffusion (denoiser + CFG + Euler), -> codes [B, L_s, 256]
  stzs::predict_prosody  a5-a8   durations, alignment, F0 / N curves
  stzs::decode           a9-a13  decoder pre-blocks + generator + iSTFT, -> waveform
  stzs::duration_head    a6      round(sum sigmoid(logits)), clamp >= 1 (bit-exact integer path)
  stzs::length_regulate  a7      exclusive-scan alignment index per aligned frame
  stzs::cfg_euler_step   a3      fused CFG combine + Euler update
  stzs::istft            a13     conv_post rows [B, Tf, n_fft + 2] -> waveform
  stzs::istft_stream     a14     one chunk of the streaming iSTFT with its carried frame tail
  stzs::bilstm           a5, a8  one named BiLSTM of the model (text encoder, DurationEncoder, duration, shared)
  stzs::denoiser_fwd     a2      one preconditioned denoiser evaluation D(x, sigma) (CFG rows)
  stzs::f0n_predictor    a8      shared BiLSTM + F0 / N AdaIN-block branches
  stzs::decoder_pre      a9      F0/N convs, asr_res, encode + 4 decode AdaIN blocks -> generator input
  stzs::sine_gen         a10     harmonic source + its STFT features
  stzs::conv_transpose_up a11    noise conv + LeakyReLU + polyphase ConvTranspose1d (+ ReflectionPad)
  stzs::mrf_resblock     a12     the MRF of one generator stage (AdaIN + Snake + dilated convs)
  stzs::conv_post_istft  a13     conv_post + exp/sin spectrum + iSTFT
  stzs::code_quantize    (f)1    the discrete style-code quantiser (README.md:5)

Model-bound operators take an integer engine handle from `register(engine)` (the packed weights live in
the engine's device arena).  Every operator is registered for the HIP device ONLY
(`device_types="cuda"`, which is HIP on ROCm): there is deliberately no CPU implementation, so a CPU
tensor raises instead of silently running a fallback.  Fake (meta) implementations give output shapes
for tracing; outputs are fresh tensors (never the engine's cached buffers).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Tuple

import torch
from torch.library import custom_op, register_fake

from . import _lib as L

_ENGINES = {}


def register(engine) -> int:
    """engine handle for the model-bound operators."""
    h = len(_ENGINES) + 1
    _ENGINES[h] = engine
    return h


def _eng(handle: int, *tensors):
    eng = _ENGINES.get(int(handle))
    if eng is None:
        raise RuntimeError(f"stzs: unknown engine handle {handle} (stzs.ops.register(engine) first)")
    for t in tensors:
        if t is not None and t.device != eng.device:
            raise RuntimeError(f"stzs: operand on {t.device}, engine on {eng.device} (HIP-only operators)")
    return eng


def _stream(t: torch.Tensor):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


# ------------------------------------------------------------------ model-bound (engine handle)
@custom_op("stzs::synth", mutates_args=(), device_types="cuda")
def synth(handle: int, tokens: torch.Tensor, ref_wav: torch.Tensor, noise: torch.Tensor,
          durations: torch.Tensor, steps: int, cfg_scale: float, seeds: List[int]) -> torch.Tensor:
    eng = _eng(handle, tokens, ref_wav, noise)
    out = eng.synth(tokens, ref_wav, steps=steps, cfg_scale=cfg_scale, noise=noise, durations=durations.cpu(),
                    seeds=list(seeds))  # raises on an LSTM exchange timeout (synth's status check)
    return out["wav"].clone()


@register_fake("stzs::synth")
def _(handle, tokens, ref_wav, noise, durations, steps, cfg_scale, seeds):
    n = torch.library.get_ctx().new_dynamic_size()
    return tokens.new_empty((tokens.shape[0], n), dtype=torch.float32)


@custom_op("stzs::sample_style", mutates_args=(), device_types="cuda")
def sample_style(handle: int, h_txt: torch.Tensor, prompt: torch.Tensor, noise: torch.Tensor, steps: int,
                 cfg_scale: float) -> torch.Tensor:
    """h_txt [B, T_txt, d_txt] (bf16 or fp32), prompt [B, L_s, 256] fp32, noise [B, L_s, 256] -> codes fp32."""
    from .engine import Act
    eng = _eng(handle, h_txt, prompt, noise)
    B, T, D = h_txt.shape
    ht = eng.buf("op.h_txt", (B, T, (D + 7) // 8 * 8), eng.adt, zero=True)
    ht[:, :, :D].copy_(h_txt)
    return eng.sample_style(Act(ht, 0, D), prompt.float().contiguous(), noise.float().contiguous(), steps,
                            cfg_scale).clone()


@register_fake("stzs::sample_style")
def _(handle, h_txt, prompt, noise, steps, cfg_scale):
    return noise.new_empty(noise.shape, dtype=torch.float32)


@custom_op("stzs::predict_prosody", mutates_args=(), device_types="cuda")
def predict_prosody(handle: int, h_txt: torch.Tensor, codes: torch.Tensor,
                    durations: Optional[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """-> (dur int32 [B, T_txt], idx int32 [B, T40], F0 fp32 [B, T80], N fp32 [B, T80]); durations forces dur."""
    from .engine import Act
    eng = _eng(handle, h_txt, codes)
    B, T, D = h_txt.shape
    ht = eng.buf("op.h_txt", (B, T, (D + 7) // 8 * 8), eng.adt, zero=True)
    ht[:, :, :D].copy_(h_txt)
    pro = eng.predict_prosody(Act(ht, 0, D), codes.float().contiguous(),
                              durations.cpu() if durations is not None else None)
    eng.check_status()  # an LSTM exchange timeout makes every output of this call invalid: raise
    return pro["dur"].clone(), pro["idx"].clone(), pro["F0"].contiguous().clone(), pro["N"].contiguous().clone()


@register_fake("stzs::predict_prosody")
def _(handle, h_txt, codes, durations):
    B, T = h_txt.shape[0], h_txt.shape[1]
    t40 = torch.library.get_ctx().new_dynamic_size()
    i32 = dict(dtype=torch.int32)
    return (h_txt.new_empty((B, T), **i32), h_txt.new_empty((B, t40), **i32),
            h_txt.new_empty((B, 2 * t40), dtype=torch.float32), h_txt.new_empty((B, 2 * t40), dtype=torch.float32))


@custom_op("stzs::decode", mutates_args=(), device_types="cuda")
def decode(handle: int, asr: torch.Tensor, F0: torch.Tensor, N: torch.Tensor, codes: torch.Tensor,
           seeds: List[int]) -> torch.Tensor:
    """asr [B, T40, d_txt] (aligned text features), F0 / N [B, 2 T40], codes [B, L_s, 256] -> wav [B, 600 T40]."""
    eng = _eng(handle, asr, F0, N, codes)
    S = eng.spec
    B, T40, D = asr.shape
    enc_in = eng.act("dec.enc_in", B, T40, S.d_txt + 2)
    enc_in.t[:, :, :D].copy_(asr)
    pro = dict(asr_buf=enc_in, F0=F0.float().contiguous(), N=N.float().contiguous(), T40=T40)
    return eng.decode(pro, codes.float().contiguous(), list(seeds)).clone()


@register_fake("stzs::decode")
def _(handle, asr, F0, N, codes, seeds):
    return asr.new_empty((asr.shape[0], 600 * asr.shape[1]), dtype=torch.float32)


# ------------------------------------------------------------------ stateless kernels
@custom_op("stzs::duration_head", mutates_args=(), device_types="cuda")
def duration_head(logits: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """logits fp32 [B, T, nbins] -> (dur int32 [B, T] = max(1, round(sum_j sigmoid)), dsum fp32 [B, T])."""
    lg = logits.float().contiguous()
    B, T, nb = lg.shape
    dur = torch.empty(B, T, dtype=torch.int32, device=lg.device)
    dsum = torch.empty(B, T, dtype=torch.float32, device=lg.device)
    a = L.DurArgs()
    a.logits, a.override_dur, a.dur, a.dsum = lg.data_ptr(), None, dur.data_ptr(), dsum.data_ptr()
    a.ldl, a.bsl, a.B, a.T, a.nbins = nb, T * nb, B, T, nb
    L.check(L.load().stzs_durations(C.byref(a), _stream(lg)), "stzs::duration_head")
    return dur, dsum


@register_fake("stzs::duration_head")
def _(logits):
    B, T = logits.shape[0], logits.shape[1]
    return logits.new_empty((B, T), dtype=torch.int32), logits.new_empty((B, T), dtype=torch.float32)


@custom_op("stzs::length_regulate", mutates_args=(), device_types="cuda")
def length_regulate(dur: torch.Tensor, n_frames: int) -> torch.Tensor:
    """dur int32 [B, T] -> token index per aligned frame int32 [B, n_frames] (-1 past sum(dur))."""
    d = dur.to(torch.int32).contiguous()
    B, T = d.shape
    idx = torch.empty(B, n_frames, dtype=torch.int32, device=d.device)
    total = torch.empty(B, dtype=torch.int32, device=d.device)
    a = L.AlignArgs()
    a.dur, a.idx, a.total, a.B, a.T, a.T40 = d.data_ptr(), idx.data_ptr(), total.data_ptr(), B, T, n_frames
    L.check(L.load().stzs_alignment(C.byref(a), _stream(d)), "stzs::length_regulate")
    return idx


@register_fake("stzs::length_regulate")
def _(dur, n_frames):
    return dur.new_empty((dur.shape[0], n_frames), dtype=torch.int32)


@custom_op("stzs::cfg_euler_step", mutates_args=(), device_types="cuda")
def cfg_euler_step(x: torch.Tensor, D: torch.Tensor, cfg: bool, scale: float, sigma: float,
                   sigma_next: float) -> torch.Tensor:
    """x, D fp32 [R, ...] (R = 2B with CFG: conditional rows first) -> x + (sigma' - sigma)(x - Dg) / sigma."""
    y = x.float().contiguous().clone()
    Dd = D.float().contiguous()
    R = y.shape[0]
    B = R // 2 if cfg else R
    N = y.numel() // R
    L.check(L.load().stzs_cfg_euler(y.data_ptr(), Dd.data_ptr(), B, N, int(cfg), float(scale), float(sigma),
                                    float(sigma_next - sigma), _stream(y)), "stzs::cfg_euler_step")
    return y


@register_fake("stzs::cfg_euler_step")
def _(x, D, cfg, scale, sigma, sigma_next):
    return x.new_empty(x.shape, dtype=torch.float32)


@custom_op("stzs::istft", mutates_args=(), device_types="cuda")
def istft(post: torch.Tensor, n_fft: int, hop: int) -> torch.Tensor:
    """post fp32 [B, Tf, >= n_fft + 2] (n_fft/2+1 log-magnitudes | n_fft/2+1 phase arguments) -> wav [B, (Tf-1) hop]."""
    p = post.float().contiguous()
    B, Tf, ld = p.shape
    wav = torch.empty(B, (Tf - 1) * hop, dtype=torch.float32, device=p.device)
    a = L.IstftArgs()
    a.post, a.wav, a.ldp, a.bsp, a.bsw = p.data_ptr(), wav.data_ptr(), ld, Tf * ld, wav.shape[1]
    a.B, a.Tf, a.n_fft, a.hop_s = B, Tf, n_fft, hop
    L.check(L.load().stzs_istft(C.byref(a), _stream(p)), "stzs::istft")
    return wav


@register_fake("stzs::istft")
def _(post, n_fft, hop):
    return post.new_empty((post.shape[0], (post.shape[1] - 1) * hop), dtype=torch.float32)


def _span(f0, Fc, final, n_fft, hop):
    n0, n1 = C.c_int64(), C.c_int64()
    halo = L.load().stzs_istft_stream_span(f0, Fc, int(final), n_fft, hop, C.byref(n0), C.byref(n1))
    L.check(min(halo, 0), "stzs::istft_stream span")
    return halo, n0.value, n1.value


@custom_op("stzs::istft_stream", mutates_args=(), device_types="cuda")
def istft_stream(post: torch.Tensor, tail: torch.Tensor, f0: int, final: bool, n_fft: int,
                 hop: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """one chunk: post [B, Fc, ld] = frames [f0, f0 + Fc), tail [B, halo, ld] = the previous chunk's returned
    tail (any contents at f0 = 0) -> (its samples [B, n1 - n0], the tail for the next chunk)."""
    p = post.float().contiguous()
    B, Fc, ld = p.shape
    halo, n0, n1 = _span(f0, Fc, final, n_fft, hop)
    tin = tail.float().contiguous()
    if tin.shape != (B, halo, ld):
        raise RuntimeError(f"stzs::istft_stream: tail must be [B, {halo}, {ld}], got {tuple(tin.shape)}")
    wav = torch.empty(B, n1 - n0, dtype=torch.float32, device=p.device)
    tout = torch.zeros(B, halo, ld, dtype=torch.float32, device=p.device)
    a = L.IstftStreamArgs()
    a.post, a.tail_in, a.tail_out, a.wav = p.data_ptr(), tin.data_ptr(), tout.data_ptr(), wav.data_ptr()
    a.ldp, a.bsp, a.bsw, a.ldt = ld, Fc * ld, n1 - n0, ld
    a.B, a.f0, a.Fc, a.final_chunk, a.n_fft, a.hop_s = B, f0, Fc, int(final), n_fft, hop
    L.check(L.load().stzs_istft_stream(C.byref(a), _stream(p)), "stzs::istft_stream")
    return wav, tout


@register_fake("stzs::istft_stream")
def _(post, tail, f0, final, n_fft, hop):
    B, Fc, ld = post.shape
    _, n0, n1 = _span(f0, Fc, final, n_fft, hop)  # host arithmetic only
    return post.new_empty((B, n1 - n0), dtype=torch.float32), post.new_empty(tail.shape, dtype=torch.float32)


# ------------------------------------------------------------------ per-row operators (SURVEY §8(b) list)
# Activations cross this boundary channels-last, [B, T, C] (the kernels' layout) by default; with nct=True they
# cross as torch Conv1d tensors, [B, C, T] (SURVEY §8(b) "NCT at the boundary"): the transpose is folded into the
# copy each operator already makes into / out of the engine's buffers (no extra pass).  Outputs are fp32 copies.

def _out(view: torch.Tensor, nct: bool = False) -> torch.Tensor:
    """an fp32 COPY of an engine buffer view [B, T, C] ([B, C, T] with nct): never the view itself (in fp32 engines
    `.float()` would return the cached buffer, which the next call of the op overwrites), so outputs never alias
    engine storage."""
    if nct:
        return view.transpose(1, 2).to(torch.float32, memory_format=torch.contiguous_format, copy=True)
    return view.to(torch.float32, copy=True)


def _ntc(x: torch.Tensor, nct: bool) -> torch.Tensor:
    """the channels-last view of an operand given as [B, T, C], or as [B, C, T] with nct (a view, no copy)"""
    return x.transpose(1, 2) if nct else x


def _act_in(eng, key, x: torch.Tensor, dtype=None, nct: bool = False):
    """x [B, T, C] ([B, C, T] with nct) -> an engine Act (row pitch padded to 8) holding x in `dtype` (default: the
    engine's activation dtype, fp32 in precise mode); the copy into the buffer does the transpose."""
    from .engine import Act
    x = _ntc(x, nct)
    dtype = eng.adt if dtype is None else dtype
    B, T, Cn = x.shape
    t = eng.buf("op." + key, (B, T, (Cn + 7) // 8 * 8), dtype, zero=True)
    t[:, :, :Cn].copy_(x)
    return Act(t, 0, Cn)


_LSTMS = {"te.lstm": lambda W: W.te_lstm, "pr.dur_lstm": lambda W: W.pr_dur_lstm, "pr.shared": lambda W: W.pr_shared}


@custom_op("stzs::bilstm", mutates_args=(), device_types="cuda")
def bilstm(handle: int, name: str, x: torch.Tensor) -> torch.Tensor:
    """a5 / a8 / text encoder: the named single-layer BiLSTM ("te.lstm", "pr.de{i}", "pr.dur_lstm", "pr.shared") of
    the packed model: x [B, T, in] -> h [B, T, 2H] fp32 (bf16 state in the exchange, fp32 gates)."""
    eng = _eng(handle, x)
    W = eng.W
    if name.startswith("pr.de"):
        lw = W.pr_de[int(name[5:])]
    elif name in _LSTMS:
        lw = _LSTMS[name](W)
    else:
        raise RuntimeError(f"stzs::bilstm: unknown LSTM {name!r}")
    xa = _act_in(eng, "lstm.x", x)
    y = eng.act("op.lstm.y", x.shape[0], x.shape[1], 2 * lw.H, eng.adt)
    eng.lstm(lw, xa, y, "op." + name)
    eng.check_status()
    return _out(y.t[:, :, :2 * lw.H])


def _spec(handle):
    """the registered engine's spec (host metadata: usable by the fake implementations)."""
    eng = _ENGINES.get(int(handle))
    if eng is None:
        raise RuntimeError(f"stzs: unknown engine handle {handle}")
    return eng.spec


@register_fake("stzs::bilstm")
def _(handle, name, x):
    return x.new_empty((x.shape[0], x.shape[1], _spec(handle).pr_hid), dtype=torch.float32)  # 2H = pr_hid = d_txt


@custom_op("stzs::denoiser_fwd", mutates_args=(), device_types="cuda")
def denoiser_fwd(handle: int, h_txt: torch.Tensor, prompt: torch.Tensor, x: torch.Tensor, sigma: float,
                 cfg: bool) -> torch.Tensor:
    """a2: one EDM-preconditioned denoiser evaluation D(x, sigma).  h_txt [B, T_txt, d_txt], prompt [B, L_s, code],
    x [R, L_s, code] (R = 2B with cfg: conditional rows, then null-prompt rows) -> D fp32 [R, L_s, code]."""
    eng = _eng(handle, h_txt, prompt, x)
    ha = _act_in(eng, "h_txt", h_txt)
    xs = x.float().contiguous()
    return eng.denoiser_fwd(ha, prompt.float().contiguous(), xs, float(sigma), bool(cfg)).clone()


@register_fake("stzs::denoiser_fwd")
def _(handle, h_txt, prompt, x, sigma, cfg):
    return x.new_empty(x.shape, dtype=torch.float32)


@custom_op("stzs::f0n_predictor", mutates_args=(), device_types="cuda")
def f0n_predictor(handle: int, en: torch.Tensor, codes: torch.Tensor, nct: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """a8: aligned predictor features en [B, T40, pr_in] ([B, pr_in, T40] with nct), codes [B, L_s, code] -> (F0, N)
    fp32 [B, 2 T40]."""
    eng = _eng(handle, en, codes)
    F0, Nn = eng.f0n_predictor(_act_in(eng, "en", en, nct=nct), codes.float().contiguous())
    eng.check_status()
    return F0.contiguous().clone(), Nn.contiguous().clone()


@register_fake("stzs::f0n_predictor")
def _(handle, en, codes, nct=False):
    B, T40 = en.shape[0], en.shape[2 if nct else 1]
    return en.new_empty((B, 2 * T40), dtype=torch.float32), en.new_empty((B, 2 * T40), dtype=torch.float32)


@custom_op("stzs::decoder_pre", mutates_args=(), device_types="cuda")
def decoder_pre(handle: int, asr: torch.Tensor, F0: torch.Tensor, N: torch.Tensor, codes: torch.Tensor,
                nct: bool = False) -> torch.Tensor:
    """a9: asr [B, T40, d_txt], F0 / N [B, 2 T40], codes [B, L_s, code] -> generator input fp32 [B, 2 T40, dec_out]
    (nct: asr [B, d_txt, T40] in, [B, dec_out, 2 T40] out)."""
    eng = _eng(handle, asr, F0, N, codes)
    S = eng.spec
    asr = _ntc(asr, nct)
    B, T40, D = asr.shape
    enc_in = eng.act("dec.enc_in", B, T40, S.d_txt + 2, eng.dec_dt)
    enc_in.t[:, :, :D].copy_(asr)
    pro = dict(asr_buf=enc_in, F0=F0.float().contiguous(), N=N.float().contiguous(), T40=T40)
    gen_in, _ = eng.decoder_pre(pro, codes.float().contiguous())
    return _out(gen_in.t[:, :, :S.dec_out], nct)


@register_fake("stzs::decoder_pre")
def _(handle, asr, F0, N, codes, nct=False):
    T40 = asr.shape[2 if nct else 1]
    shp = (asr.shape[0], _spec(handle).dec_out, 2 * T40) if nct else (asr.shape[0], 2 * T40, _spec(handle).dec_out)
    return asr.new_empty(shp, dtype=torch.float32)


@custom_op("stzs::sine_gen", mutates_args=(), device_types="cuda")
def sine_gen(handle: int, F0: torch.Tensor, seeds: List[int], nct: bool = False) -> torch.Tensor:
    """a10: harmonic source of F0 [B, T80] and its n_fft STFT -> (real | imag) fp32 [B, T80 hop / hop_s + 1, n_fft + 2]
    ([B, n_fft + 2, Tf] with nct)."""
    eng = _eng(handle, F0)
    S = eng.spec
    har = eng.sine_gen(F0.float().contiguous(), list(seeds))
    Tf = F0.shape[1] * S.hop // S.istft_hop + 1  # (the engine's buffer has rows up to a multiple of the noise stride)
    return _out(har.t[:, :Tf, :S.har_ch], nct)


@register_fake("stzs::sine_gen")
def _(handle, F0, seeds, nct=False):
    S = _spec(handle)
    Tf = F0.shape[1] * S.hop // S.istft_hop + 1
    return F0.new_empty((F0.shape[0], S.har_ch, Tf) if nct else (F0.shape[0], Tf, S.har_ch), dtype=torch.float32)


@custom_op("stzs::conv_transpose_up", mutates_args=(), device_types="cuda")
def conv_transpose_up(handle: int, x: torch.Tensor, har: torch.Tensor, stage: int, nct: bool = False) -> torch.Tensor:
    """a11: generator stage `stage`'s LeakyReLU(0.1) + polyphase ConvTranspose1d (+ ReflectionPad(1,0) on the last
    stage) + noise conv of the harmonic features har [B, Tf, n_fft + 2] -> fp32 [B, T_up, gen_ch[stage]] (nct: x, har
    and the output as [B, C, T])."""
    eng = _eng(handle, x, har)
    S = eng.spec
    from .engine import Act
    har = _ntc(har, nct)
    B, Tf, hc = har.shape
    hb = eng.buf("op.har", (B, Tf, (hc + 31) // 32 * 32), eng.dec_dt, zero=True)
    hb[:, :, :hc].copy_(har)
    xu = eng.upsample(_act_in(eng, "ups.x", x, eng.dec_dt, nct), Act(hb, 0, hc), int(stage))
    return _out(xu.t[:, :, :S.gen_ch[stage]], nct)


@register_fake("stzs::conv_transpose_up")
def _(handle, x, har, stage, nct=False):
    S = _spec(handle)
    T_up = x.shape[2 if nct else 1] * S.up_rates[stage] + (1 if stage == len(S.up_rates) - 1 else 0)
    shp = (x.shape[0], S.gen_ch[stage], T_up) if nct else (x.shape[0], T_up, S.gen_ch[stage])
    return x.new_empty(shp, dtype=torch.float32)


@custom_op("stzs::mrf_resblock", mutates_args=(), device_types="cuda")
def mrf_resblock(handle: int, x: torch.Tensor, codes: torch.Tensor, stage: int, nct: bool = False) -> torch.Tensor:
    """a12: the multi-receptive-field fusion of generator stage `stage` (its rb_kernels AdaIN + Snake + dilated-conv
    resblocks, averaged), AdaIN style from the pooled acoustic codes: x [B, T, C] -> fp32 [B, T, C] (nct: [B, C, T])."""
    eng = _eng(handle, x, codes)
    gbd = eng.dec_style(codes.float().contiguous())
    y = eng.mrf(_act_in(eng, "mrf.x", x, eng.dec_dt, nct), int(stage), gbd, eng.W.dec_norm)
    return _out(y.t[:, :, :x.shape[1 if nct else 2]], nct)


@register_fake("stzs::mrf_resblock")
def _(handle, x, codes, stage, nct=False):
    return x.new_empty(x.shape, dtype=torch.float32)


@custom_op("stzs::conv_post_istft", mutates_args=(), device_types="cuda")
def conv_post_istft(handle: int, x: torch.Tensor, nct: bool = False) -> torch.Tensor:
    """a13: LeakyReLU(0.01) + conv_post + exp / sin spectrum + iSTFT: x [B, Tf, gen_ch[-1]] ([B, gen_ch[-1], Tf] with
    nct) -> wav fp32 [B, (Tf-1) hop_s]."""
    eng = _eng(handle, x)
    wav = eng.istft(eng.conv_post(_act_in(eng, "post.x", x, eng.dec_dt, nct)))
    return wav.clone()


@register_fake("stzs::conv_post_istft")
def _(handle, x, nct=False):
    return x.new_empty((x.shape[0], (x.shape[2 if nct else 1] - 1) * _spec(handle).istft_hop), dtype=torch.float32)


@custom_op("stzs::code_quantize", mutates_args=(), device_types="cuda")
def code_quantize(handle: int, z: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """discrete style codes (README.md:5): z [B, L_s, code] fp32 -> (indices int32 [B, L_s, G], dequantised
    codes fp32 [B, L_s, code]); bit-exact against oracle quantize_codes."""
    eng = _eng(handle, z)
    S = eng.spec
    B, Lr, D = z.shape
    G = S.code_dim // S.vq_group
    idx = torch.empty(B, Lr, G, dtype=torch.int32, device=z.device)
    out = torch.empty(B, Lr, D, dtype=torch.float32, device=z.device)
    eng.code_quantize(z.float().contiguous(), idx, out)
    return idx, out


@register_fake("stzs::code_quantize")
def _(handle, z):
    G = z.shape[2] // _spec(handle).vq_group
    return z.new_empty((z.shape[0], z.shape[1], G), dtype=torch.int32), z.new_empty(z.shape, dtype=torch.float32)


OPS = ["synth", "sample_style", "predict_prosody", "decode", "duration_head", "length_regulate",
       "cfg_euler_step", "istft", "istft_stream", "bilstm", "denoiser_fwd", "f0n_predictor", "decoder_pre",
       "sine_gen", "conv_transpose_up", "mrf_resblock", "conv_post_istft", "code_quantize"]
