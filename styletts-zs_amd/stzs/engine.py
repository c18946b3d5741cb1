"""StyleTTS-ZS synthesis engine on MI355X: the L4 host pipeline over libstzs_hip.so.

API (the upstream inference API is "Under construction",
`/root/reference/README.md:15-16`, so this pins it in the StyleTTS2-family shape
`inference(text, ref_s, diffusion_steps, embedding_scale)`):

    eng = StyleTTSZS(spec, params, device="cuda:0")
    out = eng.synth(tokens, ref_wav, steps=2, cfg_scale=5.0, noise=eps, durations=dur)
    codes = eng.sample_style(h_txt, prompt, eps, steps, cfg_scale)     # (a) style diffusion
    pro   = eng.predict_prosody(h_txt, codes, durations)               # (b) duration/prosody
    wav   = eng.decode(pro, codes, seeds)                              # (c) iSTFT decoder

Every FLOP of synth() -- including the reference-prompt front end (log-mel + prompt encoder, SURVEY
§8(f) rank 1) -- runs in a hand-written gfx950 kernel reached through the C-ABI; PyTorch only
provides device memory (caching allocator) and the stream.  Buffers are cached per shape so a whole
synth() can be captured into one HIP graph (`capture()`), which removes all host launch overhead.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as L
from .spec import Spec
from .weights import ConvW, PackedModel

_DT = {torch.float32: L.F32, torch.bfloat16: L.BF16, torch.float8_e4m3fn: L.F8}
# split-K slices per bf16 denoiser layer linear (stzs_conv_args.splitk), a per-engine setting.  At batch 1 (100
# rows with CFG) ffn2 has 8 output tiles, each streaming its 64 K-steps through one CU's LDS-DMA ring; 4 slices
# spread that over 32 CUs (14.9 -> 10.5 us; configs[1] p50 10.1 -> 9.9 ms).  The K = 512 linears lose (the hand-off
# costs more than their 16 K-steps), and so does every linear at 6 400 rows (ffn2 26.7 -> 40.5 us; bench value
# -1.5%), so throughput engines keep it off (DN_SPLITK) and the batch-1 latency engine uses LATENCY_DN_SPLITK
# (tools/gemm_bench.py, DESIGN.md §5 "Batch-1 latency").  Within one engine the table is a property of the weight,
# applied at every row count, so its results stay batch-invariant.  STZS_DN_SPLITK overrides the default of an
# engine built without dn_splitk: "0" = off, or e.g. "ff2=4,o=2".
DN_SPLITK = {}
LATENCY_DN_SPLITK = dict(ff2=4)
# small-M linears on the whole chip (csrc/rows.hip, STZS_CONV_ROWS): per denoiser linear the number of K slices Z
# (1 = no split).  The batch-1 latency engine's table; like the split-K table it is a property of the weight applied
# at every row count (batch-invariant), and it takes precedence over dn_splitk.  STZS_DN_ROWS overrides the default
# ({}): "0" = off, or e.g. "qkv=1,ff2=4".
DN_ROWS = {}
LATENCY_DN_ROWS = dict(inp=1, qkv=1, o=1, q=1, co=1, ff1=1, ff2=4, out=1)
# in-launch split-K (input-channel chunks, csrc/conv.hip conv_mfma) of the text-encoder k5 convs: at batch 1 their
# grid is 4 workgroups of 80 K-steps each.  A per-engine property of the weight (batch-invariant); the batch-1
# latency engine's value.  STZS_TE_SPLITK overrides an engine built without te_splitk.
TE_SPLITK = 0
LATENCY_TE_SPLITK = 4
# split-K slices of the decoder / predictor AdaIN-block convs (their generic-layout copies, BlkW.conv1s / conv2s) in
# the batch-1 latency engine: at 200-400 frames a decoder conv is 16 tiles x 108 K-steps on 16 CUs; 0 = off.  16 (r05)
# = one input-channel chunk per slice for every block conv (<= 9 chunks): the DEEP form (csrc/conv.hip)
BLK_SPLITK = 0
LATENCY_BLK_SPLITK = 16


_ES = {L.F32: 4, L.BF16: 2, L.F8: 1}


def _ln_cost(a):
    """(FLOP, bytes) of a row LayerNorm launch: the rows read once and written once (the FLOPs are negligible)."""
    return 0, a.R * a.C * (_ES[a.in_dtype] + _ES[a.out_dtype])


def _table_env(var, default):
    v = os.environ.get(var)
    if v is None:
        return dict(default)
    if v.strip() in ("", "0"):
        return {}
    return {k: int(n) for k, n in (kv.split("=") for kv in v.split(","))}


def _dn_splitk_default():
    return _table_env("STZS_DN_SPLITK", DN_SPLITK)


def _rup(x, m):
    return (x + m - 1) // m * m




@dataclass
class Act:
    """channels-last activation view: buffer [B, T, ld], logical channels [c0, c0 + C)."""
    t: torch.Tensor
    c0: int = 0
    C: int = -1

    def __post_init__(self):
        if self.C < 0:
            self.C = self.t.shape[-1] - self.c0

    @property
    def B(self):
        return self.t.shape[0]

    @property
    def T(self):
        return self.t.shape[1]

    @property
    def ld(self):
        return self.t.shape[2]

    @property
    def bs(self):
        """batch stride in elements: the tensor's own (a view of the first T rows of a longer buffer -- the harmonic
        source's -- keeps the buffer's stride; for contiguous buffers this is T * ld)"""
        return self.t.stride(0)

    @property
    def ptr(self):
        return self.t.data_ptr() + self.c0 * self.t.element_size()

    @property
    def dt(self):
        return _DT[self.t.dtype]

    def sl(self, c0, C):
        return Act(self.t, self.c0 + c0, C)

    def rows(self, b0, nb):
        return Act(self.t[b0:b0 + nb], self.c0, self.C)


def sigma_schedule(spec: Spec, steps: int):
    """Distilled pins 1: [smax, 0], 2: [smax, 0.5, 0]; otherwise Karras(rho) + trailing 0 (a1)."""
    if steps == 1:
        return [spec.sigma_max, 0.0]
    if steps == 2:
        return [spec.sigma_max, 0.5, 0.0]
    lo, hi = spec.sigma_min ** (1 / spec.rho), spec.sigma_max ** (1 / spec.rho)
    return [(hi + i / (steps - 1) * (lo - hi)) ** spec.rho for i in range(steps)] + [0.0]


def edm_coeffs(spec: Spec, sigma: float):
    sd = spec.sigma_data
    return dict(c_in=1.0 / math.sqrt(sigma ** 2 + sd ** 2), c_skip=sd ** 2 / (sigma ** 2 + sd ** 2),
                c_out=sigma * sd / math.sqrt(sigma ** 2 + sd ** 2), c_noise=math.log(sigma) / 4.0)


def fourier_features(spec: Spec, c_noise: float) -> np.ndarray:
    half = spec.dn_fourier // 2
    f = np.exp(-math.log(10000.0) * np.arange(half) / half)
    arg = 1000.0 * c_noise * f
    return np.concatenate([np.cos(arg), np.sin(arg)]).astype(np.float32)


class _StatsRef:
    """InstanceNorm statistics as fp32 (sum, sumsq) partials of `nch` chunks of `chunk_rows` rows, [B][nch][ld][2]
    in `part`, finalised into mean / rstd (stzs_chan_stats_final) only when something needs them: a generic-path
    conv reads the partials in its AdaIN prologue instead (stzs_conv_args.pro_part, the same bits)."""

    def __init__(self, eng, part, ld, nch, T, B, mean, rstd, chunk_rows):
        self.eng, self.part, self.ld, self.nch, self.T, self.B = eng, part, ld, nch, T, B
        self.mean, self.rstd, self.chunk_rows, self.done = mean, rstd, chunk_rows, False

    def finalize(self):
        if not self.done:
            s = L.StatsArgs()
            s.mean, s.rstd, s.partial = self.mean.data_ptr(), self.rstd.data_ptr(), self.part.data_ptr()
            s.stat_bs, s.B, s.T, s.C, s.eps = self.ld, self.B, self.T, self.ld, 1e-5
            self.eng.launches += 1
            L.check(self.eng.lib.stzs_chan_stats_final(C.byref(s), self.chunk_rows, self.eng.stream()),
                    "chan_stats_final")
            self.done = True

    def mean_ptr(self):
        self.finalize()
        return self.mean.data_ptr()

    def rstd_ptr(self):
        self.finalize()
        return self.rstd.data_ptr()


class _StatPtr:
    """the mean (which 0) or rstd (1) of a _StatsRef, usable wherever a tensor's data_ptr() is taken (finalises)."""

    def __init__(self, ref, which):
        self.ref, self.which = ref, which

    def data_ptr(self):
        return self.ref.mean_ptr() if self.which == 0 else self.ref.rstd_ptr()

    def tensor(self):
        self.ref.finalize()
        return self.ref.mean if self.which == 0 else self.ref.rstd

    def clone(self):
        return self.tensor().clone()

    def __getitem__(self, k):
        return self.tensor()[k]


class StyleTTSZS:
    def __init__(self, spec: Spec, params, device="cuda:0", fill=True, fp8_denoiser=False, precise_decoder=False,
                 packed: PackedModel = None, branch_streams=False, precise=False, dn_splitk=None, dn_rows=None,
                 te_splitk=None, blk_splitk=None, dur_overlap=None):
        """packed: an already packed (e.g. RCCL-broadcast, stzs/dist.py) PackedModel on `device`; params unused.
        fp8_denoiser: run the per-layer denoiser linears (qkv, o, q, co, ff1, ff2) on e4m3fn MFMA with
        per-row activation / per-column weight scales (configs[4]); bf16 otherwise.
        precise_decoder: PARITY mode for the decoder -- pre-blocks, generator and conv_post keep fp32 activations
        and run every conv on split bf16 operands (hi*hi + hi*lo + lo*hi, STZS_CONV_W_X3, csrc/conv.hip conv_x3).
        precise: the whole pipeline in that mode -- text encoder, style diffusion and prosody predictor too (fp32
        activations, split-operand convs / linears / LSTM recurrences, fp32 attention, libm activations) -- the
        mode that meets the north-star log-mel L1 <= 1e-3 END TO END vs the fp32 oracle (tools/precision_probe.py:
        2.2e-4 in emulation); bf16 weights/activations alone cost ~5e-2.  The reference-prompt
        front end stays bf16: its output is quantised to discrete codes.
        branch_streams: run the independent branches (text encoder || prompt encoder, F0 || N predictor branches)
        on forked side streams (graph-capturable: the fork/join is stream-ordered); each branch has its own
        scratch (statistics slab / workspace), results bit-identical to the single-stream order.
        dur_overlap: with durations given, the alignment reads them directly and the duration LSTM runs in ONE
        launch with the shared F0/N LSTM (stzs_lstm_pair), its projection and durations kernel after the F0/N
        branches -- bit-identical (default on; env STZS_DUR_OVERLAP=0 turns it off)."""
        self.spec = spec
        self.fp8_denoiser = fp8_denoiser
        precise_decoder = precise_decoder or precise
        self.precise = precise_decoder
        self.precise_all = precise
        # precise + fp8_denoiser: the configs[4] long-form mode -- the style sampler on the fp8 denoiser (bf16
        # activations), text encoder / prosody predictor / decoder precise (the F0 phase the harmonic source
        # integrates over 30 s needs the predictor's fp32-level F0: DESIGN.md §3)
        self.lowp_dn = bool(precise and fp8_denoiser)
        self.dec_dt = torch.float32 if precise_decoder else torch.bfloat16
        self.adt = torch.float32 if precise else torch.bfloat16  # text / predictor activations
        self.sdt = torch.bfloat16 if self.lowp_dn else self.adt  # style-sampler activations
        self.device = torch.device(device)
        self.lib = L.load()
        L.check(self.lib.stzs_init(self.device.index or 0), "stzs_init")
        if packed is not None:
            assert packed.spec == spec and packed.arena.buf.device == self.device and \
                packed.precise == precise_decoder and packed.precise_all == precise and \
                getattr(packed, "lowp_denoiser", False) == self.lowp_dn, \
                "packed model: spec / device / precise mode differ"
            self.W = packed
        else:
            self.W = PackedModel(spec, params, self.device, fill=fill, precise=precise_decoder, precise_all=precise,
                                 lowp_denoiser=self.lowp_dn)
        self._bufs = {}
        self._retired = []
        self._consts = {}
        self.branch_streams = branch_streams
        self._branch = ""  # scratch-key suffix of the branch being enqueued (see fork())
        self._side = {}  # (fork depth, branch) -> side stream
        self._depth = 0  # nesting depth of fork() calls being enqueued
        self.dur_overlap = bool(int(os.environ.get("STZS_DUR_OVERLAP", "1"))) if dur_overlap is None else \
            bool(dur_overlap)
        self.launches = 0
        self.lstm_spin_limit = 0  # 0 = the library default; tests force tiny values
        # split-K of the bf16 denoiser layer linears (stzs_conv_args.splitk): a property of the weight, used at
        # every batch size so results stay batch-invariant; {} turns it off
        self.dn_splitk = _dn_splitk_default() if dn_splitk is None else dict(dn_splitk)
        # small-M whole-chip form of the bf16 denoiser linears (csrc/rows.hip): {linear: K slices}; a per-engine
        # property of the weight like dn_splitk (batch-invariant), taking precedence over it
        self.dn_rows = _table_env("STZS_DN_ROWS", DN_ROWS) if dn_rows is None else dict(dn_rows)
        # split-K slices of the text-encoder convs (LATENCY_TE_SPLITK); 0 = off
        self.te_splitk = int(os.environ.get("STZS_TE_SPLITK", TE_SPLITK)) if te_splitk is None else int(te_splitk)
        # split-K slices of the bf16 AdaIN-block convs (LATENCY_BLK_SPLITK); 0 = the register-direct form
        self.blk_splitk = int(os.environ.get("STZS_BLK_SPLITK", BLK_SPLITK)) if blk_splitk is None else int(blk_splitk)
        # InstanceNorm statistics of <= 8 partial chunks handed to the consuming generic-path conv unfinalised
        # (stzs_conv_args.pro_part: the prologue finalises them, bit-identical, one launch less per statistics) --
        # the engines whose AdaIN-block convs run the generic path (blk_splitk); STZS_DEFER_STATS=0|1 overrides
        self.defer_stats = os.environ.get("STZS_DEFER_STATS", "1" if self.blk_splitk else "0") != "0"
        # (r06) small batches (<= 4 utterances): the generator MRF's three resblocks advanced side by side, each layer's
        # three convs in one launch (stzs_conv1d_group, csrc/mrfv.hip mrfv_trio) -- bit-identical; STZS_MRF_TRIO=0: off
        self.mrf_trio = os.environ.get("STZS_MRF_TRIO", "1") != "0"
        # (r06) the batch-1 engine (blk_splitk): the prosody predictor's F0 and N branches in lockstep, each conv pair
        # in one launch pair (stzs_conv1d_group -> conv_mfma_pair) -- bit-identical; STZS_F0N_PAIR=0: off
        self.f0n_pair = os.environ.get("STZS_F0N_PAIR", "1") != "0"
        # (r06) the denoiser layers' cross-attention K / V projections as one stacked linear; STZS_KV_FUSE=0: per layer
        self.kv_fuse = os.environ.get("STZS_KV_FUSE", "1") != "0"
        # the per-utterance linears (one row per utterance or per sigma step: the sigma-embedding MLP, the pooled-
        # prompt projection, the decoder / predictor AdaIN gamma-beta GEMMs) on the whole-chip small-M form at every
        # batch size (a per-weight choice: batch-invariant); on the tiled GEMM they ran on 1-4 workgroups each.
        # STZS_SMALL_ROWS=0 turns it off.
        self.small_rows = os.environ.get("STZS_SMALL_ROWS", "1") != "0"
        # with the denoiser linears on the small-M rows form (dn_rows): each adaLN / affine LayerNorm fused into the
        # one linear that reads it (stzs_ln_linear, csrc/lnrows.hip) instead of its own launch.  STZS_LN_FUSE=0: off
        self.ln_fuse = os.environ.get("STZS_LN_FUSE", "1") != "0"
        # rows-form linears with K <= rows16_maxk on the 16-row register-direct form (csrc/lnrows.hip rows16: up to 16
        # K-steps of both operands in flight, no cross-wave reduction, no K slices).  STZS_ROWS16=0: csrc/rows.hip
        self.rows16 = os.environ.get("STZS_ROWS16", "1") != "0"
        self.rows16_split = os.environ.get("STZS_ROWS16_SPLIT", "1") != "0"  # (the Z-slice form: batch-1 ffn2)
        # (unsliced up to K 512: ffn2, K 2048, as one 64-K-step chain measured no faster than rows.hip Z 4, r04_t;
        # with its 4 slices on the split form it is, r04_x)
        self.rows16_maxk = int(os.environ.get("STZS_ROWS16_MAXK", "512"))
        # the last generator stage's noise conv fused into its ConvTranspose (bf16 engines); STZS_UPS_NOISE=0: off
        self.ups_noise_fused = os.environ.get("STZS_UPS_NOISE", "1") != "0"
        # the first stage's strided noise conv on super-rows of the harmonic source (register-direct kernel, bf16
        # engines); STZS_NOISE_SUPER=0: the stride-6 conv_mfma form
        self.noise_super = os.environ.get("STZS_NOISE_SUPER", "1") != "0"
        # precise mode: the FRAG32 convs (MRF, AdaIN-block k3) on the split-operand register-direct kernel
        # (csrc/mrfx.hip) instead of the LDS-ring conv_x3; STZS_MRFX=0: conv_x3
        self.mrfx = os.environ.get("STZS_MRFX", "1") != "0"
        # diagnostic conv flag bits ORed into every stzs_conv1d call (e.g. STZS_CONV_LINEAR_IDS = 128)
        self.conv_flags = int(os.environ.get("STZS_CONV_FLAGS", "0"), 0)
        # device status word collecting the LSTM exchange's spin-timeout flag over every launch (eager or
        # graph-replayed); check_status() reads it and raises
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.prompt_idx = None  # discrete prompt codes of the last prompt_encode (device int32 [B, L_s, G])

    def check_status(self, reset=True):
        """raise RuntimeError if any LSTM exchange since the last check timed out (its h-states are wrong).
        Synchronizes the device (one 4-B copy)."""
        v = int(self.status.item())
        if reset and v:
            self.status.zero_()
        if v & L.STATUS_LSTM_TIMEOUT:
            raise RuntimeError("stzs_lstm: exchange spin timed out (LSTM workgroups not co-resident?); "
                               "the prosody outputs of this call are invalid")
        return v

    @classmethod
    def from_checkpoint(cls, path: str, device="cuda:0", **kw) -> "StyleTTSZS":
        """engine on the parameters of a safetensors checkpoint (stzs/checkpoint.py), spec from its metadata."""
        from .checkpoint import load_params
        params, spec = load_params(path)
        return cls(spec, params, device=device, **kw)

    # ------------------------------------------------------------------ plumbing
    def stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def buf(self, key, shape, dtype=torch.bfloat16, zero=False):
        """cached device buffer: ONE storage per (key, dtype), reused by capacity for every shape that fits, so a
        stream of distinct request lengths (stzs/scheduler.py) does not allocate a buffer set per length.  The
        address is stable while the shape fits (graph-capturable); a shape change re-zeroes zero=True buffers
        (their padding rows / channels are read by the kernels); growth allocates 1.25x the request and keeps
        the old storage alive in self._retired, so graphs captured on it stay valid."""
        k = (key, dtype)
        shape = tuple(int(v) for v in shape)
        n = 1
        for v in shape:
            n *= v
        ent = self._bufs.get(k)
        # a storage a captured graph reads (ent[3], set by capture()) is never re-viewed at another shape:
        # the graph would replay over the other shape's data and padding
        if ent is None or ent[0].numel() < n or (ent[3] and ent[1] != shape):
            if ent is not None:
                self._retired.append(ent[0])
            cap = n if ent is None else max(n, int(ent[0].numel() * 1.25))
            store = torch.zeros(max(cap, 1), dtype=dtype, device=self.device) if zero else \
                torch.empty(max(cap, 1), dtype=dtype, device=self.device)
            ent = self._bufs[k] = [store, shape, store[:n].view(shape), False]
            return ent[2]
        if ent[1] != shape:
            ent[1] = shape
            ent[2] = ent[0][:n].view(shape)
            if zero:
                ent[2].zero_()
        return ent[2]

    def buffer_bytes(self) -> int:
        """device bytes held by the buffer cache (live storages + retired ones kept for captured graphs)."""
        live = sum(e[0].numel() * e[0].element_size() for k, e in self._bufs.items() if isinstance(k, tuple))
        return live + sum(t.numel() * t.element_size() for t in self._retired)

    def act(self, key, B, T, C, dtype=torch.bfloat16):
        return Act(self.buf(key, (B, T, _rup(C, 8)), dtype, zero=True), 0, C)

    def _t(self, x):
        """weight reference -> device tensor (arena name, or an already-resolved tensor)."""
        return x if isinstance(x, torch.Tensor) else self.W.t(x)

    def _call(self, fn, arg, what, cost=None, b=None):
        """one library launch (b: a second struct argument, stzs_lstm_pair); cost = (algorithmic FLOP, algorithmic
        bytes) of it, recorded with HIP events when a timer of every launch is running (start_timer("*"), the
        per-stage roofline of bench.py)."""
        self.launches += 1
        args = (C.byref(arg),) if b is None else (C.byref(arg), C.byref(b))
        tm = self.timer
        if tm is not None and tm["all"] and cost is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(fn(*args, self.stream()), what)
            e1.record()
            tm["rec"].append((what, e0, e1, float(cost[0]), float(cost[1]), None, self.stage))
            return
        L.check(fn(*args, self.stream()), what)

    # ------------------------------------------------------------------ ops
    def conv(self, cw: ConvW, x: Act, y: Act, *, T_out=None, pad=0, dil=1, stride=1, pro=None, pro_act=L.ACT_NONE,
             pro_slope=0.0, pro_alpha=None, cscale=1.0, res: Act = None, res_tdiv=1, acc_in: Act = None,
             alpha=1.0, beta=0.0, gate=None, gate_bs=0, epi_act=L.ACT_NONE, epi_slope=0.0, ups_pad=0,
             T_final=0, refl=0, flags=0, stats_key=None, x_scale=None, post_ln=None, pre_ln=None, splitk=0, rows=0,
             attn=None, collect=None, what="conv"):
        """-> y, or (y, (mean, rstd, stat_bs)) with stats_key: InstanceNorm statistics of the stored
        output fused into the conv epilogue (per-tile partials) + one small finalize launch.
        collect (a list): append the conv's stzs_conv_args to it instead of launching (the caller launches the
        collected problems with stzs_conv1d_group, and finalises their statistics -- returned unfinalised, per-key
        slabs -- with _finalize_group).
        post_ln (stzs_rowln_args) / attn ((q, k, v, o) Acts): the LayerNorm / attention that consumes y, launched
        behind the linear.  (r03 also ran them, and the sampler's CFG + Euler step, inside the small-M linear's launch
        by its last-arriving workgroups: bit-identical but slower at batch 1, removed in r04 -- DESIGN.md §5.)
        pre_ln (stzs_rowln_args): the LayerNorm whose output x is, launched before the linear -- or, on the small-M
        rows form, fused into it (stzs_ln_linear, csrc/lnrows.hip: the normalised rows never leave the chip)."""
        W = self.W
        a = L.ConvArgs()
        a.x, a.w, a.y = x.ptr, self._t(cw.w).data_ptr(), y.ptr
        a.bias = self._t(cw.b).data_ptr() if cw.b is not None else None
        a.ldx, a.bsx, a.ldy, a.bsy = x.ld, x.bs, y.ld, y.bs
        a.B, a.T_in, a.Ci, a.Co, a.ks, a.dil, a.stride, a.pad = x.B, x.T, cw.Ci, cw.Co, cw.ks, dil, stride, pad
        assert x.C == cw.Ci, (what, x.C, cw.Ci)
        if cw.ups:
            a.T_out = x.T + 1
            a.ups, a.ups_pad, a.T_final, a.refl = cw.ups, ups_pad, T_final, refl
            a.pad = 1
        else:
            a.T_out = T_out if T_out is not None else (x.T + 2 * pad - dil * (cw.ks - 1) - 1) // stride + 1
        a.ci_pad, a.co_pad, a.cic = cw.ci_pad, cw.co_pad, cw.cic
        a.in_dtype, a.out_dtype = x.dt, y.dt
        pro_ref = None
        if pro is not None:  # AdaIN: (mean, rstd, stat_bs, gb_ptr, gb_bs, beta_off)
            mean, rstd, stat_bs, gbp, gb_bs, boff = pro
            a.pro_mode = L.PRO_ADAIN
            if isinstance(mean, _StatPtr) and not mean.ref.done:
                pro_ref = mean.ref  # (resolved below, once the path is known)
            else:
                a.pro_mean, a.pro_rstd = mean.data_ptr(), rstd.data_ptr()
            a.stat_bs = stat_bs
            a.pro_gb, a.gb_bs, a.gb_beta_off = gbp, gb_bs, boff
        a.pro_act, a.pro_slope, a.pro_cscale = pro_act, pro_slope, cscale
        a.pro_alpha = self._t(pro_alpha).data_ptr() if pro_alpha is not None else None
        if res is not None:
            assert res.t.dtype == y.t.dtype
            a.res, a.ldr, a.bsr = res.ptr, res.ld, (res.bs if res.B > 1 or res.B == y.B else 0)
        a.res_tdiv = res_tdiv
        if acc_in is not None:
            a.acc_in, a.lda, a.bsa = acc_in.ptr, acc_in.ld, acc_in.bs
        if gate is not None:
            a.gate, a.gate_bs = gate, gate_bs
        a.alpha, a.beta, a.epi_act, a.epi_slope = alpha, beta, epi_act, epi_slope
        if cw.f8:
            assert x.t.dtype == torch.float8_e4m3fn and x_scale is not None, what
            a.x_scale, a.w_scale = x_scale.data_ptr(), self._t(cw.wscale).data_ptr()
        if (cw.ks == 1 and stride == 1 and pad == 0 and not cw.ups and pro is None and pro_act == L.ACT_NONE
                and not getattr(cw, "frag32", False)  # (the 1x1 block shortcuts on the register-direct form)
                and cscale == 1.0 and x.t.dtype in (torch.bfloat16, torch.float8_e4m3fn)
                and x.c0 + cw.ci_pad <= x.ld and a.T_out == x.T):
            flags |= 8  # STZS_CONV_A_DMA: every row readable over ci_pad channels -> LDS-DMA GEMM path
        fx3_conv = (cw.ks in (3, 7, 11) and epi_act == L.ACT_NONE and gate is None and
                    (pro_act == L.ACT_SNAKE or (cw.ks == 3 and acc_in is None) or
                     (cw.Co <= 32 and cw.ks == 7 and pro_act == L.ACT_LEAKY and pro is None and res is None and
                      acc_in is None and stats_key is None)))  # (the last: conv_post on the narrow form)
        fx3_lin = (cw.ks == 1 and pad == 0 and pro is None and pro_act == L.ACT_NONE and stats_key is None and
                   a.T_out == x.T and epi_act in (L.ACT_NONE, L.ACT_GELU, L.ACT_SILU) and res_tdiv == 1)
        if (getattr(cw, "fx3", None) is not None and self.mrfx and x.t.dtype == torch.float32 and
                y.t.dtype == torch.float32 and stride == 1 and not cw.ups and (fx3_conv or fx3_lin) and
                (res is None or res.t.dtype == torch.float32) and x.ptr % 32 == 0 and y.ptr % 32 == 0):
            # precise mode, register-direct: split bf16 operands on the mrfv data movement (csrc/mrfx.hip; the linears
            # on its FLAT form mrfx_lin)
            a.w, a.cic = self._t(cw.fx3).data_ptr(), 128
            flags = (flags & ~8) | L.CONV_W_FRAG32X3
        elif cw.wx3 is not None:  # precise mode: split bf16 operands (csrc/conv.hip conv_x3)
            a.w, a.cic = self._t(cw.wx3).data_ptr(), 32
            flags = (flags & ~8) | L.CONV_W_X3
        elif cw.w32 is not None:  # fp32 operands on fp32 MFMA (csrc/conv.hip conv_f32)
            a.w, a.cic = self._t(cw.w32).data_ptr(), 32
            flags = (flags & ~8) | L.CONV_W_F32
        elif getattr(cw, "frag32", False):
            flags |= L.CONV_W_FRAG32  # register-direct MRF kernel (csrc/mrfv.hip)
        elif getattr(cw, "lane16", False):
            flags |= L.CONV_W_LANE16  # MRF-family kernel (csrc/mrf.hip)
        elif getattr(cw, "narrow32", False):
            flags |= L.CONV_W_NARROW32  # narrow conv (csrc/mrf.hip)
        a.flags = flags | self.conv_flags
        nk = cw.ci_pad // 32
        if rows > 0 and not (nk % (4 * rows) == 0 and nk // (4 * rows) in (1, 2, 4, 8, 16)):
            rows = 0  # (a function of K only: batch invariance holds)
        if (rows > 0 and cw.ks == 1 and stride == 1 and pad == 0 and not cw.ups and pro is None and
                pro_act == L.ACT_NONE and not cw.f8 and cw.wx3 is None and cw.w32 is None and stats_key is None and
                (x.t.dtype == torch.float32 or (x.t.dtype == torch.bfloat16 and cscale == 1.0)) and
                epi_act in (L.ACT_NONE, L.ACT_GELU, L.ACT_SILU) and
                x.c0 + cw.ci_pad <= x.ld and a.T_out == x.T):
            # small-M linear on the whole chip (csrc/rows.hip): 16-column tiles x K split in `rows` slices
            a.flags = (a.flags & ~8) | L.CONV_ROWS
            a.splitk = rows if rows > 1 else 0
            if rows > 1:
                nb = self.lib.stzs_conv_rows_workspace(x.B * x.T, cw.Co, rows)
                a.splitk_ws = self._scratch("rows_ws", nb // 4 + 1).data_ptr()
                a.splitk_ctr = self._counters("rows_ctr", nb // (rows * 16)).data_ptr()
            splitk = 0
        if a.flags & 8:  # LDS-DMA GEMM: the slices split the K-steps (a function of K only: batch invariance holds)
            splitk = min(splitk, 4)  # (gemm_glds takes 2 or 4 slices)
            while splitk > 1 and (cw.ci_pad // 32) % splitk:
                splitk //= 2
        elif splitk > 1:  # conv_mfma: the slices split the input-channel chunks (2..16, at most one slice per chunk;
            # one chunk per slice takes the DEEP form: the slice's whole weight stream issued at entry)
            splitk = min(splitk, 16, cw.ci_pad // cw.cic)
        if splitk > 1 and (a.flags & 8) and not cw.f8 and cw.wx3 is None and cw.w32 is None:
            # in-launch split-K (stzs_conv_args.splitk): per-branch fp32 slabs + self-resetting tile counters
            nb = self.lib.stzs_conv_splitk_workspace(x.B * x.T, cw.co_pad, splitk)
            assert nb > 0, (what, splitk)
            a.splitk, a.splitk_ws = splitk, self._scratch("sk_ws", nb // 4).data_ptr()
            a.splitk_ctr = self._counters("sk_ctr", nb // (splitk * 32768)).data_ptr()
        elif (splitk > 1 and not (a.flags & (8 | L.CONV_ROWS | L.CONV_W_X3 | L.CONV_W_F32 | L.CONV_W_FRAG32 |
                                             L.CONV_W_LANE16 | L.CONV_W_NARROW32 | L.CONV_W_FRAG32X3)) and not cw.f8):
            # conv_mfma split over input-channel chunks: one 64-KB fp32 slab per (128-row tile, slice) + a ticket
            # per tile (grid.x is at most B x ceil(T_out / 128))
            tiles = x.B * ((a.T_out + 127) // 128) * (cw.co_pad // 128)
            a.splitk = splitk
            gs = f".g{len(collect)}" if collect is not None else ""  # (a collected problem: its own slabs)
            a.splitk_ws = self._scratch("csk_ws" + gs, tiles * splitk * 16384).data_ptr()
            a.splitk_ctr = self._counters("csk_ctr" + gs, tiles).data_ptr()
        if pro_ref is not None:
            generic = not (a.flags & (8 | L.CONV_ROWS | L.CONV_W_X3 | L.CONV_W_F32 | L.CONV_W_FRAG32 |
                                      L.CONV_W_LANE16 | L.CONV_W_NARROW32 | L.CONV_W_FRAG32X3)) and not cw.f8
            if generic and pre_ln is None and pro_ref.nch <= 8:  # the prologue finalises the partials itself
                a.pro_part, a.pro_ld, a.pro_nch, a.pro_T, a.pro_eps = pro_ref.part.data_ptr(), pro_ref.ld, pro_ref.nch, \
                    pro_ref.T, 1e-5
            else:
                a.pro_mean, a.pro_rstd = pro_ref.mean_ptr(), pro_ref.rstd_ptr()
        st = None
        if stats_key is not None:
            Cc = _rup(cw.Co, 8)
            ntile = (a.T_out + L.CONV_STAT_ROWS - 1) // L.CONV_STAT_ROWS
            defer = collect is not None or (self.defer_stats and ntile <= 8)
            # (deferred: the partials must outlive this launch until their consumer reads them -- a slab per key)
            slab = self._scratch("stat_slab." + stats_key, y.B * ntile * Cc * 2, 1024) if defer else self._slab(y.B * ntile * Cc * 2)
            a.stat_part, a.stat_ld = slab.data_ptr(), Cc
            st = (slab, Cc, self.buf(stats_key + ".m", (y.B, Cc), torch.float32),
                  self.buf(stats_key + ".r", (y.B, Cc), torch.float32), defer, ntile)
        tm = self.timer
        launch = lambda: self.lib.stzs_conv1d(C.byref(a), self.stream())
        fused = False
        if pre_ln is not None:
            nk = cw.ci_pad // 32
            fused = bool(a.flags & L.CONV_ROWS) and a.splitk <= 1 and res is None and gate is None and \
                st is None and pre_ln.C == cw.Ci == cw.ci_pad and nk in (4, 8, 16) and pre_ln.out_dtype == L.BF16 and \
                pre_ln.act == L.ACT_NONE and (pre_ln.x or 0) % 16 == 0 and pre_ln.ldx % 8 == 0 and \
                pre_ln.gdiv > 0 and pre_ln.R < (1 << 22) - 16 and \
                (not pre_ln.G or (pre_ln.gs % 8 == 0 and pre_ln.G % 32 == 0)) and \
                (not pre_ln.Bt or (pre_ln.bs % 8 == 0 and pre_ln.Bt % 32 == 0))
            # (every condition stzs_ln_linear checks, csrc/lnrows.hip: a shape it refuses takes the two launches)
            if fused:
                launch = lambda: self.lib.stzs_ln_linear(C.byref(a), C.byref(pre_ln), self.stream())
            else:
                self._call(self.lib.stzs_row_layernorm, pre_ln, what + ".ln", cost=_ln_cost(pre_ln))
        # a rows-form linear on the 16-row register-direct form (stzs_ln_linear, ln = NULL): K <= rows16_maxk as one
        # sequential chain per element (its K slices dropped), or with its Z in {2, 4} slices of 4..16 K-steps
        nk = cw.ci_pad // 32
        r16 = (pre_ln is None and self.rows16 and bool(a.flags & L.CONV_ROWS) and st is None and
               (res is None or res_tdiv == 1) and x.ptr % 16 == 0 and x.ld % 8 == 0 and x.bs % 8 == 0)
        r16_split = r16 and self.rows16_split and a.splitk in (2, 4) and nk % a.splitk == 0 and \
            nk // a.splitk in (4, 8, 16)
        r16 = r16_split or (r16 and nk in (4, 8, 16, 32, 64) and cw.ci_pad <= self.rows16_maxk)
        if r16:
            if not r16_split:
                a.splitk = 0
            launch = lambda: self.lib.stzs_ln_linear(C.byref(a), None, self.stream())
        if collect is not None:
            assert not fused and not r16 and pre_ln is None and post_ln is None and attn is None, what
            collect.append(a)
        elif tm is not None and (tm["all"] or what in tm["tags"]):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self.launches += 1
            L.check(launch(), what)
            e1.record()
            flops = 2.0 * y.B * a.T_out * (cw.ups or 1) * cw.Co * cw.Ci * cw.ks
            if cw.wx3 is not None:  # precise mode: 3 bf16 MFMA products per fp32 product (bf16x3-equivalent FLOP)
                flops *= 3.0
            # algorithmic bytes: input tile once + output once (+ residual/acc reads), bf16/f32 as stored, + the
            # weights once (bf16; e4m3 for the fp8 linears; hi + lo for the split-operand precise form)
            wbytes = (cw.ups or 1) * cw.Co * cw.Ci * cw.ks * (1 if cw.f8 else (4 if cw.wx3 is not None else 2))
            opnd = lambda v: v.B * v.T * v.C * v.t.element_size() if v is not None else 0
            byt = x.B * x.T * x.C * x.t.element_size() + y.B * a.T_out * (cw.ups or 1) * cw.Co * y.t.element_size() + \
                opnd(res) + opnd(acc_in) + wbytes
            if fused:  # the LayerNorm's input rows instead of x
                byt += pre_ln.R * pre_ln.C * (4 if pre_ln.in_dtype == L.F32 else 2) - x.B * x.T * x.C * x.t.element_size()
            tm["rec"].append((what, e0, e1, flops, byt, (cw.ks, dil, a.T_out, cw.Co), self.stage))
        elif fused or r16:
            self.launches += 1
            L.check(launch(), what)
        else:
            self._call(self.lib.stzs_conv1d, a, what)
        if post_ln is not None:  # the LayerNorm that consumes this linear's output (stzs_rowln_args)
            self._call(self.lib.stzs_row_layernorm, post_ln, what + ".ln", cost=_ln_cost(post_ln))
        if attn is not None:  # the attention whose q (k, v) this linear produced
            self.attention(*attn)
        if st is None:
            return y
        slab, Cc, mean, rstd, defer, ntile = st
        ref = _StatsRef(self, slab, Cc, ntile, a.T_out, y.B, mean, rstd, L.CONV_STAT_ROWS)
        if not defer:
            ref.finalize()
            return y, (mean, rstd, Cc)
        return y, (_StatPtr(ref, 0), _StatPtr(ref, 1), Cc)

    def _rows_z(self, cw: ConvW) -> int:
        """1 = the whole-chip small-M form (one K slice: no hand-off state) for a per-utterance linear whose K gives
        every wave the same K-step count, 0 = the tiled path -- a function of the weight's shape only (the native
        composite operators, csrc/abi_ops.hip, apply the same rule: bit-identical)."""
        nk = cw.ci_pad // 32
        return int(self.small_rows and nk % 4 == 0 and nk // 4 in (1, 2, 4, 8, 16))

    def _scratch(self, name, n, minimum=1 << 20):
        """fp32 scratch shared by consecutive launches of ONE branch (a conv's statistics partials, consumed by
        the finalize launch right behind it; the standalone statistics workspace).  Each forked branch has its
        own (key suffix self._branch): concurrent branches sharing one slab would race on the partials.  A
        grown slab's old storage is retired, not freed: launches already enqueued (or captured) on it --
        possibly on another stream -- still read it, and a freed block could be handed to another stream's
        allocation while they run.  minimum: the smallest storage (the shared slabs start at 4 MB so they rarely grow;
        the per-key deferred-statistics slabs are sized exactly -- a batch-1 partial is a few KB)."""
        key = name + self._branch
        t = self._bufs.get(key)
        if t is None or t.numel() < n:
            if t is not None:
                self._retired.append(t)
            t = self._bufs[key] = torch.empty(max(n, minimum), dtype=torch.float32, device=self.device)
        return t

    def _counters(self, name, n):
        """int32 hand-off counters of ONE branch, zero when allocated; every kernel that uses them leaves them zero
        (the split-K tile tickets).  Grown storages are retired, like _scratch."""
        key = name + self._branch
        t = self._bufs.get(key)
        if t is None or t.numel() < n:
            if t is not None:
                self._retired.append(t)
            t = self._bufs[key] = torch.zeros(max(n, 4096), dtype=torch.int32, device=self.device)
        return t

    def _slab(self, n):
        return self._scratch("stat_slab", n)

    def fork(self, site, *fns):
        """run fns[0] on the current stream and fns[1:] on side streams forked from it (waits on the current
        stream, joined back into it before returning); sequential unless branch_streams is on (True, or a set of
        fork sites holding `site`: "enc" = text || prompt encoder, "f0n" = F0 || N predictor branches, "src" =
        decoder pre-blocks || harmonic source).
        Forks nest: a fork inside a branch takes side streams and scratch keys of its own depth, so an inner
        branch never queues behind (or shares scratch with) an outer one.  -> outputs"""
        on = self.branch_streams is True or (isinstance(self.branch_streams, (set, frozenset)) and
                                             site in self.branch_streams)
        if not on or len(fns) < 2:
            return [f() for f in fns]
        cur = torch.cuda.current_stream(self.device)
        d, outer = self._depth, self._branch
        side = []
        for i in range(1, len(fns)):
            if (d, i) not in self._side:
                self._side[(d, i)] = torch.cuda.Stream(self.device)
            side.append(self._side[(d, i)])
        for st in side:
            st.wait_stream(cur)
        outs = []
        self._depth = d + 1
        try:
            for i, f in enumerate(fns):
                self._branch = outer if i == 0 else f"{outer}@b{d}.{i}"
                with torch.cuda.stream(cur if i == 0 else side[i - 1]):
                    outs.append(f())
        finally:
            self._branch, self._depth = outer, d
        for st in side:
            cur.wait_stream(st)
        return outs

    timer = None
    stage = ""  # label of the synth() stage being enqueued (set by the caller; recorded with each timed launch)

    def start_timer(self, tags):
        """record HIP events around every conv launch whose tag is in `tags` (same stream as the kernel); tags "*":
        every conv launch and every other launch whose algorithmic cost the engine models (attention, LSTM
        recurrences, LayerNorm rows, statistics, harmonic source, iSTFT)."""
        self.timer = dict(tags=set(tags) if tags != "*" else set(), all=tags == "*", rec=[])

    def stop_timer(self):
        """-> [(tag, seconds, FLOP, bytes, conv shape | None, stage)] of the recorded launches, in launch order."""
        tm, self.timer = self.timer, None
        torch.cuda.synchronize(self.device)
        return [(w, e0.elapsed_time(e1) * 1e-3, f, b, shp, stg) for (w, e0, e1, f, b, shp, stg) in tm["rec"]]

    def stats(self, x: Act, key):
        """InstanceNorm statistics of x over time -> (mean, rstd, stat_bs); with defer_stats and <= 8 256-row chunks
        only the partials pass runs here (the consuming conv's prologue, or the first other use, finalises)."""
        Cc = _rup(x.C, 8)
        mean = self.buf(key + ".m", (x.B, Cc), torch.float32)
        rstd = self.buf(key + ".r", (x.B, Cc), torch.float32)
        nch = (x.T + 255) // 256
        defer = self.defer_stats and nch <= 8
        nws = self.lib.stzs_chan_stats_workspace(x.B, x.T, Cc) // 4 + 1
        ws = self._scratch("stat_ws." + key, nws, 1024) if defer else self._scratch("stat_ws", nws)
        a = L.StatsArgs()
        a.x, a.mean, a.rstd, a.partial = x.ptr, mean.data_ptr(), rstd.data_ptr(), ws.data_ptr()
        a.ld, a.bs, a.stat_bs, a.B, a.T, a.C, a.dtype, a.eps = x.ld, x.bs, Cc, x.B, x.T, Cc, x.dt, 1e-5
        cost = (0, x.B * x.T * x.C * x.t.element_size())
        if not defer:
            self._call(self.lib.stzs_chan_stats, a, "chan_stats", cost=cost)
            return mean, rstd, Cc
        self._call(self.lib.stzs_chan_stats_partial, a, "chan_stats", cost=cost)
        ref = _StatsRef(self, ws, Cc, nch, x.T, x.B, mean, rstd, 256)
        return _StatPtr(ref, 0), _StatPtr(ref, 1), Cc

    def rowln(self, x: Act, y: Act, *, G=None, gs=0, Bt=None, bs=0, gdiv=1, gadd=1.0, act=L.ACT_NONE, slope=0.0,
              R=None, y_scale=None, what="rowln"):
        a = L.RowLNArgs()
        a.y_scale = y_scale.data_ptr() if y_scale is not None else None
        a.x, a.y, a.G, a.Bt = x.ptr, y.ptr, G, Bt
        a.ldx, a.ldy, a.gs, a.bs = x.ld, y.ld, gs, bs
        a.R = R if R is not None else x.B * x.T
        a.C, a.gdiv, a.in_dtype, a.out_dtype, a.act = x.C, gdiv, x.dt, y.dt, act
        a.gadd, a.eps, a.slope = gadd, 1e-5, slope
        assert x.ld * x.T == x.bs and y.ld * y.T == y.bs
        self._call(self.lib.stzs_row_layernorm, a, what, cost=_ln_cost(a))

    def quant(self, x: Act, y: Act, scale: torch.Tensor, what="quant"):
        """bf16 rows -> e4m3fn rows + per-row scale (stzs_quant_rows)."""
        a = L.QuantArgs()
        a.x, a.y, a.scale, a.ldx, a.ldy = x.ptr, y.ptr, scale.data_ptr(), x.ld, y.ld
        a.R, a.C = x.B * x.T, x.C
        assert x.ld * x.T == x.bs and y.ld * y.T == y.bs
        self._call(self.lib.stzs_quant_rows, a, what, cost=(0, a.R * a.C * (x.t.element_size() + 1)))

    def _attn_args(self, q: Act, k: Act, v: Act, o: Act):
        S = self.spec
        a = L.AttnArgs()
        a.q, a.k, a.v, a.o = q.ptr, k.ptr, v.ptr, o.ptr
        a.ldq, a.ldk, a.ldv, a.ldo = q.ld, k.ld, v.ld, o.ld
        a.bsq, a.bsk, a.bsv, a.bso = q.bs, k.bs, v.bs, o.bs
        a.R, a.Lq, a.Lk, a.heads, a.dh = q.B, q.T, k.T, S.dn_heads, S.dn_head_dim
        a.precise = int(q.t.dtype == torch.float32)  # fp32 operands: the fp32 attention kernel
        return a

    def attention(self, q: Act, k: Act, v: Act, o: Act):
        a = self._attn_args(q, k, v, o)
        self._call(self.lib.stzs_attention, a, "attention",
                   cost=(4.0 * a.R * a.heads * a.Lq * a.Lk * a.dh,
                         a.R * (2 * a.Lq + 2 * a.Lk) * a.heads * a.dh * q.t.element_size()))

    def lstm(self, lw, x: Act, y: Act, key):
        a, cost = self._lstm_args(lw, x, y, key)
        self._call(self.lib.stzs_lstm, a, key + ".rec", cost=cost)  # recurrent products + gate rows in, h rows out
        return y

    def lstm_pair(self, r0, r1):
        """two independent recurrences r = (lw, x, y, key) of one shape class in ONE launch (stzs_lstm_pair: side by
        side on the chip; each output the same bits as its own lstm() call): both input projections, then the
        paired recurrence on separate exchange state."""
        a0, c0 = self._lstm_args(*r0)
        a1, c1 = self._lstm_args(*r1, pair=True)
        self._call(self.lib.stzs_lstm_pair, a0, r0[3] + ".rec+" + r1[3] + ".rec",
                   cost=(c0[0] + c1[0], c0[1] + c1[1]), b=a1)
        return r0[2], r1[2]

    def _lstm_args(self, lw, x: Act, y: Act, key, pair=False):
        """input projection (one MFMA GEMM over all steps) + the recurrence's arguments -> (LstmArgs, cost)"""
        gx = self.act(key + ".gx", x.B, x.T, 8 * lw.H, torch.float32)
        self.conv(lw.ih, x, gx, what=key + ".ih")
        a = L.LstmArgs()
        a.gx, a.whhT, a.y = gx.ptr, self._t(lw.whhT).data_ptr(), y.ptr
        if lw.whx3 is not None:  # precise: split-operand recurrence, fp32 h out
            assert y.t.dtype == torch.float32
            a.whhT, a.precise = self._t(lw.whx3).data_ptr(), 1
        nx = self.lib.stzs_lstm_workspace(x.B, lw.H, 2)
        sk = self._branch + ("@pair" if pair else "")  # concurrent recurrences (branches, a pair) never share them
        xchg = self.buf("lstm.xchg" + sk, (max(nx, 16),), torch.uint8, zero=True)
        sync = self.buf("lstm.sync" + sk, (4096,), torch.uint8, zero=True)
        a.xchg, a.sync = xchg.data_ptr(), sync.data_ptr()
        a.ldg, a.bsg, a.ldy, a.bsy = gx.ld, gx.bs, y.ld, y.bs
        a.B, a.T, a.H, a.ndir = x.B, x.T, lw.H, 2
        a.status, a.spin_limit = self.status.data_ptr(), self.lstm_spin_limit
        # (flops, bytes): recurrent products; gate rows in, h rows out, W_hh once
        return a, (2.0 * x.B * x.T * 2 * 4 * lw.H * lw.H,
                   x.B * x.T * (8 * lw.H * 4 + 2 * lw.H * y.t.element_size()) + 2 * 4 * lw.H * lw.H * 2)

    def copy2d(self, x: Act, y: Act, R, Cn, bsx=None):
        a = L.CopyArgs()
        a.x, a.y, a.ldx, a.bsx, a.ldy, a.bsy = x.ptr, y.ptr, x.ld, x.bs if bsx is None else bsx, y.ld, y.bs
        a.B, a.R, a.C, a.in_dtype, a.out_dtype = y.B, R, Cn, x.dt, y.dt
        self._call(self.lib.stzs_copy2d, a, "copy2d")

    def mean_rows(self, x: torch.Tensor, c0, Cn, key):
        y = self.buf(key, (x.shape[0], Cn), torch.float32)
        self.launches += 1
        L.check(self.lib.stzs_mean_rows(x.data_ptr(), y.data_ptr(), x.shape[0], x.shape[1], x.shape[2],
                                        x.shape[1] * x.shape[2], c0, Cn, Cn, self.stream()), "mean_rows")
        return y

    # ------------------------------------------------------------------ front ends
    def text_encode(self, tokens: torch.Tensor) -> Act:
        """tokens int32 [B, T] (device) -> h_txt bf16 [B, T, d_txt] (StyleTTS2 TextEncoder):
        embedding gather, te_layers x (k5 conv on MFMA, LayerNorm + LeakyReLU 0.2), then the BiLSTM
        (input projection on MFMA + the register-resident exchange recurrence of csrc/lstm.hip)."""
        S, W = self.spec, self.W
        B, T = tokens.shape
        e = self.act("te.e", B, T, S.d_txt, self.adt)
        c = self.act("te.c", B, T, S.d_txt, self.adt)
        self.launches += 1
        emb = self.lib.stzs_embed_f32 if self.adt == torch.float32 else self.lib.stzs_embed
        L.check(emb(tokens.data_ptr(), W.t(W.te_emb).data_ptr(), e.ptr, B, T, S.d_txt, e.ld, self.stream()), "embed")
        for i in range(S.te_layers):
            self.conv(W.te_conv[i], e, c, pad=S.te_kernel // 2, splitk=0 if self.adt == torch.float32 else self.te_splitk,
                      what=f"te.conv{i}")
            g, b = W.te_ln[i]
            self.rowln(c, e, G=W.t(g).data_ptr(), gs=0, Bt=W.t(b).data_ptr(), bs=0, gadd=0.0,
                       act=L.ACT_LEAKY, slope=0.2, what=f"te.ln{i}")
        h = self.act("te.h", B, T, S.d_txt, self.adt)
        return self.lstm(W.te_lstm, e, h, "te.lstm")

    def log_mel(self, wav: torch.Tensor, dtype=torch.bfloat16) -> Act:
        """reference wav fp32 [B, N] (device) -> log-mel [B, N/hop + 1, n_mels]:
        windowed reflect-padded frames -> bf16 DFT GEMM on MFMA (cos | -sin basis, fp32 out) -> power, sparse
        mel filterbank, log (csrc/frontend.hip)."""
        S, W = self.spec, self.W
        B, N = wav.shape
        Fr = N // S.hop + 1
        dft = W.fe_dft
        frames = self.act("fe.frames", B, Fr, dft.ci_pad)
        a = L.FramesArgs()
        a.wav, a.window, a.y = wav.data_ptr(), W.t(W.fe_win).data_ptr(), frames.ptr
        a.ldw, a.ldy, a.bsy = N, frames.ld, frames.bs
        a.B, a.N, a.F, a.n_fft, a.win, a.hop = B, N, Fr, S.mel_nfft, S.mel_win, S.hop
        self._call(self.lib.stzs_stft_frames, a, "stft_frames")
        nbin = S.mel_nfft // 2 + 1
        spec = self.act("fe.spec", B, Fr, 2 * nbin, torch.float32)
        self.conv(dft, Act(frames.t, 0, S.mel_win), spec, what="fe.dft")
        mel = self.act("fe.mel", B, Fr, S.n_mels, dtype)
        a = L.LogMelArgs()
        a.spec, a.fb, a.ranges, a.y = spec.ptr, W.t(W.fe_fb).data_ptr(), W.t(W.fe_rng).data_ptr(), mel.ptr
        a.lds, a.bss, a.ldy, a.bsy = spec.ld, spec.bs, mel.ld, mel.bs
        a.B, a.F, a.nbin, a.n_mels, a.out_dtype = B, Fr, nbin, S.n_mels, mel.dt
        self._call(self.lib.stzs_log_mel, a, "log_mel")
        return mel

    def prompt_encode(self, ref_wav: torch.Tensor, prompt_idx: torch.Tensor = None) -> torch.Tensor:
        """reference-prompt front end on HIP: ref wav [B, N] -> DISCRETE style codes
        (README.md:5): log-mel -> 2 x (k5 conv + LeakyReLU 0.2) -> adaptive average pool to L_s rows ->
        projection -> product VQ (stzs_code_quantize).  Returns the dequantised codes fp32 [B, L_s, code];
        the indices stay in self.prompt_idx [B, L_s, G] (int32).  prompt_idx: teacher-forced indices (the
        front end is skipped, the codebook rows are gathered)."""
        S, W = self.spec, self.W
        G = S.code_dim // S.vq_group
        if prompt_idx is not None:
            B = prompt_idx.shape[0]
            idx = self.buf("prompt.idx", (B, S.L_s, G), torch.int32)
            idx.copy_(prompt_idx.to(torch.int32).reshape(B, S.L_s, G))
            out = self.buf("prompt", (B, S.L_s, S.code_dim), torch.float32)
            self.code_quantize(None, idx, out, lookup=True)
            self.prompt_idx = idx
            return out
        z = self.prompt_features(ref_wav)
        B = z.shape[0]
        idx = self.buf("prompt.idx", (B, S.L_s, G), torch.int32)
        out = self.buf("prompt", (B, S.L_s, S.code_dim), torch.float32)
        self.code_quantize(z, idx, out)
        self.prompt_idx = idx
        return out

    def code_quantize(self, z, idx: torch.Tensor, out: torch.Tensor, lookup=False):
        """product VQ of z fp32 [B, L, code] -> idx int32 [B, L, G] + dequantised rows out (lookup: idx given)."""
        S, W = self.spec, self.W
        a = L.VqArgs()
        a.x = z.data_ptr() if z is not None else None
        a.codebook, a.idx, a.y = W.t(W.pe_vq).data_ptr(), idx.data_ptr(), out.data_ptr()
        G = S.code_dim // S.vq_group
        a.ldx, a.ldi, a.ldy = S.code_dim, G, S.code_dim
        a.R, a.G, a.K, a.dg, a.lookup = idx.shape[0] * idx.shape[1], G, S.vq_size, S.vq_group, int(lookup)
        self._call(self.lib.stzs_code_quantize, a, "code_quantize")

    def prompt_features(self, ref_wav: torch.Tensor) -> torch.Tensor:
        """ref wav [B, N] -> continuous prompt codes fp32 [B, L_s, code] (before the quantiser)."""
        S, W = self.spec, self.W
        wav = ref_wav.to(self.device, torch.float32).contiguous()
        B = wav.shape[0]
        mel = self.log_mel(wav)
        Fr = mel.T
        c0 = self.act("fe.c0", B, Fr, S.pe_ch)
        c1 = self.act("fe.c1", B, Fr, S.pe_ch)
        self.conv(W.pe_conv0, mel, c0, pad=2, epi_act=L.ACT_LEAKY, epi_slope=0.2, what="pe.conv0")
        self.conv(W.pe_conv1, c0, c1, pad=2, epi_act=L.ACT_LEAKY, epi_slope=0.2, what="pe.conv1")
        pooled = self.act("fe.pool", B, S.L_s, S.pe_ch)
        a = L.PoolArgs()
        a.x, a.y, a.ldx, a.bsx, a.ldy, a.bsy = c1.ptr, pooled.ptr, c1.ld, c1.bs, pooled.ld, pooled.bs
        a.B, a.T, a.L, a.C, a.in_dtype, a.out_dtype = B, Fr, S.L_s, S.pe_ch, L.BF16, L.BF16
        self._call(self.lib.stzs_pool_rows, a, "pool_rows")
        out = self.buf("prompt.z", (B, S.L_s, S.code_dim), torch.float32)
        self.conv(W.pe_proj, pooled, Act(out), what="pe.proj")
        return out

    # ------------------------------------------------------------------ (a) style diffusion
    def sample_style(self, h_txt: Act, prompt: torch.Tensor, eps: torch.Tensor, steps: int,
                     cfg_scale: float = 1.0) -> torch.Tensor:
        """a1-a4: Euler sampling over the distilled / Karras sigma schedule with classifier-free guidance.
        h_txt [B, T, d_txt] bf16, prompt [B, L_s, code] fp32, eps [B, L_s, code] -> codes fp32 [B, L_s, code]."""
        S = self.spec
        B = h_txt.B
        cfg = cfg_scale != 1.0
        R = 2 * B if cfg else B
        sig = sigma_schedule(S, steps)
        if h_txt.t.dtype != self.sdt:  # (the long-form mode: precise fp32 text rows into the bf16 / fp8 sampler)
            hs = self.act("dn.h_txt", B, h_txt.T, h_txt.C, self.sdt)
            self.copy2d(h_txt, hs, h_txt.T, h_txt.C)
            h_txt = hs
        st = self.denoiser_prepare(h_txt, prompt, sig[:steps], cfg)
        x = self.buf("dn.x", (R, S.L_s, S.code_dim), torch.float32)
        N = S.L_s * S.code_dim
        self.launches += 1
        L.check(self.lib.stzs_state_init(x.data_ptr(), eps.data_ptr(), B, N, int(cfg), float(sig[0]), self.stream()),
                "state_init")
        D = self.act("dn.D", R, S.L_s, S.code_dim, torch.float32)
        for i in range(steps):
            self.denoiser_step(st, i, Act(x), D)
            self.launches += 1
            L.check(self.lib.stzs_cfg_euler(x.data_ptr(), D.t.data_ptr(), B, N, int(cfg), float(cfg_scale),
                                            float(sig[i]), float(sig[i + 1] - sig[i]), self.stream()), "cfg_euler")
        return x[:B]

    def denoiser_fwd(self, h_txt: Act, prompt: torch.Tensor, x: torch.Tensor, sigma: float, cfg: bool) -> torch.Tensor:
        """a2 alone: ONE preconditioned denoiser evaluation D(x, sigma) (EDM c_skip / c_out / c_in / c_noise) on the
        rows x [R, L_s, code] fp32 (R = 2B with CFG: conditional rows, then the null-prompt rows) -> D fp32
        [R, L_s, code] (a device buffer of the engine)."""
        S = self.spec
        st = self.denoiser_prepare(h_txt, prompt, [float(sigma)], cfg)
        D = self.act("dn.D", x.shape[0], S.L_s, S.code_dim, torch.float32)
        self.denoiser_step(st, 0, Act(x), D)
        return D.t

    def denoiser_prepare(self, h_txt: Act, prompt: torch.Tensor, sigmas, cfg: bool) -> dict:
        """step-invariant part of a sampling run: the cross-attention context [ctx_txt(h) ; ctx_prm(prompt | null)]
        and its per-layer K/V, the pooled prompt, and the conditioning of EVERY sigma at once (rows s * R + r):
        adaLN-single input, its two projections and the per-layer expansion -> 5 launches instead of 5 per NFE."""
        S, W = self.spec, self.W
        B, T = h_txt.B, h_txt.T
        R = 2 * B if cfg else B
        Ls, d, cd = S.L_s, S.dn_d, S.code_dim
        Lc = T + Ls
        steps = len(sigmas)
        ctx = self.act("dn.ctx", R, Lc, d, self.sdt)
        # ctx_txt rows: the conv writes T rows per utterance into a buffer of Lc rows per utterance
        self._conv_rows(W.dn_ctx_txt, h_txt, ctx.t, 0, 0, "dn.ctx_txt")
        pa = Act(prompt)
        self._conv_rows(W.dn_ctx_prm, pa, ctx.t, 0, T, "dn.ctx_prm")
        if cfg:
            self._conv_rows(W.dn_ctx_txt, h_txt, ctx.t, B, 0, "dn.ctx_txt.u")
            f32 = self.sdt == torch.float32
            nul = Act(W.t(W.dn_ctx_null32 if f32 else W.dn_ctx_null)[None])
            dst = Act(ctx.t[B:]).rows(0, B)
            a = L.CopyArgs()
            a.x, a.y = nul.ptr, dst.t.data_ptr() + T * ctx.ld * ctx.t.element_size()
            a.ldx, a.bsx, a.ldy, a.bsy = d, 0, ctx.ld, Lc * ctx.ld
            a.B, a.R, a.C, a.in_dtype, a.out_dtype = B, Ls, d, nul.dt, ctx.dt
            self._call(self.lib.stzs_copy2d, a, "ctx_null")
        pm = self.mean_rows(prompt, 0, cd, "dn.pm")
        pool = self.buf("dn.pool", (R, d), torch.float32)
        self.conv(W.dn_pool, Act(pm[:, None]), Act(pool[:B, None]), rows=self._rows_z(W.dn_pool), what="dn.pool")
        if cfg:
            a = L.CopyArgs()
            a.x, a.y = W.t(W.dn_pool_null).data_ptr(), pool[B:].data_ptr()
            a.ldx, a.bsx, a.ldy, a.bsy = d, 0, d, d
            a.B, a.R, a.C, a.in_dtype, a.out_dtype = B, 1, d, L.F32, L.F32
            self._call(self.lib.stzs_copy2d, a, "pool_null")
        kv = []
        if getattr(W, "dn_kv_all", None) is not None and self.kv_fuse:
            # (r06) all layers' K / V of the shared context in one linear (weights.py dn_kv_all); layer l's [K | V] are
            # channels [2 d l, 2 d (l + 1)) of its rows
            nl = len(W.dn_layers)
            kva = self.act("dn.kv_all", R, Lc, 2 * d * nl, self.sdt)
            self.conv(W.dn_kv_all, ctx, kva, what="dn.kv")
            kv = [Act(kva.t, 2 * d * l, 2 * d) for l in range(nl)]
        else:
            for l, lw in enumerate(W.dn_layers):
                kvl = self.act(f"dn.kv{l}", R, Lc, 2 * d, self.sdt)
                self.conv(lw["kv"], ctx, kvl, what=f"dn.kv{l}")
                kv.append(kvl)
        # sigma embeddings for all steps
        fkey = ("dn.four", tuple(float(v) for v in sigmas))
        fo = self._consts.get(fkey)
        if fo is None:  # host constant, uploaded once (never inside a graph capture)
            four = np.stack([fourier_features(S, edm_coeffs(S, v)["c_noise"]) for v in sigmas])
            fo = self._consts[fkey] = torch.from_numpy(four)[None].to(self.device)
        t0 = self.act("dn.t0", 1, steps, d, torch.float32)
        temb = self.act("dn.temb", 1, steps, d, torch.float32)
        self.conv(W.dn_t0, Act(fo), t0, epi_act=L.ACT_SILU, rows=self._rows_z(W.dn_t0), what="dn.t0")
        self.conv(W.dn_t1, t0, temb, rows=self._rows_z(W.dn_t1), what="dn.t1")
        cb = self.buf("dn.cb", (steps * R, d), self.sdt)
        mod = self.buf("dn.mod", (steps * R, 6 * d), torch.float32)
        fmod = self.buf("dn.fmod", (steps * R, 2 * d), torch.float32)
        modx = self.buf("dn.modx", (S.dn_layers, steps * R, 6 * d), torch.float32)
        fmodx = self.buf("dn.fmodx", (1, steps * R, 2 * d), torch.float32)
        self.launches += 1
        cond = self.lib.stzs_dn_cond_steps_f32 if cb.dtype == torch.float32 else self.lib.stzs_dn_cond_steps
        L.check(cond(pool.data_ptr(), temb.t.data_ptr(), cb.data_ptr(), R, d, steps, self.stream()), "dn_cond_steps")
        self.conv(W.dn_ada, Act(cb[:, None]), Act(mod[:, None]), what="dn.ada")
        self.conv(W.dn_final_ada, Act(cb[:, None]), Act(fmod[:, None]), what="dn.final_ada")
        self.launches += 2
        L.check(self.lib.stzs_adaln_expand(mod.data_ptr(), W.t(W.dn_table).data_ptr(), modx.data_ptr(), steps * R, d,
                                           6, S.dn_layers, 0b010010, self.stream()), "adaln_expand")
        L.check(self.lib.stzs_adaln_expand(fmod.data_ptr(), None, fmodx.data_ptr(), steps * R, d, 2, 1, 0b10,
                                           self.stream()), "adaln_expand.f")
        return dict(R=R, sig=list(sigmas), kv=kv, modx=modx, fmodx=fmodx)

    def denoiser_step(self, st: dict, i: int, xa: Act, D: Act):
        """one NFE: D = c_skip x + c_out F(c_in x, sigma_i) for the R rows of xa, with the conditioning prepared
        by denoiser_prepare (6 layers: adaLN-modulated self-attention, cross-attention, GELU FFN)."""
        S, W = self.spec, self.W
        R, kv, modx, fmodx = st["R"], st["kv"], st["modx"], st["fmodx"]
        Ls, d = S.L_s, S.dn_d
        h = self.act("dn.h", R, Ls, d, torch.float32)
        an = self.act("dn.a", R, Ls, d, self.sdt)
        qkv = self.act("dn.qkv", R, Ls, 3 * d, self.sdt)
        o = self.act("dn.o", R, Ls, d, self.sdt)
        q = self.act("dn.q", R, Ls, d, self.sdt)
        ff = self.act("dn.ff", R, Ls, S.dn_ffn, self.sdt)
        pos = Act(W.t(W.dn_pos)[None])
        fsz = 4
        f8 = self.fp8_denoiser
        if f8:  # e4m3fn operand rows + per-row scales for the layer linears
            an8 = self.act("dn.a8", R, Ls, d, torch.float8_e4m3fn)
            o8 = self.act("dn.o8", R, Ls, d, torch.float8_e4m3fn)
            ff8 = self.act("dn.ff8", R, Ls, S.dn_ffn, torch.float8_e4m3fn)
            s_an = self.buf("dn.a8s", (R * Ls,), torch.float32)
            s_o = self.buf("dn.o8s", (R * Ls,), torch.float32)
            s_ff = self.buf("dn.ff8s", (R * Ls,), torch.float32)
        co = edm_coeffs(S, st["sig"][i])
        rk = {} if (f8 or self.sdt == torch.float32) else self.dn_rows
        if f8:
            ain, sin, sfx = an8, s_an, "8"
        else:
            ain, sin, sfx = an, None, ""
        # adaLN / LayerNorm rows of this step: ln1_l, ca_ln_l, ln2_l for every layer, then lnf; each one
        # after the first is launched right behind the residual linear that produces its input (post_ln), or on the
        # rows form runs inside the linear that reads it (pre_ln, stzs_ln_linear).
        # (Fusing them into that linear's epilogue -- last-arriving tile of a row block, sc1 hand-off --
        # was tried: bit-identical but 1.6x slower at batch 1, the block's rows then normalise on one CU.)
        lns = []
        for l, lw in enumerate(W.dn_layers):
            mb = modx[l, i * R].data_ptr()  # this step's rows of layer l's modulation
            lns.append(self._ln_args(h, ain, G=mb + d * fsz, gs=6 * d, Bt=mb, bs=6 * d, gdiv=Ls, y_scale=sin))
            lns.append(self._ln_args(h, ain, G=W.t(lw["ln_g"]).data_ptr(), Bt=W.t(lw["ln_b"]).data_ptr(),
                                     y_scale=sin))
            lns.append(self._ln_args(h, ain, G=mb + 4 * d * fsz, gs=6 * d, Bt=mb + 3 * d * fsz, bs=6 * d, gdiv=Ls,
                                     y_scale=sin))
        fb = fmodx[0, i * R].data_ptr()
        lns.append(self._ln_args(h, an, G=fb + d * fsz, gs=2 * d, Bt=fb, bs=2 * d, gdiv=Ls))
        # on the rows form each LayerNorm runs inside the linear that reads it (pre_ln) instead of behind its producer
        fl = bool(rk) and self.ln_fuse
        post = lambda k: None if fl else lns[k]
        pre = lambda k: lns[k] if fl else None
        self.conv(W.dn_in, xa, h, cscale=co["c_in"], res=pos, rows=rk.get("inp", 0), post_ln=post(0), what="dn.in")
        sk = {} if (f8 or self.sdt == torch.float32) else self.dn_splitk
        for l, lw in enumerate(W.dn_layers):
            mb = modx[l, i * R].data_ptr()
            self.conv(lw["qkv" + sfx], ain, qkv, x_scale=sin, splitk=sk.get("qkv", 0), rows=rk.get("qkv", 0),
                      pre_ln=pre(3 * l), attn=(qkv.sl(0, d), qkv.sl(d, d), qkv.sl(2 * d, d), o), what="qkv")
            xo, so = (o8, s_o) if f8 else (o, None)
            if f8:
                self.quant(o, o8, s_o)
            self.conv(lw["o" + sfx], xo, h, res=h, gate=mb + 2 * d * fsz, gate_bs=6 * d, x_scale=so,
                      post_ln=post(3 * l + 1), splitk=sk.get("o", 0), rows=rk.get("o", 0), what="sa_o")
            self.conv(lw["q" + sfx], ain, q, x_scale=sin, splitk=sk.get("q", 0), rows=rk.get("q", 0),
                      pre_ln=pre(3 * l + 1), attn=(q, kv[l].sl(0, d), kv[l].sl(d, d), o), what="ca_q")
            if f8:
                self.quant(o, o8, s_o)
            self.conv(lw["co" + sfx], xo, h, res=h, x_scale=so, post_ln=post(3 * l + 2), splitk=sk.get("co", 0),
                      rows=rk.get("co", 0), what="ca_o")
            self.conv(lw["ff1" + sfx], ain, ff, epi_act=L.ACT_GELU, x_scale=sin, splitk=sk.get("ff1", 0),
                      rows=rk.get("ff1", 0), pre_ln=pre(3 * l + 2), what="ff1")
            xf, sf = (ff8, s_ff) if f8 else (ff, None)
            if f8:
                self.quant(ff, ff8, s_ff)
            self.conv(lw["ff2" + sfx], xf, h, res=h, gate=mb + 5 * d * fsz, gate_bs=6 * d, x_scale=sf,
                      post_ln=post(3 * l + 3), splitk=sk.get("ff2", 0), rows=rk.get("ff2", 0), what="ff2")
        self.conv(W.dn_out, an, D, alpha=co["c_out"], acc_in=xa, beta=co["c_skip"], rows=rk.get("out", 0),
                  pre_ln=pre(len(lns) - 1), what="dn.out")

    def _ln_args(self, x: Act, y: Act, *, G=None, gs=0, Bt=None, bs=0, gdiv=1, gadd=0.0, y_scale=None):
        """stzs_rowln_args of a modulated LayerNorm x -> y (launched by stzs_row_layernorm behind the linear that
        produces x: conv(post_ln=...))."""
        a = L.RowLNArgs()
        a.x, a.y, a.G, a.Bt = x.ptr, y.ptr, G, Bt
        a.ldx, a.ldy, a.gs, a.bs = x.ld, y.ld, gs, bs
        a.R, a.C, a.gdiv, a.in_dtype, a.out_dtype, a.act = x.B * x.T, x.C, gdiv, x.dt, y.dt, L.ACT_NONE
        a.gadd, a.eps, a.slope = gadd, 1e-5, 0.0
        a.y_scale = y_scale.data_ptr() if y_scale is not None else None
        return a

    def _conv_rows(self, cw, x: Act, dst: torch.Tensor, b0, t0, what):
        """linear over x [B, T, C] written to dst[b0 + b, t0 + t, :] (dst rows have a larger T)."""
        B, T = x.B, x.T
        y = Act(dst[b0:b0 + B])
        a_y = Act(y.t, 0, cw.Co)
        # shift the output base by t0 rows; the batch stride stays that of dst
        view = _OffsetAct(a_y, t0 * dst.shape[2])
        self.conv(cw, x, view, T_out=T, what=what)

    # ------------------------------------------------------------------ (b) prosody predictor
    def predict_prosody(self, h_txt: Act, codes: torch.Tensor, durations=None, n_frames=None):
        """durations: optional int tensor [B, T_txt] (host or device); n_frames: their per-utterance sum if
        known (avoids the device->host sync, e.g. under graph capture).  Returns dict of device tensors."""
        if self.dur_overlap and durations is not None and (n_frames is not None or durations.device.type == "cpu"):
            # the alignment reads the given durations, so the duration LSTM no longer gates the frame branch: it
            # runs in ONE launch with the shared F0/N LSTM (stzs_lstm_pair), its projection and the durations kernel
            # after the F0/N branches -- every output the same bits as the sequential order
            d, ov = self.duration_encoder(h_txt, codes, durations)
            if n_frames is not None:
                T40 = int(n_frames)
            else:
                tot = durations.to(torch.int64).sum(1)
                assert int(tot.min()) == int(tot.max()), \
                    "one batch must share its total frame count (stzs.scheduler.BucketScheduler groups by it)"
                T40 = int(tot[0])
            pro = self.prosody_frames(h_txt, codes, d, ov, T40, pair_dur=True)
            du = self.duration_head(d, ov, hd=pro.pop("_hd"))
            pro.update(du, dur=du["dur"])
            return pro
        du = self.predict_durations(h_txt, codes, durations)
        if n_frames is not None:
            T40 = int(n_frames)
        else:
            if durations is not None and durations.device.type == "cpu":
                tot = durations.to(torch.int64).sum(1)
            else:
                tot = du["dur"].to(torch.int64).sum(1).cpu()  # host sync: the frame count sizes every later buffer
            assert int(tot.min()) == int(tot.max()), \
                "one batch must share its total frame count (stzs.scheduler.BucketScheduler groups by it)"
            T40 = int(tot[0])
        return self.prosody_frames(h_txt, codes, du["d"], du["dur"], T40, du)

    def predict_durations(self, h_txt: Act, codes: torch.Tensor, durations=None) -> dict:
        """a5-a6: DurationEncoder + duration LSTM + head -> dict(dur int32 [B, T], dsum, logits, d) (device)."""
        d, ov = self.duration_encoder(h_txt, codes, durations)
        return self.duration_head(d, ov)

    def duration_encoder(self, h_txt: Act, codes: torch.Tensor, durations=None):
        """a5: DurationEncoder (LSTM + AdaLN layers) -> (d [B, T, pr_in], the given durations as an int32 device
        tensor -- the caller's own when it is one (contiguous [B, T]: read in place, stream-ordered), else the copy
        pr.dur_ov -- or None)."""
        S, W = self.spec, self.W
        B, T = h_txt.B, h_txt.T
        pin = S.pr_in
        xin = self.act("pr.xin", B, T, pin, self.adt)
        assert h_txt.t.dtype == self.adt
        a = L.PrPrepArgs()
        a.codes, a.h, a.y = codes.data_ptr(), h_txt.ptr, xin.ptr
        a.ldc, a.bsc, a.ldh, a.bsh, a.ldy, a.bsy = codes.shape[2], codes.shape[1] * codes.shape[2], h_txt.ld, \
            h_txt.bs, xin.ld, xin.bs
        a.B, a.L, a.T, a.c0, a.Cs, a.Ch, a.yc0 = B, S.L_s, T, S.style_ac, S.style_pr, S.d_txt, S.d_txt
        a.f32 = int(self.adt == torch.float32)
        self._call(self.lib.stzs_predictor_prep, a, "pr_prep")
        hout = self.act("pr.hout", B, T, S.pr_hid, self.adt)
        nl = S.pr_layers
        if getattr(W, "pr_aln_all", None) is not None and self.kv_fuse:
            # (r06) every layer's AdaLN gamma / beta from the style columns (never rewritten by the layers: d_txt ==
            # pr_hid) in one stacked linear, layer i's at channels [2 pr_hid i, 2 pr_hid (i + 1))
            gb = self.act("pr.gb_all", B, T, 2 * S.pr_hid * nl, torch.float32)
            self.conv(W.pr_aln_all, xin.sl(S.d_txt, S.style_pr), gb, what="pr.aln")
            g_at, gs = (lambda i: gb.ptr + 2 * S.pr_hid * i * 4), 2 * S.pr_hid * nl
        else:
            gb = self.act("pr.gb", B, T, 2 * S.pr_hid, torch.float32)
            g_at, gs = (lambda i: gb.ptr), 2 * S.pr_hid
        for i in range(nl):
            self.lstm(W.pr_de[i], xin, hout, f"pr.de{i}")
            if gs == 2 * S.pr_hid:
                self.conv(W.pr_aln[i], xin.sl(S.d_txt, S.style_pr), gb, what=f"pr.aln{i}")
            self.rowln(hout, Act(xin.t, 0, S.pr_hid), G=g_at(i), gs=gs, Bt=g_at(i) + S.pr_hid * 4,
                       bs=gs, gdiv=1, gadd=1.0, what=f"pr.adaln{i}")
        ov = None
        if durations is not None:
            if (durations.device.type != "cpu" and durations.dtype == torch.int32 and durations.is_contiguous() and
                    tuple(durations.shape) == (B, T)):
                ov = durations  # (read only by the alignment and the durations kernel: no device copy, r06)
            else:
                ov = self.buf("pr.dur_ov", (B, T), torch.int32)
                if durations.device.type == "cpu":
                    ov.copy_(durations.to(torch.int32))
                elif durations.data_ptr() != ov.data_ptr():
                    ov.copy_(durations)
        return xin, ov

    def duration_head(self, d: Act, ov=None, hd: Act = None) -> dict:
        """a6: duration LSTM + projection + durations kernel (sum of the bin sigmoids, rounded, >= 1; the given
        durations `ov` override it); hd: the duration LSTM's output when already run (lstm_pair)
        -> dict(dur int32 [B, T], dsum, logits, d)."""
        S, W = self.spec, self.W
        B, T = d.B, d.T
        if hd is None:
            hd = self.act("pr.hd", B, T, S.pr_hid, self.adt)
            self.lstm(W.pr_dur_lstm, d, hd, "pr.dur_lstm")
        logits = self.act("pr.logits", B, T, S.dur_bins, torch.float32)
        self.conv(W.pr_dur_proj, hd, Act(logits.t, 0, S.dur_bins), what="pr.dur_proj")
        dur = self.buf("pr.dur", (B, T), torch.int32)
        dsum = self.buf("pr.dsum", (B, T), torch.float32)
        a = L.DurArgs()
        a.logits, a.override_dur, a.dur, a.dsum = logits.ptr, (ov.data_ptr() if ov is not None else None), \
            dur.data_ptr(), dsum.data_ptr()
        a.ldl, a.bsl, a.B, a.T, a.nbins = logits.ld, logits.bs, B, T, S.dur_bins
        self._call(self.lib.stzs_durations, a, "durations")
        return dict(dur=dur, dsum=dsum, logits=logits, d=d)

    def prosody_frames(self, h_txt: Act, codes: torch.Tensor, d: Act, dur: torch.Tensor, T40: int,
                       extra: dict = None, pair_dur=False) -> dict:
        """a7-a8 for a batch sharing T40 aligned frames: alignment, gathers, shared LSTM, F0 / N curves.
        pair_dur: the duration LSTM over d runs in the shared LSTM's launch (its output as "_hd")."""
        S, W = self.spec, self.W
        B, T = h_txt.B, h_txt.T
        pin = S.pr_in
        idx = self.buf("pr.idx", (B, T40), torch.int32)
        total = self.buf("pr.total", (B,), torch.int32)
        a = L.AlignArgs()
        a.dur, a.idx, a.total, a.B, a.T, a.T40 = dur.data_ptr(), idx.data_ptr(), total.data_ptr(), B, T, T40
        self._call(self.lib.stzs_alignment, a, "alignment")
        en = self.act("pr.en", B, T40, pin, self.adt)
        self.gather(d, idx, en, pin)
        enc_in = self.act("dec.enc_in", B, T40, S.d_txt + 2, self.dec_dt)
        if h_txt.t.dtype != enc_in.t.dtype:  # precise decoder on bf16 text rows: gather, then widen to fp32
            e16 = self.act("dec.enc_in16", B, T40, S.d_txt)
            self.gather(h_txt, idx, e16, S.d_txt)
            self.copy2d(e16, enc_in, T40, S.d_txt)
        else:
            self.gather(h_txt, idx, enc_in, S.d_txt)
        hd = self.act("pr.hd", B, T, S.pr_hid, self.adt) if pair_dur else None
        F0, Nn = self.f0n_predictor(en, codes, dur_rec=(W.pr_dur_lstm, d, hd, "pr.dur_lstm") if pair_dur else None)
        out = dict(extra or {}, dur=dur, idx=idx, T40=T40, en=en, asr_buf=enc_in, d=d, F0=F0, N=Nn)
        if pair_dur:
            out["_hd"] = hd
        return out

    def f0n_predictor(self, en: Act, codes: torch.Tensor, dur_rec=None):
        """a8: shared BiLSTM over the aligned frames, then per branch (F0, N) three AdaIN residual blocks (the
        middle one x2 upsampling) and a 1x1 projection.  en [B, T40, pr_in] bf16 -> F0, N fp32 [B, 2 T40]."""
        S, W = self.spec, self.W
        B, T40 = en.B, en.T
        xs = self.act("pr.xs", B, T40, S.pr_hid, self.adt)
        if dur_rec is None:
            self.lstm(W.pr_shared, en, xs, "pr.shared")
        else:  # dur_rec = (lw, x, y, key): the duration LSTM beside it, one launch
            self.lstm_pair((W.pr_shared, en, xs, "pr.shared"), dur_rec)
        sg = self.mean_rows(codes, S.style_ac, S.style_pr, "pr.sg")
        ng = W.pr_norm
        gbp = self.buf("pr.gbn", (B, ng.total), torch.float32)
        self.conv(ng.lin, Act(sg[:, None]), Act(gbp[:, None]), rows=self._rows_z(ng.lin), what="pr.norms")
        T80 = 2 * T40
        F0 = self.buf("pr.F0", (B, T80, 1), torch.float32)
        Nn = self.buf("pr.N", (B, T80, 1), torch.float32)
        c0, c1, c2 = S.f0n_ch

        s0 = self.stats(xs, "pr.xs.s1")  # (both branches' first AdaIN normalise xs: its statistics once, r06)
        bs = self.branch_streams
        forked = bs is True or (isinstance(bs, (set, frozenset)) and "f0n" in bs)
        if self.f0n_pair and self.blk_splitk and not forked:
            # (r06) the two branches in lockstep, each block's two convs of both branches as one launch pair
            # (stzs_conv1d_group -> conv_mfma_pair / splitk_epi_pair): same bits as branch after branch
            ys = {br: (self.act(f"pr.{br}.y0", B, T40, c0, self.adt), self.act(f"pr.{br}.y1", B, T80, c1, self.adt),
                       self.act(f"pr.{br}.y2", B, T80, c2, self.adt)) for br in ("f0", "n")}
            ins = {"f0": xs, "n": xs}
            for i in range(3):
                self._blk_pair([(W.pr_blk[f"pr.{br}{i}"], ins[br], ys[br][i], f"pr.{br}{i}", s0 if i == 0 else None)
                                for br in ("f0", "n")], ng, gbp, self.adt)
                ins = {br: ys[br][i] for br in ("f0", "n")}
            for br, out in (("f0", F0), ("n", Nn)):
                self.conv(W.pr_blk[f"pr.{br}_proj"], ys[br][2], Act(out, 0, 1), what=f"pr.{br}_proj")
            return F0[:, :, 0], Nn[:, :, 0]

        def branch(br, out):
            y0 = self.act(f"pr.{br}.y0", B, T40, c0, self.adt)
            y1 = self.act(f"pr.{br}.y1", B, T80, c1, self.adt)
            y2 = self.act(f"pr.{br}.y2", B, T80, c2, self.adt)
            self.blk(W.pr_blk[f"pr.{br}0"], xs, y0, ng, gbp, f"pr.{br}0", self.adt, s1=s0)
            self.blk(W.pr_blk[f"pr.{br}1"], y0, y1, ng, gbp, f"pr.{br}1", self.adt)
            self.blk(W.pr_blk[f"pr.{br}2"], y1, y2, ng, gbp, f"pr.{br}2", self.adt)
            self.conv(W.pr_blk[f"pr.{br}_proj"], y2, Act(out, 0, 1), what=f"pr.{br}_proj")
        self.fork("f0n", lambda: branch("f0", F0), lambda: branch("n", Nn))
        return F0[:, :, 0], Nn[:, :, 0]

    def gather(self, x: Act, idx, y: Act, Cn):
        a = L.GatherArgs()
        a.x, a.idx, a.y = x.t.data_ptr(), idx.data_ptr(), y.t.data_ptr()
        a.ldx, a.bsx, a.ldy, a.bsy = x.ld, x.bs, y.ld, y.bs
        a.B, a.Tsrc, a.Tdst, a.C, a.xc0, a.yc0, a.dtype = x.B, x.T, y.T, Cn, x.c0, y.c0, x.dt
        self._call(self.lib.stzs_gather_rows, a, "gather")

    def blk(self, bw, x: Act, out: Act, ng, gb: torch.Tensor, key, dt=torch.bfloat16, s1=None):
        """AdainResBlk1d: out = (conv2(act(AdaIN(conv1(up(act(AdaIN(x))))))) + sc(x)) / sqrt 2.
        s1: x's statistics when the caller already has them (self.stats(x, ...))."""
        B, T = x.B, x.T
        off1, n1 = ng.offsets[bw.name + ".norm1"]
        off2, n2 = ng.offsets[bw.name + ".norm2"]
        gbase, gbs = gb.data_ptr(), ng.total
        m1, r1, sb1 = s1 if s1 is not None else self.stats(x, key + ".s1")
        # batch-1 engine: the generic-layout copies split-K (blk_splitk), else the register-direct convs
        sk = self.blk_splitk if dt == torch.bfloat16 else 0
        c1 = bw.conv1s if (sk and bw.conv1s is not None) else bw.conv1
        c2 = bw.conv2s if (sk and bw.conv2s is not None) else bw.conv2
        To = 2 * T if bw.up else T
        r = self.act(key + ".r", B, To, bw.dout, dt)
        if bw.up:
            u = self.act(key + ".u", B, To, bw.din, dt)
            a = L.DwupArgs()
            a.x, a.y, a.mean, a.rstd, a.gb = x.ptr, u.ptr, m1.data_ptr(), r1.data_ptr(), gbase + off1 * 4
            a.w, a.wb = self.W.t(bw.pool_w).data_ptr(), self.W.t(bw.pool_b).data_ptr()
            a.ldx, a.bsx, a.ldy, a.bsy, a.stat_bs, a.gb_bs, a.gb_beta_off = x.ld, x.bs, u.ld, u.bs, sb1, gbs, n1
            a.B, a.T, a.C, a.slope, a.dtype = B, T, bw.din, 0.2, x.dt
            self._call(self.lib.stzs_adain_dwup, a, key + ".dwup")
            _, (m2, r2, sb2) = self.conv(c1, u, r, pad=1, stats_key=key + ".s2", splitk=sk, what=key + ".conv1")
        else:
            _, (m2, r2, sb2) = self.conv(c1, x, r, pad=1, pro=(m1, r1, sb1, gbase + off1 * 4, gbs, n1),
                                         pro_act=L.ACT_LEAKY, pro_slope=0.2, stats_key=key + ".s2", splitk=sk,
                                         what=key + ".conv1")
        if bw.sc is not None:
            scb = self.act(key + ".sc", B, T, bw.dout, dt)
            self.conv(bw.scs if (sk and bw.scs is not None) else bw.sc, x, scb, splitk=sk, what=key + ".sc")
            res = scb
        else:
            res = x
        self.conv(c2, r, out, pad=1, pro=(m2, r2, sb2, gbase + off2 * 4, gbs, n2), pro_act=L.ACT_LEAKY,
                  pro_slope=0.2, res=res, res_tdiv=2 if bw.up else 1, alpha=1.0 / math.sqrt(2.0), splitk=sk,
                  what=key + ".conv2")
        return out

    def _blk_pair(self, items, ng, gb: torch.Tensor, dt):
        """blk() for two independent blocks of the same shape (items: (bw, x, out, key, s1) each), advanced side by
        side: statistics, upsampling and shortcuts one block after the other, each conv pair collected into one
        stzs_conv1d_group call (the library pairs the batch-1 DEEP split-K convs, else runs them in turn)."""
        gbase, gbs = gb.data_ptr(), ng.total
        sk = self.blk_splitk if dt == torch.bfloat16 else 0
        st = []
        for bw, x, out, key, s1 in items:
            m1, r1, sb1 = s1 if s1 is not None else self.stats(x, key + ".s1")
            st.append((m1, r1, sb1))
        refs = [m.ref for m, _, _ in st if isinstance(m, _StatPtr) and not m.ref.done]
        if len(refs) == len(items) and len({id(r) for r in refs}) == len(refs) and all(it[0].up for it in items):
            self._finalize_group(refs)  # (the upsampling blocks' dwup reads mean / rstd: both finalised in one launch)
        grp, st2, rs = [], [], []
        for (bw, x, out, key, _), (m1, r1, sb1) in zip(items, st):
            off1, n1 = ng.offsets[bw.name + ".norm1"]
            c1 = bw.conv1s if (sk and bw.conv1s is not None) else bw.conv1
            To = 2 * x.T if bw.up else x.T
            r = self.act(key + ".r", x.B, To, bw.dout, dt)
            rs.append(r)
            if bw.up:
                u = self.act(key + ".u", x.B, To, bw.din, dt)
                a = L.DwupArgs()
                a.x, a.y, a.mean, a.rstd, a.gb = x.ptr, u.ptr, m1.data_ptr(), r1.data_ptr(), gbase + off1 * 4
                a.w, a.wb = self.W.t(bw.pool_w).data_ptr(), self.W.t(bw.pool_b).data_ptr()
                a.ldx, a.bsx, a.ldy, a.bsy, a.stat_bs, a.gb_bs, a.gb_beta_off = x.ld, x.bs, u.ld, u.bs, sb1, gbs, n1
                a.B, a.T, a.C, a.slope, a.dtype = x.B, x.T, bw.din, 0.2, x.dt
                self._call(self.lib.stzs_adain_dwup, a, key + ".dwup")
                _, s2 = self.conv(c1, u, r, pad=1, stats_key=key + ".s2", splitk=sk, collect=grp, what=key + ".conv1")
            else:
                _, s2 = self.conv(c1, x, r, pad=1, pro=(m1, r1, sb1, gbase + off1 * 4, gbs, n1), pro_act=L.ACT_LEAKY,
                                  pro_slope=0.2, stats_key=key + ".s2", splitk=sk, collect=grp, what=key + ".conv1")
            st2.append(s2)
        self._launch_group(grp, "blk.conv1")
        res = []
        for bw, x, out, key, _ in items:
            if bw.sc is not None:
                scb = self.act(key + ".sc", x.B, x.T, bw.dout, dt)
                self.conv(bw.scs if (sk and bw.scs is not None) else bw.sc, x, scb, splitk=sk, what=key + ".sc")
                res.append(scb)
            else:
                res.append(x)
        grp = []
        for (bw, x, out, key, _), (m2, r2, sb2), r, rr in zip(items, st2, rs, res):
            off2, n2 = ng.offsets[bw.name + ".norm2"]
            c2 = bw.conv2s if (sk and bw.conv2s is not None) else bw.conv2
            self.conv(c2, r, out, pad=1, pro=(m2, r2, sb2, gbase + off2 * 4, gbs, n2), pro_act=L.ACT_LEAKY,
                      pro_slope=0.2, res=rr, res_tdiv=2 if bw.up else 1, alpha=1.0 / math.sqrt(2.0), splitk=sk,
                      collect=grp, what=key + ".conv2")
        self._launch_group(grp, "blk.conv2")

    # ------------------------------------------------------------------ (c) decoder
    def decode(self, pro: dict, codes: torch.Tensor, seeds, istft=True) -> torch.Tensor:
        """a9-a13: decoder pre-blocks, generator, conv_post + iSTFT.  pro: asr_buf (aligned text features in the
        decoder input buffer), F0 / N [B, T80], T40 -> wav fp32 [B, 600 T40] (or conv_post rows, istft=False)."""
        # the harmonic source depends on F0 only: forkable beside the decoder pre-blocks (fork site "src")
        (gen_in, gbd), har = self.fork("src", lambda: self.decoder_pre(pro, codes),
                                       lambda: self.sine_gen(pro["F0"], seeds))
        return self.generator(gen_in, pro["F0"], seeds, gbd, istft=istft, har=har)

    def dec_style(self, codes: torch.Tensor) -> torch.Tensor:
        """every AdaIN gamma / beta of the decoder from the pooled acoustic codes: ONE GEMM -> [B, total] fp32."""
        S, W = self.spec, self.W
        B = codes.shape[0]
        sa = self.mean_rows(codes, 0, S.style_ac, "dec.sa")
        ng = W.dec_norm
        gbd = self.buf("dec.gbn", (B, ng.total), torch.float32)
        self.conv(ng.lin, Act(sa[:, None]), Act(gbd[:, None]), rows=self._rows_z(ng.lin), what="dec.norms")
        return gbd

    def decoder_pre(self, pro: dict, codes: torch.Tensor):
        """a9: F0 / N stride-2 convs, asr_res, the encode block and the four decode blocks (1024 channels,
        the last one x2 upsampling) -> (generator input [B, T80, dec_out], decoder AdaIN gammas/betas)."""
        S, W = self.spec, self.W
        enc_in, F0, Nn, T40 = pro["asr_buf"], pro["F0"], pro["N"], pro["T40"]
        B = enc_in.B
        T80 = 2 * T40
        gbd = self.dec_style(codes)
        ng = W.dec_norm
        dcat = S.dec_enc + 2 + S.dec_asr_res
        dt = self.dec_dt
        cats = [self.act("dec.catA", B, T40, dcat, dt), self.act("dec.catB", B, T40, dcat, dt)]
        cF, cN = S.dec_enc + S.dec_asr_res, S.dec_enc + S.dec_asr_res + 1
        for j, cat in enumerate(cats):
            a = L.F0nArgs()
            a.f0, a.n = F0.data_ptr(), Nn.data_ptr()
            a.wf, a.wn = W.t(W.dec_f0).data_ptr(), W.t(W.dec_n).data_ptr()
            a.y0, a.y1 = cat.t.data_ptr(), (enc_in.t.data_ptr() if j == 0 else None)
            a.ldf, a.ldy0, a.bsy0, a.ldy1, a.bsy1 = F0.stride(0), cat.ld, cat.bs, enc_in.ld, enc_in.bs
            a.B, a.T80, a.cf0, a.cn0, a.cf1, a.cn1, a.dtype = B, T80, cF, cN, S.d_txt, S.d_txt + 1, cat.dt
            assert enc_in.t.dtype == cat.t.dtype
            self._call(self.lib.stzs_f0n_down, a, "f0n_down")
            self.conv(W.dec_asr_res, Act(enc_in.t, 0, S.d_txt), cat.sl(S.dec_enc, S.dec_asr_res), what="asr_res")
        self.blk(W.dec_blk["dec.encode"], Act(enc_in.t, 0, S.d_txt + 2), cats[0].sl(0, S.dec_enc), ng, gbd, "dec.encode",
                 dt)
        src = 0
        for i in range(3):
            self.blk(W.dec_blk[f"dec.decode{i}"], Act(cats[src].t, 0, dcat), cats[1 - src].sl(0, S.dec_enc), ng, gbd,
                     f"dec.decode{i}", dt)
            src = 1 - src
        gen_in = self.act("dec.gen_in", B, T80, S.dec_out, dt)
        self.blk(W.dec_blk["dec.decode3"], Act(cats[src].t, 0, dcat), gen_in, ng, gbd, "dec.decode3", dt)
        return gen_in, gbd

    def sine_gen(self, F0: torch.Tensor, seeds) -> Act:
        """a10: NSF harmonic source from F0 [B, T80] (SineGen: fp64 frame-rate phase prefix, counter-RNG noise,
        Linear(9->1) + tanh) and its n_fft-point STFT (real | imag) -> har [B, Tf, har_ch] (csrc/source.hip)."""
        S, W = self.spec, self.W
        B, T80 = F0.shape[0], F0.shape[1]
        N = T80 * S.hop
        Tf = N // S.istft_hop + 1
        nh = S.harmonic_num + 1
        if isinstance(seeds, torch.Tensor) and seeds.device.type != "cpu":
            sd = seeds.to(torch.int32)
        else:
            skey = ("seeds", tuple(int(v) for v in seeds))
            sd = self._consts.get(skey)
            if sd is None:  # uploaded once per distinct seed list (graph-capture safe afterwards)
                host = torch.as_tensor(np.asarray(seeds, dtype=np.uint32).view(np.int32).copy())
                sd = self._consts[skey] = host.to(self.device)
        pref = self.buf("gen.pref", (B, nh, T80), torch.float32)
        # row pitch = the noise convs' padded K (32): the 1x1 noise conv then takes the LDS-DMA GEMM path
        dt = self.dec_dt
        # rows rounded up to a multiple of the first stage's noise-conv stride (zero past Tf): the buffer then reads as
        # whole super-rows (engine.upsample's super-row noise conv); the Act is the view of its Tf frames
        hb = self.buf("gen.har", (B, self._har_rows(Tf), _rup(S.har_ch, 32)), dt, zero=True)
        har = Act(hb[:, :Tf], 0, S.har_ch)
        a = L.SourceArgs()
        a.f0, a.seeds, a.merge_w, a.prefix, a.har = F0.data_ptr(), sd.data_ptr(), W.t(W.src_merge).data_ptr(), \
            pref.data_ptr(), har.ptr
        a.ldf, a.ldh, a.bsh = F0.stride(0), har.ld, har.bs
        a.B, a.T80, a.hop, a.n_fft, a.hop_s, a.nh = B, T80, S.hop, S.n_fft, S.istft_hop, nh
        a.sr, a.sine_amp, a.noise_std, a.voiced_thr = float(S.sr), S.sine_amp, S.noise_std, S.voiced_threshold
        a.har_dtype = har.dt
        self._call(self.lib.stzs_harmonic_source, a, "harmonic_source",  # F0 in, prefix, STFT rows out
                   cost=(0, B * T80 * 4 * (1 + 2 * nh) + B * Tf * S.har_ch * har.t.element_size()))
        return har

    def _har_rows(self, Tf: int) -> int:
        """rows allocated for Tf harmonic-source frames: a multiple of the stage-0 noise-conv stride"""
        s = math.prod(self.spec.up_rates[1:]) if len(self.spec.up_rates) > 1 else 1
        return _rup(Tf, s)

    def upsample(self, x: Act, har: Act, i: int) -> Act:
        """a11: generator stage i's noise conv of the harmonic features + LeakyReLU(0.1) -> polyphase
        ConvTranspose1d(k = 2 r, s = r) (+ ReflectionPad(1,0) on the last stage) + the noise conv as residual."""
        S, W = self.spec, self.W
        B = x.B
        n_up = len(S.up_rates)
        r, k = S.up_rates[i], S.up_kernels[i]
        c = S.gen_ch[i]
        last = i == n_up - 1
        Tcur = x.T
        Tn = Tcur * r + (1 if last else 0)
        dt = self.dec_dt
        xu = self.act(f"gen.x{i}", B, Tn, c, dt)
        nzw = self.W.ups_nz[i] if (self.ups_noise_fused and i < len(self.W.ups_nz)) else None
        if nzw is not None and dt == torch.bfloat16 and har.ld >= 32:
            # the 1x1 noise conv fused into the ConvTranspose (csrc/ups.hip STZS_CONV_UPS_NOISE): one more K-step per
            # column tile on the harmonic-source rows; its output never goes through HBM
            self.conv(nzw, x, xu, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=(k - r) // 2, T_final=Tcur * r,
                      refl=1 if last else 0, res=Act(har.t, 0, har.ld), flags=L.CONV_UPS_NOISE,
                      gate=self._t(nzw.nz32).data_ptr(), what=f"ups{i}")
            return xu
        xsrc = self.act(f"gen.xsrc{i}", B, Tn, c, dt)
        sup = W.noise_sup[i] if (not last and i < len(W.noise_sup)) else None
        sf0 = int(np.prod(S.up_rates[i + 1:])) if not last else 1
        rows_alloc = har.bs // har.ld  # rows of the buffer behind the Tf-frame view (zero past Tf)
        if (sup is not None and self.noise_super and har.dt == L.BF16 and har.bs % (sf0 * har.ld) == 0 and
                rows_alloc // sf0 >= Tn + 1 and sf0 * har.ld == sup.Ci and har.t.stride(1) == har.ld):
            # the strided noise conv on SUPER-ROWS (weights.noise_super_weights): the harmonic-source buffer read as
            # [B, rows / s, s * 32] is a k3 stride-1 conv over 192 channels -> the register-direct kernel (mrfv.hip)
            # instead of a stride-6 conv staging 6 rows of 64 B per output row
            hs = har.t.as_strided((B, rows_alloc // sf0, sf0 * har.ld), (har.bs, sf0 * har.ld, 1))
            self.conv(sup, Act(hs), xsrc, pad=1, T_out=Tn, what=f"noise_conv{i}")
        elif not last:
            # (T_out explicit: the harmonic buffer holds rows past the Tf frames -- zeros, rounded up for the super-row
            # view -- so har.T would over-count the output rows)
            self.conv(W.noise_conv[i], har.sl(0, S.har_ch), xsrc, stride=sf0, pad=(sf0 + 1) // 2, T_out=Tn,
                      what=f"noise_conv{i}")
        else:
            self.conv(W.noise_conv[i], har.sl(0, S.har_ch), xsrc, T_out=Tn, what=f"noise_conv{i}")
        self.conv(W.ups[i], x, xu, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=(k - r) // 2, T_final=Tcur * r,
                  refl=1 if last else 0, res=xsrc, what=f"ups{i}")
        return xu

    def conv_post(self, x: Act) -> Act:
        """LeakyReLU(0.01) + conv_post (128 -> 22, k7) -> fp32 rows [B, Tf, 22] (log-magnitude | phase argument)."""
        S, W = self.spec, self.W
        post = self.act("gen.post", x.B, x.T, S.har_ch, torch.float32)
        self.conv(W.conv_post, x, Act(post.t, 0, S.har_ch), pad=3, pro_act=L.ACT_LEAKY, pro_slope=0.01,
                  what="conv_post")
        return post

    def istft(self, post: Act) -> torch.Tensor:
        """a13: exp / sin spectrum, 20-point irfft, Hann overlap-add (hop 5), window-envelope normalisation."""
        S = self.spec
        B, Tcur = post.B, post.T
        Nout = (Tcur - 1) * S.istft_hop
        wav = self.buf("gen.wav", (B, Nout), torch.float32)
        a = L.IstftArgs()
        a.post, a.wav, a.ldp, a.bsp, a.bsw = post.ptr, wav.data_ptr(), post.ld, post.bs, Nout
        a.B, a.Tf, a.n_fft, a.hop_s = B, Tcur, S.n_fft, S.istft_hop
        self._call(self.lib.stzs_istft, a, "istft", cost=(0, B * Tcur * S.har_ch * 4 + B * Nout * 4))
        return wav

    def generator(self, x: Act, F0: torch.Tensor, seeds, gbd, trace=None, istft=True, har: Act = None):
        """a10-a13: harmonic source, per stage the noise conv + ConvTranspose up-sampling and the MRF, then
        conv_post and the iSTFT.  har: precomputed harmonic-source features (the chunked decoder's window slice)."""
        S, W = self.spec, self.W
        ng = W.dec_norm
        if har is None:
            har = self.sine_gen(F0, seeds)
        if trace is not None:
            trace["har"] = har
        for i in range(len(S.up_rates)):
            xu = self.upsample(x, har, i)
            if trace is not None:
                trace[f"mrf_in{i}"] = xu
            x = self.mrf(xu, i, gbd, ng)
            if trace is not None:
                trace[f"mrf_out{i}"] = x
        post = self.conv_post(x)
        if trace is not None:
            trace["post"] = post
        if not istft:
            return post
        return self.istft(post)

    def _istft_chunk(self, rows_ptr, ldp, bsp, B, f0, Fc, fin, wav, tails, i):
        """one streaming-iSTFT launch: conv_post frames [f0, f0 + Fc) at rows_ptr (row pitch ldp, batch stride bsp,
        fp32) -> samples [n0, n1) of wav [B, Nout], the 3-frame tail carried in the ping-pong buffers.  -> (n0, n1)"""
        S = self.spec
        n0, n1 = C.c_int64(), C.c_int64()
        halo = self.lib.stzs_istft_stream_span(f0, Fc, fin, S.n_fft, S.istft_hop, C.byref(n0), C.byref(n1))
        L.check(min(halo, 0), "istft_stream_span")
        assert halo <= 8
        a = L.IstftStreamArgs()
        a.post = rows_ptr
        a.tail_in = tails[i % 2].data_ptr() if f0 > 0 else None
        a.tail_out = tails[(i + 1) % 2].data_ptr() if not fin else None
        a.wav = wav.data_ptr() + n0.value * 4
        a.ldp, a.bsp, a.bsw, a.ldt = ldp, bsp, wav.shape[1], tails[0].shape[2]
        a.B, a.f0, a.Fc, a.final_chunk, a.n_fft, a.hop_s = B, f0, Fc, fin, S.n_fft, S.istft_hop
        self._call(self.lib.stzs_istft_stream, a, "istft_stream")
        return n0.value, n1.value

    @staticmethod
    def chunk_windows(T40: int, chunk: int, halo: int):
        """the chunked decoder's schedule (oracle/stzs_ref.py chunk_windows): chunk i owns aligned frames
        [i chunk, min((i + 1) chunk, T40)) and is decoded over a window of fixed length W = min(chunk + 2 halo, T40)
        starting at clamp(a - halo, 0, T40 - W).  -> [(a, b, wa, wb)]"""
        W = min(chunk + 2 * halo, T40)
        out = []
        for a in range(0, T40, chunk):
            wa = min(max(0, a - halo), T40 - W)
            out.append((a, min(a + chunk, T40), wa, wa + W))
        return out

    def _copy_rows(self, x: int, ldx: int, bsx: int, y: int, ldy: int, bsy: int, nb: int, R: int, Cn: int, dti, dto):
        """stzs_copy2d on raw byte addresses: nb blocks of R rows x Cn columns (source block stride bsx elements)"""
        a = L.CopyArgs()
        a.x, a.y, a.ldx, a.bsx, a.ldy, a.bsy = x, y, ldx, bsx, ldy, bsy
        a.B, a.R, a.C, a.in_dtype, a.out_dtype = nb, R, Cn, dti, dto
        self._call(self.lib.stzs_copy2d, a, "copy_windows")

    def decode_chunked(self, pro: dict, codes: torch.Tensor, seeds, chunk: int, halo: int, batch_windows=True,
                       max_pass_rows: int = 64):
        """configs[4] CHUNKED streaming decoder (oracle/stzs_ref.py decode_chunked): each chunk of `chunk` aligned
        frames is decoded over its fixed-length window (chunk_windows) -- pre-blocks and generator on the window alone,
        AdaIN with WINDOW-local InstanceNorm statistics -- on the slice of the whole utterance's harmonic-source
        features (global phase prefix and noise counters); its own conv_post frames go through the streaming iSTFT with
        the carried tail.  The first chunk's window is decoded alone (its audio is ready after one window's decode);
        with batch_windows every later window is then decoded in ONE pass, the windows as the rows of one batch
        (window-major, [window][utterance]): every decoder kernel is batch-invariant (per-utterance tiles and
        statistics), so this is bit-identical to decoding them one by one (batch_windows=False), in 3 passes' worth of
        launches instead of one per chunk.  A pass holds at most max(B, max_pass_rows) window rows (windows x utterances):
        a pass's audio is ready only when the whole pass is decoded and its activations scale with its rows, so at large
        B or long targets the later windows go in several passes (time to the second chunk ~ one pass's decode; peak
        activation memory ~ max_pass_rows windows).  Yields (first_sample, wav chunk [B, n]) views of one [B, 600 T40]
        buffer."""
        S = self.spec
        enc_in, F0, Nn, T40 = pro["asr_buf"], pro["F0"], pro["N"], pro["T40"]
        B = enc_in.B
        fpf = S.frame40 // S.istft_hop
        har = self.sine_gen(F0, seeds)
        Nout = T40 * S.frame40
        wav = self.buf("gen.wav_chunked", (B, Nout), torch.float32)
        ncol = _rup(S.n_fft + 2, 4)
        tails = [self.buf("gen.ctail0", (B, 8, ncol), torch.float32), self.buf("gen.ctail1", (B, 8, ncol), torch.float32)]
        dt = self.dec_dt
        wins = self.chunk_windows(T40, chunk, halo)
        Wn = wins[0][3] - wins[0][2]
        Tfw = fpf * Wn + 1
        if batch_windows:
            per = max(1, max_pass_rows // max(B, 1))  # windows per pass after the first
            rest = list(range(1, len(wins)))
            groups = [[0]] + [rest[i:i + per] for i in range(0, len(rest), per)]
        else:
            groups = [[k] for k in range(len(wins))]
        groups = [g for g in groups if g]
        F0c, Nc = F0.contiguous(), Nn.contiguous()
        cdt = L.F32 if codes.dtype == torch.float32 else L.BF16
        for ks in groups:
            nw = len(ks)
            Bw = nw * B
            enc_w = self.act("dec.enc_in_w", Bw, Wn, S.d_txt + 2, dt)
            har_w = Act(self.buf("gen.har_w", (Bw, self._har_rows(Tfw), har.ld), dt, zero=True)[:, :Tfw], 0, S.har_ch)
            F0w = self.buf("dec.F0w", (Bw, 2 * Wn), torch.float32)
            Nw = self.buf("dec.Nw", (Bw, 2 * Wn), torch.float32)
            cw_ = codes if nw == 1 else self.buf("dec.codes_w", (Bw,) + tuple(codes.shape[1:]), codes.dtype)
            esz, hsz = enc_in.t.element_size(), har.t.element_size()
            for b in range(B):
                # runs of windows whose starts are `chunk` apart: one strided copy per run and tensor
                i = 0
                while i < nw:
                    j = i + 1
                    while j < nw and wins[ks[j]][2] - wins[ks[j - 1]][2] == chunk:
                        j += 1
                    wa, cnt = wins[ks[i]][2], j - i
                    row = i * B + b  # window-major rows of the batch
                    self._copy_rows(enc_in.t.data_ptr() + (b * enc_in.bs + wa * enc_in.ld) * esz, enc_in.ld,
                                    chunk * enc_in.ld, enc_w.t.data_ptr() + row * enc_w.bs * esz, enc_w.ld,
                                    B * enc_w.bs, cnt, Wn, S.d_txt, enc_in.dt, enc_w.dt)
                    self._copy_rows(har.t.data_ptr() + (b * har.bs + fpf * wa * har.ld) * hsz, har.ld,
                                    fpf * chunk * har.ld, har_w.t.data_ptr() + row * har_w.bs * hsz, har_w.ld,
                                    B * har_w.bs, cnt, Tfw, S.har_ch, har.dt, har_w.dt)
                    for src, dst in ((F0c, F0w), (Nc, Nw)):
                        self._copy_rows(src.data_ptr() + (b * src.stride(0) + 2 * wa) * 4, 2 * Wn, 2 * chunk,
                                        dst.data_ptr() + row * 2 * Wn * 4, 2 * Wn, B * 2 * Wn, cnt, 1, 2 * Wn,
                                        L.F32, L.F32)
                    i = j
                if nw > 1:  # every window of utterance b takes its codes (source block stride 0)
                    Lc, Dc = codes.shape[1], codes.shape[2]
                    self._copy_rows(codes.data_ptr() + b * codes.stride(0) * codes.element_size(), Dc, 0,
                                    cw_.data_ptr() + b * Lc * Dc * cw_.element_size(), Dc, B * Lc * Dc, nw, Lc, Dc,
                                    cdt, cdt)
            gen_in, gbd = self.decoder_pre(dict(asr_buf=enc_w, F0=F0w, N=Nw, T40=Wn), cw_)
            post = self.generator(gen_in, F0w, seeds, gbd, istft=False, har=har_w)
            for i, k in enumerate(ks):
                a0, b0, wa, _ = wins[k]
                fin = int(b0 == T40)
                r0 = fpf * (a0 - wa)
                n0, n1 = self._istft_chunk(post.ptr + (i * B * post.bs + r0 * post.ld) * 4, post.ld, post.bs, B,
                                           fpf * a0, fpf * (b0 - a0) + fin, fin, wav, tails, k)
                yield n0, wav[:, n0:n1]

    def istft_stream(self, post: Act, chunk_frames: int):
        """iSTFT of conv_post frames [B, Tf, 22] in chunks of `chunk_frames` frames,
        the 3-frame tail carried between chunks (ping-pong buffers).  Yields (n0, wav[:, n0:n1]) as each
        chunk is enqueued; the views are slices of one [B, Nout] buffer, so no chunk overwrites another,
        and their concatenation is bit-identical to the whole-utterance iSTFT."""
        S = self.spec
        B, Tf = post.B, post.T
        Nout = (Tf - 1) * S.istft_hop
        wav = self.buf("gen.wav_stream", (B, Nout), torch.float32)
        ncol = _rup(S.n_fft + 2, 4)
        tails = [self.buf("gen.tail0", (B, 8, ncol), torch.float32), self.buf("gen.tail1", (B, 8, ncol), torch.float32)]
        n0, n1 = C.c_int64(), C.c_int64()
        f0, i = 0, 0
        while f0 < Tf:
            Fc = min(chunk_frames, Tf - f0)
            if 0 < Tf - f0 - Fc < 2:  # fold a 1-frame remainder (Tf = 600*T40/5 + 1) into this chunk
                Fc = Tf - f0
            fin = int(f0 + Fc == Tf)
            halo = self.lib.stzs_istft_stream_span(f0, Fc, fin, S.n_fft, S.istft_hop, C.byref(n0), C.byref(n1))
            L.check(min(halo, 0), "istft_stream_span")
            assert halo <= 8
            a = L.IstftStreamArgs()
            a.post = post.ptr + f0 * post.ld * 4
            a.tail_in = tails[i % 2].data_ptr() if f0 > 0 else None
            a.tail_out = tails[(i + 1) % 2].data_ptr() if not fin else None
            a.wav = wav.data_ptr() + n0.value * 4
            a.ldp, a.bsp, a.bsw, a.ldt = post.ld, post.bs, Nout, ncol
            a.B, a.f0, a.Fc, a.final_chunk, a.n_fft, a.hop_s = B, f0, Fc, fin, S.n_fft, S.istft_hop
            self._call(self.lib.stzs_istft_stream, a, "istft_stream")
            yield n0.value, wav[:, n0.value:n1.value]
            f0 += Fc
            i += 1

    def _launch_group(self, args, what):
        """the collected stzs_conv_args (conv(collect=...)) as ONE stzs_conv1d_group call"""
        arr = (L.ConvArgs * len(args))(*args)
        rc = self.lib.stzs_conv1d_group(arr, len(args), self.stream())
        if rc < 0:
            L.check(rc, what)
        self.launches += rc

    def _finalize_group(self, refs):
        """the statistics of up to three collected convs finalised in one launch (stzs_chan_stats_final_group)"""
        arr = (L.StatsArgs * len(refs))()
        for s, r in zip(arr, refs):
            s.mean, s.rstd, s.partial = r.mean.data_ptr(), r.rstd.data_ptr(), r.part.data_ptr()
            s.stat_bs, s.B, s.T, s.C, s.eps = r.ld, r.B, r.T, r.ld, 1e-5
        assert len({r.chunk_rows for r in refs}) == 1
        self.launches += 1
        L.check(self.lib.stzs_chan_stats_final_group(arr, len(refs), refs[0].chunk_rows, self.stream()),
                "chan_stats_final_group")
        for r in refs:
            r.done = True

    def _mrf_trio(self, x: Act, i, gbd, ng):
        """mrf() with the three resblocks (k 3 / 7 / 11) advanced layer by layer side by side: each layer's c1 convs in
        ONE launch (stzs_conv1d_group -> mrfv_trio at small batch), their statistics in one, the non-last c2 convs and
        their statistics likewise; the last layer's c2 convs stay one after the other (each adds the previous
        resblocks' sum, acc_in).  Per-resblock buffers; every value bit-identical to mrf()'s order."""
        S, W = self.spec, self.W
        B, T, c = x.B, x.T, x.C
        gbase, gbs = gbd.data_ptr(), ng.total
        dt = x.t.dtype
        nk = len(S.rb_kernels)
        xs = self.act(f"gen.xs{i}", B, T, c, dt)
        t1 = [self.act(f"gen.t1_{i}.{j}", B, T, c, dt) for j in range(nk)]
        bufs = [(self.act(f"gen.ba{i}.{j}", B, T, c, dt), self.act(f"gen.bb{i}.{j}", B, T, c, dt)) for j in range(nk)]
        mx, rx, sb = self.stats(x, f"gen.sx{i}")
        cur, cm, cr = [x] * nk, [mx] * nk, [rx] * nk
        nl = len(W.rb[i][0])
        for m in range(nl):
            grp, st1 = [], []
            for j, res in enumerate(W.rb[i]):
                lw = res[m]
                k, dil = lw["k"], lw["dil"]
                o1, c1 = ng.offsets[lw["n1"]]
                _, st = self.conv(lw["c1"], cur[j], t1[j], pad=dil * (k - 1) // 2, dil=dil,
                                  pro=(cm[j], cr[j], sb, gbase + o1 * 4, gbs, c1), pro_act=L.ACT_SNAKE,
                                  pro_alpha=lw["a1"], stats_key=f"gen.st{i}.{j}", collect=grp, what="rb.c1")
                st1.append(st)
            self._launch_group(grp, "rb.c1")
            self._finalize_group([st[0].ref for st in st1])
            last = m == nl - 1
            grp, st2, outs = [], [], []
            for j, res in enumerate(W.rb[i]):
                lw = res[m]
                k = lw["k"]
                o2, c2 = ng.offsets[lw["n2"]]
                tm, tr, _ = st1[j]
                kw = dict(pad=(k - 1) // 2, pro=(tm, tr, sb, gbase + o2 * 4, gbs, c2), pro_act=L.ACT_SNAKE,
                          pro_alpha=lw["a2"], res=cur[j], what="rb.c2")
                if last:  # xs = c2 / nk + cur (+ xs): the resblocks' sum in resblock order, one launch each
                    self.conv(lw["c2"], t1[j], xs, alpha=1.0 / nk, acc_in=(xs if j > 0 else None), beta=1.0, **kw)
                else:
                    out = bufs[j][0] if cur[j] is not bufs[j][0] else bufs[j][1]
                    _, st = self.conv(lw["c2"], t1[j], out, stats_key=f"gen.sc{i}.{j}.{m % 2}", collect=grp, **kw)
                    st2.append(st)
                    outs.append(out)
            if not last:
                self._launch_group(grp, "rb.c2")
                self._finalize_group([st[0].ref for st in st2])
                for j in range(nk):
                    cur[j], (cm[j], cr[j], _) = outs[j], st2[j]
        return xs

    def mrf(self, x: Act, i, gbd, ng):
        S, W = self.spec, self.W
        if (self.mrf_trio and self.timer is None and x.B <= 4 and tuple(S.rb_kernels) == (3, 7, 11) and
                len({len(res) for res in W.rb[i]}) == 1 and all(r["k"] == k for res, k in zip(W.rb[i], (3, 7, 11))
                                                               for r in res)):
            return self._mrf_trio(x, i, gbd, ng)
        B, T, c = x.B, x.T, x.C
        gbase, gbs = gbd.data_ptr(), ng.total
        dt = x.t.dtype
        xs = self.act(f"gen.xs{i}", B, T, c, dt)
        bufA = self.act(f"gen.ba{i}", B, T, c, dt)
        bufB = self.act(f"gen.bb{i}", B, T, c, dt)
        t1 = self.act(f"gen.t1_{i}", B, T, c, dt)
        mx, rx, sb = self.stats(x, f"gen.sx{i}")
        nk = len(S.rb_kernels)
        for j, res in enumerate(W.rb[i]):
            cur, cm, cr = x, mx, rx
            for m, lw in enumerate(res):
                k, dil = lw["k"], lw["dil"]
                o1, c1 = ng.offsets[lw["n1"]]
                o2, c2 = ng.offsets[lw["n2"]]
                _, (tm, tr, _) = self.conv(lw["c1"], cur, t1, pad=dil * (k - 1) // 2, dil=dil,
                                           pro=(cm, cr, sb, gbase + o1 * 4, gbs, c1), pro_act=L.ACT_SNAKE,
                                           pro_alpha=lw["a1"], stats_key=f"gen.st{i}", what="rb.c1")
                last = m == len(res) - 1
                out = xs if last else (bufA if cur is not bufA else bufB)
                r2 = self.conv(lw["c2"], t1, out, pad=(k - 1) // 2, pro=(tm, tr, sb, gbase + o2 * 4, gbs, c2),
                               pro_act=L.ACT_SNAKE, pro_alpha=lw["a2"], res=cur, alpha=(1.0 / nk) if last else 1.0,
                               acc_in=(xs if (last and j > 0) else None), beta=1.0,
                               stats_key=None if last else f"gen.sc{i}.{m % 2}", what="rb.c2")
                if not last:
                    _, (cm, cr, _) = r2
                    cur = out
        return xs

    # ------------------------------------------------------------------ end to end
    def twin(self) -> "StyleTTSZS":
        """a second engine on the SAME packed weights with its own buffer cache: two twins can synthesize
        two utterance batches concurrently on two streams (their graphs replay side by side, so one batch's
        latency-bound phases -- LSTM recurrences, statistics, small GEMMs -- overlap the other's convs)."""
        t = object.__new__(StyleTTSZS)
        t.__dict__.update(self.__dict__)
        t._bufs, t._retired, t._consts, t._side, t._branch, t.launches, t.timer = {}, [], {}, {}, "", 0, None
        t._depth = 0
        t.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        return t

    def encode_inputs(self, tokens, ref_wav, prompt_idx=None):
        """text encoder || prompt encoder (independent; forked when branch_streams) -> (h_txt, prompt codes)."""
        ref = None if ref_wav is None else ref_wav.to(self.device)
        return self.fork("enc", lambda: self.text_encode(tokens), lambda: self.prompt_encode(ref, prompt_idx))

    def capture(self, fn):
        """Capture `fn()` into one HIP graph.  fn must be replay-safe: device-resident inputs, cached
        buffers (a warm-up call on a side stream allocates them), no host syncs (synth() skips its status
        check while capturing).  -> (CheckedGraph, fn's output); graph.check() raises after a replay whose LSTM
        exchange timed out (the captured kernels OR the flag into this engine's status word)."""
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            fn()
        cur.wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fn()
        for k, ent in self._bufs.items():
            if isinstance(k, tuple):
                ent[3] = True
        return CheckedGraph(g, self), out

    def _capturing(self) -> bool:
        return torch.cuda.is_current_stream_capturing()

    def synth(self, tokens, ref_wav, steps=2, cfg_scale=1.0, noise=None, durations=None, seeds=None, codes=None,
              n_frames=None, prompt_idx=None, check=True):
        """tokens int [B, T_txt]; ref_wav fp32 [B|1, N]; noise fp32 [B, L_s, code]; durations int [B, T_txt]
        (host tensor, or device tensor + n_frames: no device sync); seeds: per-utterance source-noise
        seeds; prompt_idx: teacher-forced discrete prompt codes [B|1, L_s, G] (ref_wav then unused).
        check: raise RuntimeError if an LSTM exchange of this call timed out (its durations / prosody would be
        wrong) -- one 4-B device read, skipped while a graph is being captured (CheckedGraph.check() then);
        check=False leaves it to the caller (check_status(), or the returned `status` word).
        -> dict(wav=[B, 600*T40], prompt_idx=[B|1, L_s, G], status=int32 [1], ...)"""
        out = self._synth(tokens, ref_wav, steps, cfg_scale, noise, durations, seeds, codes, n_frames, prompt_idx)
        if check and not self._capturing():
            self.check_status()
        return out

    def _synth(self, tokens, ref_wav, steps, cfg_scale, noise, durations, seeds, codes, n_frames, prompt_idx):
        S = self.spec
        dev = self.device
        tokens = tokens.to(dev, torch.int32) if tokens.device != dev or tokens.dtype != torch.int32 else tokens
        B = tokens.shape[0]
        h, prompt = self.encode_inputs(tokens, ref_wav, prompt_idx)
        pidx = self.prompt_idx
        if prompt.shape[0] == 1 and B > 1:
            pe = self.buf("prompt.bc", (B, S.L_s, S.code_dim), torch.float32)
            pe.copy_(prompt.expand(B, -1, -1))
            prompt = pe
        if codes is None:
            eps = noise.to(dev, torch.float32)
            codes = self.sample_style(h, prompt, eps, steps, cfg_scale)
        pro = self.predict_prosody(h, codes, durations, n_frames)
        seeds = list(range(B)) if seeds is None else seeds
        wav = self.decode(pro, codes, seeds)
        return dict(wav=wav, codes=codes, h_txt=h, prompt=prompt, prompt_idx=pidx, status=self.status, **pro)


    def synth_stream(self, tokens, ref_wav, steps=2, cfg_scale=1.0, noise=None, durations=None, seeds=None,
                     codes=None, n_frames=None, chunk_s=1.0, prompt_idx=None, check=True, chunked_halo=None):
        """configs[4] long-form synthesis with the streaming iSTFT decoder: the text,
        style, prosody and conv stack run over the whole target (AdaIN instance statistics are
        utterance-global), then the waveform is emitted in `chunk_s`-second chunks.  Yields
        (first_sample, wav_chunk [B, n]) device views; their concatenation equals synth()["wav"].
        chunked_halo=H: the CHUNKED decoder instead (decode_chunked: every `chunk_s` chunk decoded over a window of
        +-H aligned frames with window-local statistics -- a different function, parity vs oracle decode_chunked):
        the first chunk is ready after the front and one window's decode."""
        S = self.spec
        dev = self.device
        tokens = tokens.to(dev, torch.int32) if tokens.device != dev or tokens.dtype != torch.int32 else tokens
        B = tokens.shape[0]
        h, prompt = self.encode_inputs(tokens, ref_wav, prompt_idx)
        if prompt.shape[0] == 1 and B > 1:
            pe = self.buf("prompt.bc", (B, S.L_s, S.code_dim), torch.float32)
            pe.copy_(prompt.expand(B, -1, -1))
            prompt = pe
        if codes is None:
            codes = self.sample_style(h, prompt, noise.to(dev, torch.float32), steps, cfg_scale)
        pro = self.predict_prosody(h, codes, durations, n_frames)
        seeds = list(range(B)) if seeds is None else seeds
        if chunked_halo is not None:  # the chunked decoder: chunk-local statistics, first audio after one window
            yield from self.decode_chunked(pro, codes, seeds, max(1, int(round(chunk_s * S.sr / S.frame40))),
                                           int(chunked_halo))
        else:
            post = self.decode(pro, codes, seeds, istft=False)
            frames = max(1, int(round(chunk_s * S.sr / S.istft_hop)))
            yield from self.istft_stream(post, frames)
        if check and not self._capturing():
            self.check_status()


# fork sites of the batch-1 latency engine: the text encoder beside the prompt encoder on a forked branch of the
# captured graph (configs[1] p50 6.06-6.20 -> 5.91 ms, 4 A/B pairs, profiles/r05_m_fork_sites_ab.log); the F0 || N
# fork measured slower (6.19-6.27 vs 6.05-6.18) and stays off.  env STZS_LATENCY_FORKS="" turns it off.
LATENCY_FORKS = frozenset(v for v in os.environ.get("STZS_LATENCY_FORKS", "enc").split(",") if v)


def latency_engine(spec: Spec, packed: PackedModel, device="cuda:0") -> "StyleTTSZS":
    """the batch-1 serving engine bench.py times for the configs[1] p50 (and tests/test_gpu_configs.py checks against
    the oracle): the same packed weights, the denoiser layer linears on the whole-chip small-M form
    (LATENCY_DN_ROWS, csrc/rows.hip) and split-K ffn2 wherever the rows form does not apply (LATENCY_DN_SPLITK);
    with durations given, the duration LSTM paired with the shared LSTM (dur_overlap, on in every engine); the text
    and prompt encoders on forked graph branches (LATENCY_FORKS)."""
    return StyleTTSZS(spec, None, device=device, packed=packed, dn_splitk=LATENCY_DN_SPLITK, dn_rows=LATENCY_DN_ROWS,
                      te_splitk=LATENCY_TE_SPLITK, blk_splitk=LATENCY_BLK_SPLITK, branch_streams=LATENCY_FORKS)


class CheckedGraph:
    """a captured HIP graph of one engine + that engine's LSTM status check (StyleTTSZS.capture).  replay()
    enqueues the graph; check() reads the engine's status word (one 4-B device read, i.e. a sync) and raises if
    any LSTM exchange of the replays since the last check timed out."""

    def __init__(self, graph, eng):
        self.graph, self.eng = graph, eng

    def replay(self):
        self.graph.replay()

    def check(self):
        return self.eng.check_status()


class _OffsetAct(Act):
    """Act whose base pointer is shifted by `off` elements (writes into a row window of a larger buffer)."""

    def __init__(self, base: Act, off: int):
        super().__init__(base.t, base.c0, base.C)
        self._off = off

    @property
    def ptr(self):
        return self.t.data_ptr() + (self.c0 + self._off) * self.t.element_size()
