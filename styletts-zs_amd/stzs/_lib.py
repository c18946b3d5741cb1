"""ctypes binding of libstzs_hip.so (the C-ABI declared in include/stzs.h).

This is also the reference-side binding stub shown in INTEGRATION.md: the structures below
mirror the header field-for-field.  The library is built in-tree by styletts-zs_amd/build.py;
there is deliberately NO fallback — importing the product path without the library raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STZS_LIB", os.path.join(_HERE, "libstzs_hip.so"))

F32, BF16, I32, F8 = 0, 1, 2, 3
OK, EINVAL, ESHAPE, EDTYPE, EHIP = 0, -1, -2, -3, -4
ACT_NONE, ACT_LEAKY, ACT_SNAKE, ACT_GELU, ACT_SILU = 0, 1, 2, 3, 4
PRO_NONE, PRO_ADAIN = 0, 1
CONV_STAT_ROWS = 64  # include/stzs.h STZS_CONV_STAT_ROWS
CONV_W_LANE16 = 16  # include/stzs.h STZS_CONV_W_LANE16
CONV_W_NARROW32 = 32  # include/stzs.h STZS_CONV_W_NARROW32
CONV_W_FRAG32 = 256  # include/stzs.h STZS_CONV_W_FRAG32
CONV_W_F32 = 64  # include/stzs.h STZS_CONV_W_F32 (fp32-MFMA conv_f32)
CONV_W_X3 = 1024  # include/stzs.h STZS_CONV_W_X3 (precise mode: split-operand bf16x3 conv_x3)
CONV_LINEAR_IDS = 128  # include/stzs.h STZS_CONV_LINEAR_IDS (diagnostic: no XCD remap)
CONV_ROWS = 2048  # include/stzs.h STZS_CONV_ROWS (small-M linear on the whole chip, csrc/rows.hip)
CONV_UPS_NOISE = 4096  # include/stzs.h STZS_CONV_UPS_NOISE (ConvTranspose + fused 1x1 noise conv, csrc/ups.hip)
CONV_MRFV_NARROW = 8192  # include/stzs.h STZS_CONV_MRFV_NARROW (register-direct MRF conv at 128 channels per workgroup)
CONV_MRFV_T128 = 32768  # include/stzs.h STZS_CONV_MRFV_T128 (register-direct MRF conv: keep 128-row tiles on small grids)
CONV_RING = 65536  # include/stzs.h STZS_CONV_RING (split-K conv_mfma: keep the 3-slot weight ring)
CONV_SK_TICKET = 131072  # include/stzs.h STZS_CONV_SK_TICKET (DEEP split-K: last-arriver combine)
CONV_W_FRAG32X3 = 16384  # include/stzs.h STZS_CONV_W_FRAG32X3 (precise register-direct MRF conv, csrc/mrfx.hip)

vp = C.c_void_p
i64 = C.c_int64
i32 = C.c_int32
f32 = C.c_float


class ConvArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("x", "w", "bias", "y", "res", "acc_in", "gate", "pro_mean", "pro_rstd",
                                  "pro_gb", "pro_alpha")] + \
               [(n, i64) for n in ("ldx", "bsx", "ldy", "bsy", "ldr", "bsr", "lda", "bsa",
                                   "gate_bs", "stat_bs", "gb_bs", "gb_beta_off")] + \
               [(n, i32) for n in ("B", "T_in", "T_out", "Ci", "Co", "ks", "dil", "stride", "pad",
                                   "ci_pad", "co_pad", "cic", "ups", "ups_pad", "T_final", "refl", "res_tdiv",
                                   "in_dtype", "out_dtype", "pro_mode", "pro_act", "epi_act", "flags")] + \
               [(n, f32) for n in ("pro_cscale", "pro_slope", "epi_slope", "alpha", "beta", "pad_f")] + \
               [("stat_part", vp), ("stat_ld", i64), ("x_scale", vp), ("w_scale", vp),
                ("splitk_ws", vp), ("splitk_ctr", vp), ("splitk", i32), ("pad_sk", i32),
                ("pro_part", vp), ("pro_ld", i64), ("pro_nch", i32), ("pro_T", i32), ("pro_eps", f32), ("pad_pp", f32)]


class StatsArgs(C.Structure):
    _fields_ = [("x", vp), ("mean", vp), ("rstd", vp), ("partial", vp),
                ("ld", i64), ("bs", i64), ("stat_bs", i64),
                ("B", i32), ("T", i32), ("C", i32), ("dtype", i32), ("eps", f32), ("pad_f", f32)]


class RowLNArgs(C.Structure):
    _fields_ = [("x", vp), ("y", vp), ("G", vp), ("Bt", vp),
                ("ldx", i64), ("ldy", i64), ("gs", i64), ("bs", i64),
                ("R", i32), ("C", i32), ("gdiv", i32), ("in_dtype", i32), ("out_dtype", i32), ("act", i32),
                ("gadd", f32), ("eps", f32), ("slope", f32), ("pad_f", f32), ("y_scale", vp)]


class QuantArgs(C.Structure):
    _fields_ = [("x", vp), ("y", vp), ("scale", vp), ("ldx", i64), ("ldy", i64), ("R", i32), ("C", i32)]


class AttnArgs(C.Structure):
    _fields_ = [("q", vp), ("k", vp), ("v", vp), ("o", vp)] + \
               [(n, i64) for n in ("ldq", "ldk", "ldv", "ldo", "bsq", "bsk", "bsv", "bso")] + \
               [(n, i32) for n in ("R", "Lq", "Lk", "heads", "dh", "precise")]


class LstmArgs(C.Structure):
    _fields_ = [("gx", vp), ("whhT", vp), ("y", vp), ("xchg", vp), ("sync", vp),
                ("ldg", i64), ("bsg", i64), ("ldy", i64), ("bsy", i64),
                ("B", i32), ("T", i32), ("H", i32), ("ndir", i32),
                ("status", vp), ("spin_limit", C.c_uint32), ("precise", C.c_uint32)]


STATUS_LSTM_TIMEOUT = 1  # include/stzs.h STZS_STATUS_LSTM_TIMEOUT


class PrPrepArgs(C.Structure):
    _fields_ = [("codes", vp), ("h", vp), ("y", vp)] + \
               [(n, i64) for n in ("ldc", "bsc", "ldh", "bsh", "ldy", "bsy")] + \
               [(n, i32) for n in ("B", "L", "T", "c0", "Cs", "Ch", "yc0", "f32")]


class DurArgs(C.Structure):
    _fields_ = [("logits", vp), ("override_dur", vp), ("dur", vp), ("dsum", vp),
                ("ldl", i64), ("bsl", i64), ("B", i32), ("T", i32), ("nbins", i32), ("pad_i", i32)]


class AlignArgs(C.Structure):
    _fields_ = [("dur", vp), ("idx", vp), ("total", vp), ("B", i32), ("T", i32), ("T40", i32), ("pad_i", i32)]


class GatherArgs(C.Structure):
    _fields_ = [("x", vp), ("idx", vp), ("y", vp)] + \
               [(n, i64) for n in ("ldx", "bsx", "ldy", "bsy")] + \
               [(n, i32) for n in ("B", "Tsrc", "Tdst", "C", "xc0", "yc0", "dtype", "pad_i")]


class DwupArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("x", "y", "mean", "rstd", "gb", "w", "wb")] + \
               [(n, i64) for n in ("ldx", "bsx", "ldy", "bsy", "stat_bs", "gb_bs", "gb_beta_off")] + \
               [("B", i32), ("T", i32), ("C", i32), ("dtype", i32), ("slope", f32), ("pad_f", f32)]


class F0nArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("f0", "n", "wf", "wn", "y0", "y1")] + \
               [(n, i64) for n in ("ldf", "ldy0", "bsy0", "ldy1", "bsy1")] + \
               [(n, i32) for n in ("B", "T80", "cf0", "cn0", "cf1", "cn1", "dtype", "pad_i")]


class SourceArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("f0", "seeds", "merge_w", "prefix", "har")] + \
               [(n, i64) for n in ("ldf", "ldh", "bsh")] + \
               [(n, i32) for n in ("B", "T80", "hop", "n_fft", "hop_s", "nh")] + \
               [(n, f32) for n in ("sr", "sine_amp", "noise_std", "voiced_thr")] + \
               [("har_dtype", i32), ("pad_i", i32)]


class IstftArgs(C.Structure):
    _fields_ = [("post", vp), ("wav", vp), ("ldp", i64), ("bsp", i64), ("bsw", i64),
                ("B", i32), ("Tf", i32), ("n_fft", i32), ("hop_s", i32)]


class IstftStreamArgs(C.Structure):
    _fields_ = [("post", vp), ("tail_in", vp), ("tail_out", vp), ("wav", vp),
                ("ldp", i64), ("bsp", i64), ("bsw", i64), ("ldt", i64),
                ("B", i32), ("f0", i32), ("Fc", i32), ("final_chunk", i32), ("n_fft", i32), ("hop_s", i32)]


class FramesArgs(C.Structure):
    _fields_ = [("wav", vp), ("window", vp), ("y", vp), ("ldw", i64), ("ldy", i64), ("bsy", i64)] + \
               [(n, i32) for n in ("B", "N", "F", "n_fft", "win", "hop")]


class LogMelArgs(C.Structure):
    _fields_ = [("spec", vp), ("fb", vp), ("ranges", vp), ("y", vp)] + \
               [(n, i64) for n in ("lds", "bss", "ldy", "bsy")] + \
               [(n, i32) for n in ("B", "F", "nbin", "n_mels", "out_dtype", "pad_i")]


class PoolArgs(C.Structure):
    _fields_ = [("x", vp), ("y", vp)] + [(n, i64) for n in ("ldx", "bsx", "ldy", "bsy")] + \
               [(n, i32) for n in ("B", "T", "L", "C", "in_dtype", "out_dtype")]


class VqArgs(C.Structure):
    _fields_ = [("x", vp), ("codebook", vp), ("idx", vp), ("y", vp), ("ldx", i64), ("ldi", i64), ("ldy", i64)] + \
               [(n, i32) for n in ("R", "G", "K", "dg", "lookup", "pad_i")]


class CopyArgs(C.Structure):
    _fields_ = [("x", vp), ("y", vp)] + [(n, i64) for n in ("ldx", "bsx", "ldy", "bsy")] + \
               [(n, i32) for n in ("B", "R", "C", "in_dtype", "out_dtype", "pad_i")]


class Tensor(C.Structure):
    """stzs_tensor_t: (data, dtype, ndim, shape[4], stride[4] in elements)"""
    _fields_ = [("data", vp), ("dtype", i32), ("ndim", i32), ("shape", i64 * 4), ("stride", i64 * 4)]


class Params(C.Structure):
    _fields_ = [("i", i32 * 16), ("f", f32 * 8)]


PACK_KSTEP, PACK_LANE16, PACK_FRAG32, PACK_NARROW32, PACK_X3, PACK_FRAG32X3 = 0, 1, 2, 3, 4, 5
GENERIC_OPS = ["cfg_euler_step", "duration_head", "length_regulate", "sine_gen", "conv_post_istft", "bilstm",
               "conv_transpose_up", "mrf_resblock", "denoiser_fwd", "decoder_pre", "f0n_predictor"]
# input-list layouts of the composite generic operators (include/stzs.h STZS_DN_* / STZS_DP_* / STZS_FN_*)
DN_NIN_BASE, DN_PER_LAYER = 25, 16
DP_BLK0, DP_NIN = 10, 45
FN_BR0, FN_PER_BRANCH, FN_NIN = 7, 23, 53


def tensor(t, dtype=None) -> Tensor:
    """stzs_tensor_t of a torch tensor (device memory; dtype inferred unless given)."""
    import torch
    d = Tensor()
    d.data = t.data_ptr()
    # (packed weights travel as raw bytes: uint8 descriptors are tagged BF16, the packed element type)
    d.dtype = dtype if dtype is not None else {torch.float32: F32, torch.bfloat16: BF16, torch.int32: I32,
                                                torch.float8_e4m3fn: F8, torch.uint8: BF16}[t.dtype]
    d.ndim = t.dim()
    for k in range(t.dim()):
        d.shape[k] = t.shape[k]
        d.stride[k] = t.stride(k)
    return d


def params(ints=(), floats=()) -> Params:
    p = Params()
    for k, v in enumerate(ints):
        p.i[k] = int(v)
    for k, v in enumerate(floats):
        p.f[k] = float(v)
    return p


# every exported symbol of include/stzs.h (tests check the .so exports exactly these)
EXPORTS = ["stzs_init", "stzs_strerror", "stzs_version", "stzs_conv1d", "stzs_conv1d_group", "stzs_conv_splitk_workspace",
           "stzs_conv_rows_workspace",
           "stzs_chan_stats_workspace",
           "stzs_chan_stats", "stzs_chan_stats_partial", "stzs_chan_stats_final", "stzs_chan_stats_final_group", "stzs_row_layernorm", "stzs_ln_linear", "stzs_quant_rows", "stzs_attention", "stzs_lstm_workspace", "stzs_lstm", "stzs_lstm_pair",
           "stzs_lstm_state_reset", "stzs_predictor_prep",
           "stzs_durations", "stzs_alignment", "stzs_gather_rows", "stzs_adain_dwup", "stzs_f0n_down",
           "stzs_harmonic_source", "stzs_istft", "stzs_istft_stream", "stzs_istft_stream_span",
           "stzs_stft_frames", "stzs_log_mel", "stzs_pool_rows", "stzs_code_quantize",
           "stzs_dn_cond", "stzs_dn_cond_steps", "stzs_adaln_expand", "stzs_cfg_euler",
           "stzs_state_init", "stzs_mean_rows", "stzs_copy2d", "stzs_embed", "stzs_embed_f32", "stzs_dn_cond_steps_f32", "stzs_pack_conv_size", "stzs_pack_conv",
           "stzs_pack_lstm", "stzs_pack_lstm_x3"] + [f"stzs_{o}{sfx}" for o in GENERIC_OPS for sfx in ("", "_workspace")]

_lib = None


class StzsError(RuntimeError):
    pass


def load():
    """Load the HIP library (raises if it was not built — no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise StzsError(f"libstzs_hip.so not found at {LIB_PATH}: run `python styletts-zs_amd/build.py` "
                        "(the product path has no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    sig = {
        "stzs_init": ([i32], i32),
        "stzs_strerror": ([i32], C.c_char_p),
        "stzs_version": ([], i32),
        "stzs_conv1d": ([P(ConvArgs), vp], i32),
        "stzs_conv1d_group": ([P(ConvArgs), i32, vp], i32),
        "stzs_conv_splitk_workspace": ([i64, i32, i32], C.c_size_t),
        "stzs_conv_rows_workspace": ([i64, i32, i32], C.c_size_t),
        "stzs_chan_stats_workspace": ([i32, i32, i32], C.c_size_t),
        "stzs_chan_stats": ([P(StatsArgs), vp], i32),
        "stzs_chan_stats_partial": ([P(StatsArgs), vp], i32),
        "stzs_chan_stats_final": ([P(StatsArgs), i32, vp], i32),
        "stzs_chan_stats_final_group": ([P(StatsArgs), i32, i32, vp], i32),
        "stzs_row_layernorm": ([P(RowLNArgs), vp], i32),
        "stzs_ln_linear": ([P(ConvArgs), P(RowLNArgs), vp], i32),
        "stzs_quant_rows": ([P(QuantArgs), vp], i32),
        "stzs_attention": ([P(AttnArgs), vp], i32),
        "stzs_lstm_workspace": ([i32, i32, i32], C.c_size_t),
        "stzs_lstm": ([P(LstmArgs), vp], i32),
        "stzs_lstm_pair": ([P(LstmArgs), P(LstmArgs), vp], i32),
        "stzs_lstm_state_reset": ([vp, vp, vp], i32),
        "stzs_predictor_prep": ([P(PrPrepArgs), vp], i32),
        "stzs_durations": ([P(DurArgs), vp], i32),
        "stzs_alignment": ([P(AlignArgs), vp], i32),
        "stzs_gather_rows": ([P(GatherArgs), vp], i32),
        "stzs_adain_dwup": ([P(DwupArgs), vp], i32),
        "stzs_f0n_down": ([P(F0nArgs), vp], i32),
        "stzs_harmonic_source": ([P(SourceArgs), vp], i32),
        "stzs_istft": ([P(IstftArgs), vp], i32),
        "stzs_istft_stream": ([P(IstftStreamArgs), vp], i32),
        "stzs_istft_stream_span": ([i32, i32, i32, i32, i32, P(i64), P(i64)], i32),
        "stzs_stft_frames": ([P(FramesArgs), vp], i32),
        "stzs_log_mel": ([P(LogMelArgs), vp], i32),
        "stzs_pool_rows": ([P(PoolArgs), vp], i32),
        "stzs_code_quantize": ([P(VqArgs), vp], i32),
        "stzs_dn_cond_steps": ([vp, vp, vp, i32, i32, i32, vp], i32),
        "stzs_dn_cond_steps_f32": ([vp, vp, vp, i32, i32, i32, vp], i32),
        "stzs_dn_cond":([vp, vp, vp, i32, i32, vp], i32),
        "stzs_adaln_expand": ([vp, vp, vp, i32, i32, i32, i32, C.c_uint32, vp], i32),
        "stzs_cfg_euler": ([vp, vp, i32, i32, i32, f32, f32, f32, vp], i32),
        "stzs_state_init": ([vp, vp, i32, i32, i32, f32, vp], i32),
        "stzs_mean_rows": ([vp, vp, i32, i32, i64, i64, i32, i32, i64, vp], i32),
        "stzs_copy2d": ([P(CopyArgs), vp], i32),
        "stzs_embed": ([vp, vp, vp, i32, i32, i32, i64, vp], i32),
        "stzs_embed_f32": ([vp, vp, vp, i32, i32, i32, i64, vp], i32),
        "stzs_pack_conv_size": ([i32, i32, i32, i32, i32], C.c_size_t),
        "stzs_pack_conv": ([vp, i32, i32, i32, i32, i32, vp], i32),
        "stzs_pack_lstm": ([vp] * 8 + [i32, i32, vp, vp, vp], i32),
        "stzs_pack_lstm_x3": ([vp] * 8 + [i32, i32, vp, vp, vp], i32),
    }
    for o in GENERIC_OPS:
        sig[f"stzs_{o}"] = ([P(Tensor), i32, P(Tensor), i32, P(Params), vp, C.c_size_t, vp], i32)
        sig[f"stzs_{o}_workspace"] = ([P(Tensor), i32, P(Params)], C.c_size_t)
    for name, (argt, rest) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    _lib = L
    return L


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().stzs_strerror(rc).decode()
        raise StzsError(f"{what}: {msg} (rc={rc})")


def strerror(rc: int) -> str:
    return load().stzs_strerror(rc).decode()
