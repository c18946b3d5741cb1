"""C-ABI checks that need no GPU: the library loads, exports exactly what include/stzs.h declares,
the ctypes structures match the C layouts (sizeof/offsetof compiled with gcc from the header), and
error codes are named.  No compute call is made here."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT


HEADERS = ("stzs.h",)


def _header(name="stzs.h"):
    return open(os.path.join(ROOT, "include", name)).read()


def test_library_exports_every_declared_symbol():
    from stzs import _lib
    assert sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")) == sorted(HEADERS)
    decl = set(re.findall(r"\b(stzs_[a-z0-9_]+)\s*\(", _header()))
    assert decl == set(_lib.EXPORTS), decl ^ set(_lib.EXPORTS)
    L = _lib.load()
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(stzs_[a-z0-9_]+)\b", nm))
    assert decl <= exported, decl - exported
    for s in decl:
        getattr(L, s)


def test_strerror_and_version():
    from stzs import _lib
    L = _lib.load()
    assert L.stzs_version() >= 1
    assert _lib.strerror(0) == "ok"
    for rc in (-1, -2, -3, -4):
        assert _lib.strerror(rc).startswith("STZS_E")


def test_workspace_queries():
    from stzs import _lib
    L = _lib.load()
    assert L.stzs_chan_stats_workspace(64, 24001, 128) == 64 * 94 * 128 * 8
    # groups x dirs x 2 buffers x 64 rows x (hi | lo) H bf16: sized for the precise split-operand rows
    # (+ the small-batch tagged-granule region: [dir][parity][2 rows][H/2 <= 128] u64 = 8 KB)
    assert L.stzs_lstm_workspace(64, 256, 2) == 8192 + 2 * 2 * 64 * 2 * 256 * 2
    # split-K slabs: ceil(rows / 64) x (co_pad / 128) tiles x splitk slices x 64 x 128 fp32; bad arguments -> 0
    assert L.stzs_conv_splitk_workspace(100, 512, 4) == 2 * 4 * 4 * 64 * 128 * 4
    assert L.stzs_conv_splitk_workspace(6400, 1536, 2) == 100 * 12 * 2 * 64 * 128 * 4
    assert L.stzs_conv_splitk_workspace(100, 500, 4) == 0 and L.stzs_conv_splitk_workspace(100, 512, 3) == 0
    assert L.stzs_conv_splitk_workspace(0, 512, 2) == 0


STRUCTS = {
    "stzs_conv_args": "ConvArgs", "stzs_stats_args": "StatsArgs", "stzs_rowln_args": "RowLNArgs",
    "stzs_attn_args": "AttnArgs", "stzs_lstm_args": "LstmArgs", "stzs_prprep_args": "PrPrepArgs",
    "stzs_dur_args": "DurArgs", "stzs_align_args": "AlignArgs", "stzs_gather_args": "GatherArgs",
    "stzs_dwup_args": "DwupArgs", "stzs_f0n_args": "F0nArgs", "stzs_source_args": "SourceArgs",
    "stzs_istft_args": "IstftArgs", "stzs_istft_stream_args": "IstftStreamArgs", "stzs_quant_args": "QuantArgs", "stzs_frames_args": "FramesArgs",
    "stzs_logmel_args": "LogMelArgs", "stzs_pool_args": "PoolArgs", "stzs_copy_args": "CopyArgs",
    "stzs_vq_args": "VqArgs", "stzs_tensor_t": "Tensor", "stzs_params_t": "Params",
}


def test_ctypes_structs_match_c_layout():
    """compile a probe with gcc against include/stzs.h and compare sizeof + every field offset."""
    from stzs import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "stzs.h"', "int main(void){"]
    for cname, pyname in STRUCTS.items():
        py = getattr(_lib, pyname)
        lines.append(f'printf("{pyname} size %zu\\n", sizeof({cname}));')
        for f, _t in py._fields_:
            lines.append(f'printf("{pyname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        open(src, "w").write("\n".join(lines))
        r = subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        out = subprocess.run([exe], capture_output=True, text=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln.strip():
            a, b, c = ln.split()
            got[(a, b)] = int(c)
    for cname, pyname in STRUCTS.items():
        py = getattr(_lib, pyname)
        assert got[(pyname, "size")] == C.sizeof(py), pyname
        for f, _t in py._fields_:
            assert got[(pyname, f)] == getattr(py, f).offset, (pyname, f)


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    """the product path refuses to run without the HIP library (no silent CPU fallback)."""
    from stzs import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.StzsError):
        _lib.load()
    # (monkeypatch restores the loaded handle; a module reload here would orphan its ctypes argtypes)


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "styletts-zs_amd", "stzs")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, re.M), f


@pytest.mark.parametrize("Tf,chunks", [(24001, [4000] * 6 + [1]), (144001, [24000] * 6 + [1]), (9, [1, 1, 2, 5]),
                                       (257, [256, 1]), (300, [2, 298])])
def test_istft_stream_spans_tile_the_output(Tf, chunks):
    """host-side span query (no GPU): the chunks' [n0, n1) tile [0, (Tf-1)*hop) exactly (row a14)."""
    from stzs import _lib
    L = _lib.load()
    assert sum(chunks) == Tf
    n0, n1 = C.c_int64(), C.c_int64()
    f0, nxt = 0, 0
    for i, Fc in enumerate(chunks):
        halo = L.stzs_istft_stream_span(f0, Fc, int(i == len(chunks) - 1), 20, 5, C.byref(n0), C.byref(n1))
        assert halo == 3
        assert n0.value == nxt and n1.value >= n0.value
        nxt = n1.value
        f0 += Fc
    assert nxt == (Tf - 1) * 5
    assert L.stzs_istft_stream_span(0, 0, 1, 20, 5, C.byref(n0), C.byref(n1)) == _lib.ESHAPE


_STRUCT_CALLS = [  # entry point, ctypes struct, extra int arguments between the struct and the stream
    ("stzs_conv1d", "ConvArgs", ()), ("stzs_chan_stats", "StatsArgs", ()), ("stzs_chan_stats_partial", "StatsArgs", ()),
    ("stzs_chan_stats_final", "StatsArgs", (64,)), ("stzs_row_layernorm", "RowLNArgs", ()),
    ("stzs_quant_rows", "QuantArgs", ()), ("stzs_attention", "AttnArgs", ()), ("stzs_lstm", "LstmArgs", ()),
    ("stzs_predictor_prep", "PrPrepArgs", ()), ("stzs_durations", "DurArgs", ()),
    ("stzs_alignment", "AlignArgs", ()), ("stzs_gather_rows", "GatherArgs", ()),
    ("stzs_adain_dwup", "DwupArgs", ()), ("stzs_f0n_down", "F0nArgs", ()),
    ("stzs_harmonic_source", "SourceArgs", ()), ("stzs_istft", "IstftArgs", ()),
    ("stzs_istft_stream", "IstftStreamArgs", ()), ("stzs_stft_frames", "FramesArgs", ()),
    ("stzs_log_mel", "LogMelArgs", ()), ("stzs_pool_rows", "PoolArgs", ()), ("stzs_copy2d", "CopyArgs", ()),
    ("stzs_code_quantize", "VqArgs", ()),
]


@pytest.mark.parametrize("name,struct,extra", _STRUCT_CALLS)
def test_entry_points_reject_before_launch(name, struct, extra):
    """SURVEY §8(b) 'Errors': every compute entry point validates its arguments before any HIP call, so a
    bad call returns a code (never launches, never crashes) -- checkable without a GPU.  NULL args and
    NULL required pointers -> STZS_EINVAL; every pointer set but an empty batch / zero sizes ->
    STZS_ESHAPE."""
    from stzs import _lib
    L = _lib.load()
    fn = getattr(L, name)
    S = getattr(_lib, struct)
    assert fn(None, *extra, None) == _lib.EINVAL
    a = S()  # all zero: required pointers NULL
    assert fn(C.byref(a), *extra, None) == _lib.EINVAL
    for f, ct in S._fields_:
        if ct is C.c_void_p:  # (every pointer field of the bindings is a void*)
            setattr(a, f, 0x1000)
    if name == "stzs_conv1d":
        a.cic = 128  # (the K-step width is validated first: EINVAL)
    assert fn(C.byref(a), *extra, None) == _lib.ESHAPE  # sizes all 0: rejected, nothing dereferenced


def test_groups_reject_before_launch():
    """stzs_conv1d_group / stzs_chan_stats_final_group: NULL arrays and n outside 1..3 -> STZS_EINVAL; problems with
    NULL pointers or empty shapes are rejected by their own checks (the grouped form is only taken after every
    problem passes stzs_conv1d's checks) -- all before any HIP call."""
    from stzs import _lib
    L = _lib.load()
    E, S = _lib.EINVAL, _lib.ESHAPE
    a = (_lib.ConvArgs * 3)()
    assert L.stzs_conv1d_group(None, 3, None) == E
    assert L.stzs_conv1d_group(a, 0, None) == E and L.stzs_conv1d_group(a, 4, None) == E
    assert L.stzs_conv1d_group(a, 3, None) == E and L.stzs_conv1d_group(a, 2, None) == E  # NULL x / w / y
    for p in a:
        p.x, p.w, p.y, p.flags = 0x1000, 0x2000, 0x3000, _lib.CONV_W_FRAG32
    assert L.stzs_conv1d_group(a, 3, None) == S  # empty shapes: the first problem's own checks
    st = (_lib.StatsArgs * 2)()
    assert L.stzs_chan_stats_final_group(None, 2, 64, None) == E
    assert L.stzs_chan_stats_final_group(st, 0, 64, None) == E and L.stzs_chan_stats_final_group(st, 2, 0, None) == E
    assert L.stzs_chan_stats_final_group(st, 2, 64, None) == E  # NULL mean / rstd / partial
    for p in st:
        p.mean, p.rstd, p.partial = 0x1000, 0x2000, 0x3000
    assert L.stzs_chan_stats_final_group(st, 2, 64, None) == S


def test_lstm_pair_rejects_before_launch():
    """stzs_lstm_pair: each recurrence validated as stzs_lstm validates it, then the pair -- one shape class (B, H,
    ndir, precise) and separate exchange state -- all before any HIP call."""
    from stzs import _lib
    L = _lib.load()
    E, S = _lib.EINVAL, _lib.ESHAPE

    def ok_args(base):
        a = _lib.LstmArgs()
        a.gx, a.whhT, a.y, a.xchg, a.sync = base, base + 0x100, base + 0x200, base + 0x300, base + 0x400
        a.ldg, a.bsg, a.ldy, a.bsy, a.B, a.T, a.H, a.ndir = 1024, 8192, 256, 2048, 1, 8, 128, 2
        return a
    a, b = ok_args(0x10000), ok_args(0x20000)
    assert L.stzs_lstm_pair(None, C.byref(b), None) == E and L.stzs_lstm_pair(C.byref(a), None, None) == E
    b.H = 64
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == S  # shape classes differ
    b.H, b.B = 128, 2
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == S
    b.B, b.precise = 1, 1
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == S
    b.precise, b.xchg = 0, a.xchg
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == E  # shared exchange workspace
    b.xchg, b.sync = 0x20300, a.sync
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == E  # shared sync words
    b.sync, b.T = 0x20400, 0
    assert L.stzs_lstm_pair(C.byref(a), C.byref(b), None) == S  # the second recurrence's own checks


def test_scalar_entry_points_reject_before_launch():
    from stzs import _lib
    L = _lib.load()
    p = C.c_void_p(0x1000)
    E, S = _lib.EINVAL, _lib.ESHAPE
    assert L.stzs_dn_cond(None, p, p, 1, 1, None) == E and L.stzs_dn_cond(p, p, p, 0, 1, None) == S
    assert L.stzs_dn_cond_steps(p, None, p, 1, 1, 1, None) == E and L.stzs_dn_cond_steps(p, p, p, 1, 1, 0, None) == S
    assert L.stzs_adaln_expand(None, p, p, 1, 1, 1, 1, 0, None) == E
    assert L.stzs_adaln_expand(p, p, p, 1, 1, 33, 1, 0, None) == S  # nchunk <= 32
    assert L.stzs_cfg_euler(p, None, 1, 1, 0, 1.0, 1.0, 0.5, None) == E
    assert L.stzs_cfg_euler(p, p, 1, 1, 0, 1.0, 0.0, 0.5, None) == S  # sigma must be > 0
    assert L.stzs_state_init(None, p, 1, 1, 0, 1.0, None) == E and L.stzs_state_init(p, p, 0, 1, 0, 1.0, None) == S
    assert L.stzs_mean_rows(p, None, 1, 1, 8, 8, 0, 8, 8, None) == E
    assert L.stzs_mean_rows(p, p, 1, 0, 8, 8, 0, 8, 8, None) == S
    assert L.stzs_embed(p, p, None, 1, 1, 8, 8, None) == E and L.stzs_embed(p, p, p, 1, 0, 8, 8, None) == S
