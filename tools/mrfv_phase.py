"""Per-workgroup phase timeline of the stage-1 MRF conv (csrc/mrfv_kernel.hpp, NCH = 1 instances of csrc/mrfv_n1.hip)
from in-kernel stamps.  A probe build (`python tools/mrfv_phase.py --build`, in this container: mrfv_n1.hip with
-DSTZS_MRFV_PROF relinked with the in-tree objects into tools/variants/libmrfvprof.so) stamps per workgroup s_memtime at
entry, after the staging barrier, after the K loop, after the epilogue's stores issued and drained, s_memrealtime at
entry / exit and the CU (HW_ID, XCC_ID).  Prints, per shape: the phase durations (median / p90, shader cycles), the
clock, and per CU the time-averaged number of resident workgroups in each phase and the share of the launch with no
workgroup in its K loop (the MFMA pipe idle by construction) -- i.e. whether one workgroup's staging / epilogue runs
beside another's K loop, or the co-resident workgroups move in phase.

    STZS_LIB=tools/variants/libmrfvprof.so python tools/mrfv_phase.py      (env: B=64, CASES=0,3)
"""
import ctypes as C
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
SO = os.path.join(ROOT, "tools", "variants", "libmrfvprof.so")
if "--build" in sys.argv:
    import build as B  # noqa: E402
    # --diag 2: the staging without its row loads (transform + LDS stores only; the early-load stage-1 path)
    diag = sys.argv[sys.argv.index("--diag") + 1] if "--diag" in sys.argv else "0"
    if diag != "0":
        SO = SO.replace(".so", f"_diag{diag}.so")
    obj = os.path.join("/tmp", f"mrfv_n1_prof{diag}.o")
    subprocess.check_call([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get("mrfv_n1.hip", []) +
                          ["-DSTZS_MRFV_PROF", f"-DSTZS_MRFV_DIAG={diag}", "-c", os.path.join(B.CSRC, "mrfv_n1.hip"), "-o", obj])
    objs = [obj if os.path.basename(s) == "mrfv_n1.hip" else os.path.join(B.BUILD, os.path.basename(s).replace(".hip", ".o"))
            for s in B.sources()]
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", SO + ".tmp"])
    os.replace(SO + ".tmp", SO)
    print(SO)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

assert os.path.basename(L.LIB_PATH).startswith("libmrfvprof"), "run with STZS_LIB=tools/variants/libmrfvprof[_diagN].so"
lib = L.load()
lib.stzs_mrfv_prof_read.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
lib.stzs_mrfv_prof_read.restype = C.c_int
NW = 8 * 16384
dev = "cuda:0"
eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=dev)
B = int(os.environ.get("B", 64))
ALL = [(24001, 128, 3, 1), (24001, 128, 3, 5), (24001, 128, 7, 3), (24001, 128, 11, 5)]
cases = [ALL[int(i)] for i in os.environ.get("CASES", "0,3").split(",")]
g = torch.Generator().manual_seed(0)
host = np.zeros(NW, dtype=np.uint64)
for (T, C_, k, dil) in cases:
    w = torch.randn(C_, C_, k, generator=g) / math.sqrt(C_ * k)
    A = Arena()
    cw = pack_conv(A, "b", w, torch.zeros(C_), frag32=True)
    A.finalize(dev)
    cw.w, cw.b = A[cw.w], A[cw.b]
    x = Act(torch.randn(B, T, C_, generator=g).to(dev, torch.bfloat16))
    y = Act(torch.zeros(B, T, C_, device=dev, dtype=torch.bfloat16))
    mean = (torch.randn(B, C_, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(B, C_, generator=g) + 0.5).to(dev)
    gb = (torch.randn(B, 2 * C_, generator=g) * 0.2).to(dev)
    al = (torch.rand(C_, generator=g) + 0.5).to(dev)
    kw = dict(pad=dil * (k - 1) // 2, dil=dil, pro=(mean, rstd, C_, gb.data_ptr(), 2 * C_, C_), pro_act=L.ACT_SNAKE,
              pro_alpha=al, stats_key="mp")
    for _ in range(5):
        eng.conv(cw, x, y, **kw)
    torch.cuda.synchronize()
    assert lib.stzs_mrfv_prof_read(None, 0, 1) == 0
    eng.conv(cw, x, y, **kw)
    assert lib.stzs_mrfv_prof_read(host.ctypes.data, NW, 1) == 0
    nwg = B * ((T + 127) // 128)
    st = host[:nwg * 8].reshape(nwg, 8).astype(np.int64)
    assert (st[:, 6] > 0).all(), "missing stamps"
    cyc = lambda i, j: st[:, j] - st[:, i]
    phases = dict(stage=cyc(0, 1), kloop=cyc(1, 2), epilogue=cyc(2, 3), drain=cyc(3, 4), total=cyc(0, 4))
    rt0, rt1 = st[:, 5], st[:, 6]
    span_us = (rt1.max() - rt0.min()) / 100.0
    clk = (st[:, 4] - st[:, 0]) / np.maximum(rt1 - rt0, 1) / 10.0  # cycles per ns = GHz
    print(f"== stage-1 k{k} d{dil} c1, B {B}: {nwg} workgroups, launch span {span_us:.1f} us, clock median "
          f"{np.median(clk):.2f} GHz", flush=True)
    for n_, v in phases.items():
        print(f"   {n_:9s} cycles: median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    # per-CU timeline on the realtime clock (10 ns): phase boundaries placed by the workgroup's own clock
    ratio = (st[:, 4] - st[:, 0]) / np.maximum(rt1 - rt0, 1)
    tb = [rt0 + (st[:, i] - st[:, 0]) / ratio for i in range(5)]  # entry, staged, kloop end, epilogue end, drained
    cu = (st[:, 7] >> 32) * 256 + ((st[:, 7] >> 8) & 0xFF)
    t_lo, t_hi = rt0.min(), rt1.max()
    grid = np.arange(t_lo, t_hi, 10)  # 100 ns steps
    occ = {p: [] for p in ("stage", "kloop", "epi", "resident")}
    none_k, cus = [], np.unique(cu)
    for c in cus:
        m = cu == c
        cnt = {p: np.zeros(len(grid)) for p in occ}
        for s0, s1, s2, s4 in zip(tb[0][m], tb[1][m], tb[2][m], tb[4][m]):
            cnt["stage"] += (grid >= s0) & (grid < s1)
            cnt["kloop"] += (grid >= s1) & (grid < s2)
            cnt["epi"] += (grid >= s2) & (grid < s4)
            cnt["resident"] += (grid >= s0) & (grid < s4)
        act = cnt["resident"] > 0
        for p in occ:
            occ[p].append(cnt[p][act].mean())
        none_k.append(((cnt["kloop"] == 0) & act).mean() / max(act.mean(), 1e-9))
    print(f"   per CU ({len(cus)} CUs, time-averaged while any workgroup is resident): resident {np.mean(occ['resident']):.2f}, "
          f"staging {np.mean(occ['stage']):.2f}, K loop {np.mean(occ['kloop']):.2f}, epilogue+drain {np.mean(occ['epi']):.2f}; "
          f"share of time with NO workgroup in its K loop {np.mean(none_k):.3f}", flush=True)
    # entry skew of co-resident workgroups: in the first round, entries per CU
    first = np.argsort(rt0)[:len(cus) * 3]
    print(f"   first-round entry spread {(rt0[first].max() - rt0[first].min()) / 100:.2f} us; "
          f"median workgroup lifetime {np.median(rt1 - rt0) / 100:.2f} us", flush=True)
