"""Phase timing of the batch-1 AdaIN-block conv (csrc/conv.hip conv_mfma, split-K over input-channel chunks) with
in-kernel s_memtime stamps.  A probe build with -DSTZS_CONV_PROF (`python tools/conv_phase.py --build`, in this
container) stamps per workgroup: entry, slice staged (+ DEEP: weights landed), K loop done, slab stored + drained,
ticket returned, combine done (last arriver), epilogue done; plus s_memrealtime (100 MHz) at entry / exit for the
dispatch spread.  Prints per phase the median / max over workgroups in shader cycles, and the launch span.

    python tools/conv_phase.py          (env: SPLITK=16, FLAGS=0 (65536: ring form))
"""
import ctypes as C
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
SO = os.path.join(ROOT, "tools", "probe", "libconvprof.so")
if "--build" in sys.argv:
    import concurrent.futures as cf

    import build as B  # noqa: E402
    tmp = os.path.join("/tmp", "convprof_build")
    os.makedirs(tmp, exist_ok=True)

    def one(f):
        o = os.path.join(tmp, os.path.basename(f) + ".o")
        subprocess.check_call([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get(os.path.basename(f), []) +
                              ["-DSTZS_CONV_PROF", "-c", f, "-o", o])
        return o
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, B.sources()))
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", SO + ".tmp"])
    os.replace(SO + ".tmp", SO)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

prof = C.CDLL(SO)
prof.stzs_conv1d.argtypes = [C.c_void_p, C.c_void_p]
prof.stzs_conv1d.restype = C.c_int
prof.stzs_conv_prof_read.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
NW = 16 * 8192
host = np.zeros(NW, dtype=np.uint64)


class Proxy:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, k):
        if k == "stzs_conv1d":
            return lambda aref, stream: prof.stzs_conv1d(C.addressof(aref._obj), stream)
        return getattr(self._lib, k)


eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
eng.lib = Proxy(eng.lib)
sk = int(os.environ.get("SPLITK", 16))
flags = int(os.environ.get("FLAGS", "0"), 0)
CASES = [(200, 514, 1024, "dec.enc.conv1"), (200, 1090, 1024, "dec.blk.conv1"), (400, 1090, 512, "dec.up.conv1"),
         (200, 512, 512, "pr.f0.0"), (400, 256, 256, "pr.f0.2")]
g = torch.Generator().manual_seed(0)
names = ["staged", "K loop", "slab drained", "ticket", "combine", "epilogue"]
for (T, Ci, Co, name) in CASES:
    w = torch.randn(Co, Ci, 3, generator=g) / math.sqrt(Ci * 3)
    A = Arena()
    cw = pack_conv(A, "a", w, torch.zeros(Co))
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    Cp = (Ci + 7) // 8 * 8
    x = Act(torch.randn(1, T, Cp, generator=g).to(torch.bfloat16).cuda(), 0, Ci)
    y = Act(torch.zeros(1, T, Co, dtype=torch.bfloat16, device="cuda:0"))
    mean = (torch.randn(1, Ci, generator=g) * 0.1).cuda()
    rstd = (torch.rand(1, Ci, generator=g) + 0.5).cuda()
    gb = (torch.randn(1, 2 * Ci, generator=g) * 0.2).cuda()

    def run():
        eng.conv(cw, x, y, pad=1, pro=(mean, rstd, Ci, gb.data_ptr(), 2 * Ci, Ci), pro_act=L.ACT_LEAKY, pro_slope=0.2,
                 stats_key="cp", splitk=sk, flags=flags)
    for _ in range(3):
        run()
    prof.stzs_conv_prof_read(None, 0, 1)
    run()
    prof.stzs_conv_prof_read(host.ctypes.data, NW, 0)
    st = host.reshape(-1, 16).astype(np.int64)
    st = st[st[:, 15] != 0]
    nwg = st.shape[0]
    last = st[:, 5] != 0
    d = {"staged": st[:, 1] - st[:, 0], "K loop": st[:, 2] - st[:, 1]}
    if sk > 1:
        d["slab drained"] = st[:, 3] - st[:, 2]
        d["ticket"] = st[:, 4] - st[:, 3]
        d["combine"] = st[last, 5] - st[last, 4]
    e = st[last]
    d["epi: acc->LDS"] = e[:, 7] - e[:, 5]
    d["epi: bias->LDS"] = e[:, 8] - e[:, 7]
    d["epi: pass 0"] = e[:, 9] - e[:, 8]
    d["epi: pass 1"] = e[:, 10] - e[:, 9]
    d["epi: stats out"] = e[:, 6] - e[:, 10]
    rt0, rt1 = st[:, 15], st[:, 14]
    print(f"{name:14s} T={T} Ci={Ci} Co={Co} sk={sk}: {nwg} workgroups, {int(last.sum())} last arrivers; entry spread "
          f"{(rt0.max() - rt0.min()) / 100:.2f} us, entry->exit median {np.median(rt1 - rt0) / 100:.2f} us max "
          f"{(rt1 - rt0).max() / 100:.2f} us, first entry -> last exit {(rt1.max() - rt0.min()) / 100:.2f} us", flush=True)
    for k, v in d.items():
        if len(v):
            print(f"    {k:14s} median {np.median(v):8.0f} cyc   max {v.max():8.0f} cyc", flush=True)
