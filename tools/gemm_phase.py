"""Phase timing of the LDS-DMA linear GEMM (csrc/conv.hip gemm_glds) with in-kernel s_memtime stamps (VERDICT r3 item 6:
where the ~13-us fixed cost of a batch-64 denoiser linear goes).  A probe build of conv.hip with -DSTZS_GEMM_PROF
(`python tools/gemm_phase.py --build`, in this container) stamps, per workgroup: start, first K-step landed, K loop
done, epilogue stores issued, stores drained.  Prints per phase the median / p90 over workgroups (cycles and us at the
stamps' 100-MHz-equivalent s_memtime rate is NOT assumed: cycles are shader clocks; us uses the measured clock), the
start-time spread over workgroups (dispatch / tail), and the launch time from HIP events.

    python tools/gemm_phase.py          (env: M=3200,6400; CASES=ffn1,qkv,out,ffn2)
"""
import ctypes as C
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
SO = os.path.join(ROOT, "tools", "probe", "libgemmprof.so")
if "--build" in sys.argv:  # the whole library (conv.hip calls into the other kernels' launchers) with the stamps on
    src = os.path.join(ROOT, "styletts-zs_amd", "csrc")
    sys.path.insert(0, os.path.join(ROOT, "styletts-zs_amd"))
    import build as B  # noqa: E402
    objs = []
    tmp = os.path.join("/tmp", "gemmprof_build")
    os.makedirs(tmp, exist_ok=True)
    import concurrent.futures as cf

    def one(f):
        o = os.path.join(tmp, os.path.basename(f) + ".o")
        subprocess.check_call([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get(os.path.basename(f), []) +
                              ["-DSTZS_GEMM_PROF", "-c", f, "-o", o])
        return o
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, B.sources()))
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", SO + ".tmp"])
    os.replace(SO + ".tmp", SO)  # (a copy of the tree never sees a partial library)
    sys.exit(0)

import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

prof = C.CDLL(SO)
prof.stzs_gemm_prof_conv.argtypes = [C.c_void_p, C.c_void_p]
prof.stzs_gemm_prof_conv.restype = C.c_int
stamps = torch.zeros(1 << 20, dtype=torch.int64, device="cuda:0")


class Proxy:
    """the engine's library with stzs_conv1d sent to the probe build, the stamp buffer in splitk_ws"""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, k):
        if k == "stzs_conv1d":
            def f(aref, stream):
                a = aref._obj
                a.splitk_ws = stamps.data_ptr()
                return prof.stzs_gemm_prof_conv(C.addressof(a), stream)
            return f
        return getattr(self._lib, k)


eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
eng.lib = Proxy(eng.lib)
cases = {"ffn1": (512, 2048, torch.bfloat16, L.ACT_GELU, False), "qkv": (512, 1536, torch.bfloat16, L.ACT_NONE, False),
         "out": (512, 512, torch.float32, L.ACT_NONE, True), "ffn2": (2048, 512, torch.float32, L.ACT_NONE, True)}
sel = os.environ.get("CASES", "ffn1,qkv,out,ffn2").split(",")
for M in [int(v) for v in os.environ.get("M", "3200,6400").split(",")]:
    for name in sel:
        K, N, odt, act, gated = cases[name]
        w = torch.randn(N, K) / math.sqrt(K)
        A = Arena()
        cw = pack_conv(A, "g", w, torch.zeros(N))
        A.finalize("cuda:0")
        cw.w, cw.b = A[cw.w], A[cw.b]
        x = Act(torch.randn(M // 50, 50, K, device="cuda:0").to(torch.bfloat16))
        y = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt))
        res = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt)) if gated else None
        gate = torch.ones(M // 50, N, device="cuda:0")

        def run():
            eng.conv(cw, x, y, epi_act=act, res=res, gate=gate.data_ptr() if gated else None, gate_bs=N)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        stamps.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        st = stamps.view(-1, 8)[:, :7].cpu()
        st = st[(st != 0).all(dim=1)].double()  # workgroups that stamped all seven points
        n = st.shape[0]
        # (s_memtime counters are per XCD and not aligned across XCDs: only differences within a workgroup are used)
        ph = {"fill (start -> K-step 0 landed)": st[:, 1] - st[:, 0], "K loop": st[:, 2] - st[:, 1],
              "epi: accumulators -> LDS": st[:, 5] - st[:, 2], "epi: bias / gate -> LDS": st[:, 6] - st[:, 5],
              "epi: vector loop (issue)": st[:, 3] - st[:, 6], "store drain": st[:, 4] - st[:, 3],
              "workgroup total": st[:, 4] - st[:, 0]}
        print(f"{name:5s} M={M} K={K} N={N}: {n} workgroups stamped, launch {us:.1f} us (events)", flush=True)
        for k, v in ph.items():
            q = torch.quantile(v, torch.tensor([0.5, 0.9], dtype=torch.float64))
            print(f"    {k:34s} median {q[0].item():8.0f} cyc  p90 {q[1].item():8.0f} cyc", flush=True)
