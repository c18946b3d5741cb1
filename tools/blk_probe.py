"""Batch-1 AdaIN-block conv probe (the latency engine's split-K conv_mfma, csrc/conv.hip): time per launch of the
decoder / predictor block conv shapes at B = 1 (HIP events over REPS launches), with the diagnostic flag bits
(1: no staging, 2: no K loop, 4: no epilogue) to split the time, and the ring depth from the launcher.

    python tools/blk_probe.py            (env: SPLITK=8, REPS=50, FLAGS="0,1,2,4", B=1, FRAG32=0)
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

dev = "cuda:0"
eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=dev)
sk = int(os.environ.get("SPLITK", 8))
B = int(os.environ.get("B", 1))
frag = os.environ.get("FRAG32", "0") != "0"  # the register-direct form (mrfv) of the throughput engine, no split
reps = int(os.environ.get("REPS", 50))
flag_list = [int(f, 0) for f in os.environ.get("FLAGS", "0,1,2,4").split(",")]
# (T, Ci, Co, name): decoder encode / decode block convs at T40 = 200, predictor F0/N blocks
CASES = [(200, 514, 1024, "dec.enc.conv1"), (200, 1024, 1024, "dec.enc.conv2"), (200, 1090, 1024, "dec.blk.conv1"),
         (400, 1090, 512, "dec.up.conv1"), (400, 512, 512, "dec.up.conv2"), (200, 512, 512, "pr.f0.0"),
         (400, 512, 256, "pr.f0.1"), (400, 256, 256, "pr.f0.2")]
g = torch.Generator().manual_seed(0)
for (T, Ci, Co, name) in CASES:
    w = torch.randn(Co, Ci, 3, generator=g) / math.sqrt(Ci * 3)
    b = torch.randn(Co, generator=g) * 0.1
    A = Arena()
    cw = pack_conv(A, "a", w, b, frag32=frag)
    A.finalize(dev)
    cw.w, cw.b = A[cw.w], A[cw.b]
    Cp = (Ci + 7) // 8 * 8
    x = Act(torch.randn(B, T, Cp, generator=g).to(torch.bfloat16).to(dev), 0, Ci)
    ske = 0 if frag else min(sk, cw.ci_pad // cw.cic)
    y = Act(torch.zeros(B, T, Co, dtype=torch.bfloat16, device=dev))
    mean = (torch.randn(B, Ci, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(B, Ci, generator=g) + 0.5).to(dev)
    gb = (torch.randn(B, 2 * Ci, generator=g) * 0.2).to(dev)
    line = []
    for fl in flag_list:
        def run():
            return eng.conv(cw, x, y, pad=1, pro=(mean, rstd, Ci, gb.data_ptr(), 2 * Ci, Ci), pro_act=L.ACT_LEAKY,
                            pro_slope=0.2, stats_key="bp", splitk=ske, flags=fl)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        line.append(f"flags {fl}: {e0.elapsed_time(e1) / reps * 1e3:6.1f} us")
    mb = Co * cw.ci_pad * 3 * 2 / 1e6
    print(f"{name:14s} sk={ske} T={T} Ci={Ci} Co={Co} w {mb:5.2f} MB  " + "  ".join(line), flush=True)
