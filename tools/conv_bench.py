"""Microbenchmark of the MRF conv shapes (stage 1: B=64, T=24001, C=128) with ablation flags.
flags: 1 = skip input staging, 2 = one tap only, 4 = skip epilogue stores, 128 = no XCD remap."""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
B = int(os.environ.get("B", 64))
cases = [(24001, 128, 3, 1), (24001, 128, 11, 5), (4000, 256, 3, 1), (4000, 256, 11, 5)]
if os.environ.get("CASE"):
    cases = [cases[int(os.environ["CASE"])]]
FLAGS = [int(f, 0) for f in os.environ.get("FLAGS", "0,128,1,2,4,3,6,5,7").split(",")]
for (T, C, k, dil) in cases:
    w = torch.randn(C, C, k) / math.sqrt(C * k)
    A = Arena()
    cw = pack_conv(A, "t", w, torch.zeros(C), lane16=os.environ.get("L16", "1") == "1")
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    x = Act(torch.randn(B, T, C, device="cuda:0").to(torch.bfloat16))
    y = Act(torch.empty(B, T, C, device="cuda:0", dtype=torch.bfloat16))
    mean = torch.zeros(B, C, device="cuda:0")
    rstd = torch.ones(B, C, device="cuda:0")
    gb = torch.zeros(B, 2 * C, device="cuda:0")
    al = torch.ones(C, device="cuda:0")
    flops = 2.0 * B * T * C * C * k
    for flags in FLAGS:
        def run():
            eng.conv(cw, x, y, pad=dil * (k - 1) // 2, dil=dil, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C),
                     pro_act=L.ACT_SNAKE, pro_alpha=al, flags=flags,
                     res=(x if os.environ.get("RES") == "1" else None),
                     stats_key=("bench.st" if os.environ.get("STATS") == "1" else None))
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 5
        e0.record()
        for _ in range(n):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        print(f"T={T} C={C} k={k} dil={dil} flags={flags}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)
