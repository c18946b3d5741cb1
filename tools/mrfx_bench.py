"""Precise-mode MRF convs on the generator shapes: the register-direct split-operand kernel (csrc/mrfx.hip,
STZS_CONV_W_FRAG32X3) vs the LDS-ring split-operand conv_x3 (csrc/convx.hip, STZS_CONV_W_X3), fp32 activations,
B = 64: time per launch (HIP events over REPS launches), bf16x3-equivalent TFLOP/s (3 bf16 products per fp32 product),
fp32 bytes (input once, output once, + residual, + accumulate), the fraction of the per-launch roofline
max(F / 2.5 PF, bytes / 8 TB/s), and the max |difference| between the two forms.

    python tools/mrfx_bench.py            (env: B=64, CASES=0,1,..., REPS=3, FLAGS=0 (4: K loop + staging only))
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
B = int(os.environ.get("B", 64))
ALL = [(24001, 128, 3, 1), (24001, 128, 3, 5), (24001, 128, 7, 3), (24001, 128, 7, 5), (24001, 128, 11, 1),
       (24001, 128, 11, 5), (4000, 256, 3, 1), (4000, 256, 7, 3), (4000, 256, 11, 5)]
cases = [ALL[int(i)] for i in os.environ.get("CASES", ",".join(str(i) for i in range(len(ALL)))).split(",")]
reps = int(os.environ.get("REPS", 3))
flags = int(os.environ.get("FLAGS", "0"), 0)
g = torch.Generator().manual_seed(0)
for (T, C, k, dil) in cases:
    w = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    b = torch.randn(C, generator=g) * 0.1
    A = Arena()
    cw = pack_conv(A, "a", w, b, frag32=True, x3=True)
    A.finalize(dev)
    cw.w, cw.wx3, cw.fx3, cw.b = A[cw.w], A[cw.wx3], A[cw.fx3], A[cw.b]
    x = Act(torch.randn(B, T, C, generator=g).to(dev))
    res = Act(torch.randn(B, T, C, generator=g).to(dev))
    acc = Act(torch.randn(B, T, C, generator=g).to(dev))
    mean = (torch.randn(B, C, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(B, C, generator=g) + 0.5).to(dev)
    gb = (torch.randn(B, 2 * C, generator=g) * 0.2).to(dev)
    al = (torch.rand(C, generator=g) + 0.5).to(dev)
    flops = 3 * 2.0 * B * T * C * C * k
    for variant in ("c1", "c2", "c2acc"):
        outs = {}
        for name, mx in (("mrfx", True), ("conv_x3", False)):
            eng.mrfx = mx
            y = Act(torch.zeros(B, T, C, device=dev))
            kw = dict(pad=dil * (k - 1) // 2, dil=dil, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C),
                      pro_act=L.ACT_SNAKE, pro_alpha=al, flags=flags if mx else 0)
            if variant != "c1":
                kw["res"] = res
            if variant == "c2acc":
                kw.update(acc_in=acc, beta=1.0, alpha=1.0 / 3)
            else:
                kw["stats_key"] = "mb." + name

            def run():
                return eng.conv(cw, x, y, **kw)
            run()
            torch.cuda.synchronize()
            outs[name] = y.t.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            nb = 4.0 * B * T * C * (2 + (variant != "c1") + (variant == "c2acc"))
            roof = max(flops / 2.5e15, nb / 8e12) * 1e6
            print(f"T={T} C={C} k={k:2d} d={dil} {variant:6s} {name:8s}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s(x3)  "
                  f"{nb / us / 1e3:7.1f} GB/s  roof frac {roof / us:.3f}", flush=True)
        d = (outs["mrfx"] - outs["conv_x3"]).abs().max().item() / outs["conv_x3"].abs().max().item()
        print(f"   mrfx vs conv_x3: max |diff| / max|y| {d:.2e}", flush=True)
