"""Register-direct MRF conv (csrc/mrfv.hip, STZS_CONV_W_FRAG32) and the LDS-ring MRF conv (csrc/mrf.hip, STZS_CONV_W_LANE16) on the generator shapes: bit-identity of outputs and fused statistics, then time per launch.

    python tools/mrfv_bench.py            (env: B=64, CASES=0,1,2,..., FLAGS=0, REPS=5)
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
ALL = [(24001, 128, 3, 1), (24001, 128, 3, 5), (24001, 128, 7, 3), (24001, 128, 11, 5),
       (4000, 256, 3, 1), (4000, 256, 7, 3), (4000, 256, 11, 5)]
cases = [ALL[int(i)] for i in os.environ.get("CASES", ",".join(str(i) for i in range(len(ALL)))).split(",")]
flags = int(os.environ.get("FLAGS", "0"), 0)
reps = int(os.environ.get("REPS", 5))
g = torch.Generator().manual_seed(0)
for (T, C, k, dil) in cases:
    w = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    b = torch.randn(C, generator=g) * 0.1
    A = Arena()
    c16 = pack_conv(A, "a", w, b, lane16=True)
    cfr = pack_conv(A, "b", w, b, frag32=True)
    A.finalize(dev)
    for cw in (c16, cfr):
        cw.w, cw.b = A[cw.w], A[cw.b]
    x = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
    res = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
    acc = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
    mean = (torch.randn(B, C, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(B, C, generator=g) + 0.5).to(dev)
    gb = (torch.randn(B, 2 * C, generator=g) * 0.2).to(dev)
    al = (torch.rand(C, generator=g) + 0.5).to(dev)
    flops = 2.0 * B * T * C * C * k
    byt = 2.0 * B * T * C * 2
    for variant in ("c1", "c2", "c2acc"):
        outs = {}
        forms = [("lane16", c16, 0), ("mrfv", cfr, 0)]
        # two chunks: also the narrow (128 channels per workgroup) register-direct form
        if C != 128:
            forms.append(("mrfvN", cfr, L.CONV_MRFV_NARROW))
        for name, cw, fl in forms:
            y = Act(torch.zeros(B, T, C, device=dev, dtype=torch.bfloat16))
            kw = dict(pad=dil * (k - 1) // 2, dil=dil, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C),
                      pro_act=L.ACT_SNAKE, pro_alpha=al, flags=flags | fl)
            if variant != "c1":
                kw["res"] = res
            if variant == "c2acc":
                kw.update(acc_in=acc, beta=1.0, alpha=1.0 / 3)
            if variant != "c2acc":
                kw["stats_key"] = "mb." + name

            def run():
                return eng.conv(cw, x, y, **kw)
            r = run()
            torch.cuda.synchronize()
            st = r[1] if isinstance(r, tuple) else None
            outs[name] = (y.t.clone(), None if st is None else (st[0].clone(), st[1].clone()))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            nb = byt * (1 + (variant != "c1") + (variant == "c2acc") * 0.5)
            print(f"T={T} C={C} k={k:2d} d={dil} {variant:6s} {name:7s}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  "
                  f"{nb / us / 1e3:7.1f} GB/s", flush=True)
        a = outs["lane16"]
        for other in [f[0] for f in forms[1:]]:
            bb = outs[other]
            same = torch.equal(a[0], bb[0]) and (a[1] is None or (torch.equal(a[1][0], bb[1][0]) and
                                                                   torch.equal(a[1][1], bb[1][1])))
            if not same:
                d = (a[0].float() - bb[0].float()).abs().max().item()
                print(f"   MISMATCH lane16 vs {other}: max |diff| {d:.3e}", flush=True)
            else:
                print(f"   lane16 == {other}: bit-identical", flush=True)
