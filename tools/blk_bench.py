"""Microbenchmark of the AdaIN residual-block convs (decoder pre-blocks and the F0 / N
predictor blocks; k3, AdaIN + LeakyReLU(0.2) prologue, 128-channel input chunks) on the LDS-ring MRF-family kernel
(csrc/mrf.hip, STZS_CONV_W_LANE16) vs the register-direct one (csrc/mrfv.hip, STZS_CONV_W_FRAG32): bit-identity of
output and fused statistics, then time per launch at the bench batch.

    python tools/blk_bench.py            (env: B=64, REPS=5)
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
reps = int(os.environ.get("REPS", 5))
# (name, T, Ci, Co, residual): v0 decoder pre-blocks (T40 = 200, T80 = 400) and predictor F0 / N blocks
SHAPES = [("dec.encode.conv1", 200, 514, 1024, False), ("dec.decode.conv1", 200, 1090, 1024, False),
          ("dec.decode.conv2", 200, 1024, 1024, True), ("dec.decode3.conv2", 400, 512, 512, True),
          ("pr.f0.0.conv1", 200, 512, 512, False), ("pr.f0.2.conv2", 400, 256, 256, True)]
g = torch.Generator().manual_seed(0)
for name, T, Ci, Co, hr in SHAPES:
    w = torch.randn(Co, Ci, 3, generator=g) / math.sqrt(Ci * 3)
    b = torch.randn(Co, generator=g) * 0.1
    A = Arena()
    c16 = pack_conv(A, "a", w, b, lane16=True)
    cfr = pack_conv(A, "b", w, b, frag32=True)
    A.finalize(dev)
    for cw in (c16, cfr):
        cw.w, cw.b = A[cw.w], A[cw.b]
    ldx = (Ci + 7) // 8 * 8
    x = Act(torch.randn(B, T, ldx, generator=g).to(dev, torch.bfloat16), 0, Ci)
    res = Act(torch.randn(B, T, Co, generator=g).to(dev, torch.bfloat16)) if hr else None
    Cs = (Ci + 7) // 8 * 8
    mean = (torch.randn(B, Cs, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(B, Cs, generator=g) + 0.5).to(dev)
    gb = (torch.randn(B, 2 * Cs, generator=g) * 0.2).to(dev)
    flops = 2.0 * B * T * Ci * Co * 3
    byt = 2.0 * B * T * (Ci + Co * (2 if hr else 1))
    outs = {}
    for form, cw in (("lane16", c16), ("mrfv", cfr)):
        y = Act(torch.zeros(B, T, Co, device=dev, dtype=torch.bfloat16))
        kw = dict(pad=1, pro=(mean, rstd, Cs, gb.data_ptr(), 2 * Cs, Cs), pro_act=L.ACT_LEAKY, pro_slope=0.2,
                  res=res, alpha=1.0 / math.sqrt(2.0) if hr else 1.0, stats_key=None if hr else "bb." + form)

        def run():
            return eng.conv(cw, x, y, **kw)
        r = run()
        torch.cuda.synchronize()
        st = r[1] if isinstance(r, tuple) else None
        outs[form] = (y.t.clone(), None if st is None else (st[0].clone(), st[1].clone()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"{name:18s} B={B} T={T} Ci={Ci} Co={Co} {form:7s}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  "
              f"{byt / us / 1e3:7.1f} GB/s", flush=True)
    a, c = outs["lane16"], outs["mrfv"]
    same = torch.equal(a[0], c[0]) and (a[1] is None or (torch.equal(a[1][0], c[1][0]) and torch.equal(a[1][1], c[1][1])))
    print("   lane16 == mrfv:", "bit-identical" if same else
          f"MISMATCH max |diff| {(a[0].float() - c[0].float()).abs().max().item():.3e}", flush=True)
