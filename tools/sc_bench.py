"""The AdaIN blocks' 1x1 shortcut convs on the decoder shapes: the LDS-DMA GEMM path (generic K-step packing) vs the
register-direct block-conv form (STZS_CONV_W_FRAG32, ks 1) -- outputs compared, time per launch.

    python tools/sc_bench.py            (env: B=64, REPS=10)
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

dev = "cuda:0"
eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=dev)
B = int(os.environ.get("B", 64))
reps = int(os.environ.get("REPS", 10))
g = torch.Generator().manual_seed(0)
for (T, Ci, Co) in [(200, 1090, 1024), (200, 514, 1024), (200, 1090, 512), (100, 1090, 1024)]:
    w = torch.randn(Co, Ci, 1, generator=g) / math.sqrt(Ci)
    A = Arena()
    ck = pack_conv(A, "k", w)
    cf = pack_conv(A, "f", w, frag32=True)
    A.finalize(dev)
    for cw in (ck, cf):
        cw.w = A[cw.w]
    ld = (Ci + 7) // 8 * 8 + 8 * 8  # (a wider row buffer, as the decoder's concatenation buffers are)
    xb = torch.zeros(B, T, ld)
    xb[..., :Ci] = torch.randn(B, T, Ci, generator=g)
    x = Act(xb.to(dev, torch.bfloat16), 0, Ci)
    outs = {}
    for name, cw in (("gemm", ck), ("frag32", cf)):
        y = Act(torch.zeros(B, T, Co, device=dev, dtype=torch.bfloat16))
        eng.conv(cw, x, y)
        torch.cuda.synchronize()
        outs[name] = y.t.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            eng.conv(cw, x, y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        fl = 2.0 * B * T * Ci * Co
        print(f"B={B} T={T} {Ci:4d} -> {Co:4d} {name:6s}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    ref = torch.einsum("btc,oc->bto", x.t[..., :Ci].float().cpu(), w[:, :, 0])
    for name, o in outs.items():
        err = (o.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
        print(f"   {name:6s} max-rel vs fp32 {err:.2e}", flush=True)
    print(f"   gemm == frag32: {torch.equal(outs['gemm'], outs['frag32'])}", flush=True)
