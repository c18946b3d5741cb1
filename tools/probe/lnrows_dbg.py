"""debug: where the fused LayerNorm image differs from stzs_row_layernorm at C = 1024"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd"), os.path.join(ROOT, "tests")]
import torch
import test_gpu_lnrows as T
from stzs.engine import StyleTTSZS
from stzs.params import init_params
from stzs.spec import SPEC_TINY
eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
for Cc in (512, 1024):
    for affine in (False, True):
        h, G, Bt = T._inputs("cuda:0", 2, 100, Cc, Cc + affine, 2)
        if affine:
            ln, yln = T._ln(eng, h, G[0], Bt[0], 0, 0, 1)
        else:
            ln, yln = T._ln(eng, h, G, Bt, Cc, Cc, 100, gadd=1.0)
        ref = T._unfused_ln(eng, ln, yln).float()
        cw = T._weights(eng, torch.eye(Cc), torch.zeros(Cc))
        y = T._fused(eng, cw, ln, yln, Cc, torch.float32, 0)
        d = (y != ref)
        idx = d.nonzero()
        print(Cc, affine, "mismatches", int(d.sum()), "of", d.numel(), "max abs", float((y - ref).abs().max()))
        if idx.numel():
            print("  rows", sorted(set((idx[:, 0] * 100 + idx[:, 1]).tolist()))[:20], "cols", sorted(set(idx[:, 2].tolist()))[:40])
            i = idx[0].tolist()
            print("  first", i, float(y[tuple(i)]), float(ref[tuple(i)]))
