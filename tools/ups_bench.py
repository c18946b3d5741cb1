"""Microbenchmark of the generator's two polyphase ConvTranspose launches at the bench workload (B = 64, 5-s
targets): the MRF-family LANE16 form (csrc/mrf.hip: one workgroup per 128-column tile, input staged per tile) vs
the input-staged-once FRAG32 form (csrc/ups.hip).  Algorithmic bytes: input once + output + residual, bf16."""
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

eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
B = int(os.environ.get("B", 64))
FLAGS = int(os.environ.get("FLAGS", "0"), 0)  # 4: skip the epilogue (ablation)
RES = os.environ.get("RES", "1") != "0"      # 0: no residual operand
for (T, Ci, Co, s, refl) in [(400, 512, 256, 10, 0), (4000, 256, 128, 6, 1)]:
    w = torch.randn(Ci, Co, 2 * s) / math.sqrt(Co * 2 * s)
    x = Act(torch.randn(B, T, Ci, device="cuda:0").to(torch.bfloat16))
    Tn = T * s + refl
    res = Act(torch.randn(B, Tn, Co, device="cuda:0").to(torch.bfloat16))
    y = Act(torch.empty(B, Tn, Co, device="cuda:0", dtype=torch.bfloat16))
    flops = 2.0 * B * (T + 1) * s * Co * Ci * 2
    byt = 2.0 * (B * T * Ci + 2 * B * Tn * Co)
    outs = {}
    for form in ("lane16", "frag32"):
        A = Arena()
        cw = pack_conv(A, "t", w, torch.zeros(Co), ups=s, lane16=form == "lane16", frag32=form == "frag32")
        A.finalize("cuda:0")
        cw.w, cw.b = A[cw.w], A[cw.b]

        def run():
            eng.conv(cw, x, y, pro_act=L.ACT_LEAKY, pro_slope=0.1, ups_pad=s // 2, T_final=T * s, refl=refl,
                     res=res if RES else None, flags=FLAGS)
        run()
        torch.cuda.synchronize()
        outs[form] = y.t.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 10
        e0.record()
        for _ in range(n):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        print(f"ups T={T} Ci={Ci} Co={Co} s={s} {form} flags={FLAGS} res={int(RES)}: {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  "
              f"{byt / us / 1e3:7.1f} GB/s (HBM roof {byt / 8e12 * 1e6:6.1f} us)", flush=True)
    print("  bit-identical:", torch.equal(outs["lane16"], outs["frag32"]))
