"""A/B of the conv_mfma tile order (flags 0 = XCD-aware, co tile fastest; 128 = the dispatcher's linear order) on
the decoder_pre / predictor / text-encoder conv shapes at one bench shard (B = 32) and the eager batch (B = 64)."""
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
cases = [(200, 1090, 1024, 3), (400, 1024, 512, 3), (400, 512, 512, 3), (400, 256, 256, 3), (80, 512, 512, 5)]
for B in [int(b) for b in os.environ.get("BS", "32,64").split(",")]:
    for (T, Ci, Co, k) in cases:
        w = torch.randn(Co, Ci, k) / math.sqrt(Ci * k)
        A = Arena()
        cw = pack_conv(A, "t", w, torch.zeros(Co))
        A.finalize("cuda:0")
        cw.w, cw.b = A[cw.w], A[cw.b]
        ld = (Ci + 7) // 8 * 8
        x = Act(torch.randn(B, T, ld, device="cuda:0").to(torch.bfloat16), 0, Ci)
        y = Act(torch.zeros(B, T, Co, device="cuda:0", dtype=torch.bfloat16))
        flops = 2.0 * B * T * Ci * Co * k
        for flags in (0, 128, 0, 128):
            def run20():
                for _ in range(20):
                    eng.conv(cw, x, y, pad=k // 2, pro_act=L.ACT_LEAKY, pro_slope=0.2, flags=flags)
            g, _ = eng.capture(run20)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            print(f"B={B} T={T} Ci={Ci} Co={Co} k={k} flags={flags}: {us:7.1f} us  {flops / us / 1e6:7.1f} TF/s",
                  flush=True)
