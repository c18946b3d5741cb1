"""Per-phase cycle counts of the persistent k3 MRF conv (csrc/mrfp.hip, diagnostic flag 2048): s_memtime deltas of
wave 0 of workgroups 0..15, summed over each workgroup's tiles, for the stage-1 generator shape.

    python tools/mrfp_prof.py          (env: B=64, DIL=1, VARIANT=c1|c2|c2acc)
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
B, T, C, k = int(os.environ.get("B", 64)), 24001, 128, 3
dil = int(os.environ.get("DIL", 1))
variant = os.environ.get("VARIANT", "c2")
g = torch.Generator().manual_seed(0)
w = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
A = Arena()
cw = pack_conv(A, "b", w, torch.zeros(C), frag32=True)
A.finalize(dev)
cw.w, cw.b = A[cw.w], A[cw.b]
x = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
res = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
y = Act(torch.zeros(B, T, C, device=dev, dtype=torch.bfloat16))
mean, rstd = torch.zeros(B, C, device=dev), torch.ones(B, C, device=dev)
gb = torch.zeros(B, 2 * C, device=dev)
al = torch.ones(C, device=dev)
kw = dict(pad=dil, dil=dil, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C), pro_act=L.ACT_SNAKE, pro_alpha=al,
          stats_key="p")
if variant != "c1":
    kw["res"] = res
if variant == "c2acc":
    kw.update(acc_in=res, beta=1.0)
eng.conv(cw, x, y, flags=2048 | L.CONV_MRF_PIPE, **kw)
torch.cuda.synchronize()
slab = eng._bufs["stat_slab"]
raw = slab[:16 * 16].view(torch.int64).cpu().view(16, 8)
ntiles = B * ((T + 63) // 64)
G = min(ntiles, 2 * torch.cuda.get_device_properties(0).multi_processor_count)
names = ["kloop", "wait+barA", "transform", "dma issue", "epilogue", "barC+res", "top"]
print(f"B={B} dil={dil} {variant}: {ntiles} tiles, grid {G}, ~{ntiles / G:.1f} tiles per workgroup")
for wg in range(16):
    r = raw[wg].tolist()
    hw = r[7] & 0xFFFFFFFF
    cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7
    tot = sum(r[:7])
    print(f"wg {wg:2d} (se {se} sh {sh} cu {cu:2d}): " + " ".join(f"{n} {v / (ntiles / G):7.0f}" for n, v in zip(names, r[:7]))
          + f" | total {tot / 1e3:8.1f} kcyc", flush=True)
