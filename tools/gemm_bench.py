"""Microbenchmark of the denoiser linears (B=64 CFG-batched: 6400 rows) through stzs_conv1d, with the
conv ablation flags (2 = one K-step only, 4 = skip the epilogue stores).  FLAGS="0,2,4".
F8=1: the fp8 e4m3 form (configs[4], gemm_glds<F8>); M=100 is configs[4]'s batch-1 CFG-batched row count."""
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
from stzs.weights import Arena, pack_conv, pack_conv_f8  # noqa: E402

eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
M = int(os.environ.get("M", 6400))
FLAGS = [int(f, 0) for f in os.environ.get("FLAGS", "0,2,4").split(",")]
F8 = os.environ.get("F8", "0") == "1"
SKS = [int(v) for v in os.environ.get("SK", "0").split(",")]  # split-K counts (stzs_conv_args.splitk)
# ROWS="0,1,2,4": 0 = the LDS-DMA GEMM (gemm_glds), Z >= 1 = the small-M form (csrc/rows.hip) with K in Z slices
ROWS = [int(v) for v in os.environ.get("ROWS", "0").split(",")]
cases = [("ffn1 gelu", 512, 2048, torch.bfloat16, L.ACT_GELU, False), ("qkv", 512, 1536, torch.bfloat16, L.ACT_NONE, False),
         ("out gated f32", 512, 512, torch.float32, L.ACT_NONE, True), ("ffn2 gated f32", 2048, 512, torch.float32, L.ACT_NONE, True),
         ("kv", 512, 1024, torch.bfloat16, L.ACT_NONE, False), ("lstm ih f32", 512, 2048, torch.float32, L.ACT_NONE, False)]
# CASES="kv,qkv": a subset by name prefix (default: the four denoiser layer linears)
_sel = os.environ.get("CASES")
cases = [c for c in cases if (_sel is None and c[0] not in ("kv", "lstm ih f32")) or
         (_sel is not None and any(c[0].startswith(n) for n in _sel.split(",")))]
for name, K, N, odt, act, gated in cases:
    w = torch.randn(N, K) / math.sqrt(K)
    A = Arena()
    cw = pack_conv_f8(A, "g", w, torch.zeros(N)) if F8 else pack_conv(A, "g", w, torch.zeros(N))
    A.finalize("cuda:0")
    cw.w, cw.b = A[cw.w], A[cw.b]
    if F8:
        cw.wscale = A[cw.wscale]
        x = Act(torch.randn(M // 50, 50, K, device="cuda:0").clamp(-4, 4).to(torch.float8_e4m3fn))
        xs = torch.ones(M, device="cuda:0")
    else:
        x = Act(torch.randn(M // 50, 50, K, device="cuda:0").to(torch.bfloat16))
        xs = None
    y = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt))
    res = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt)) if gated else None
    gate = torch.ones(M // 50, N, device="cuda:0")
    flops = 2.0 * M * N * K
    for flags, sk, rz in [(f, k, z) for f in FLAGS for k in SKS for z in ROWS]:
        def run():
            eng.conv(cw, x, y, epi_act=act, res=res, gate=gate.data_ptr() if gated else None, gate_bs=N, flags=flags,
                     x_scale=xs, splitk=sk, rows=rz)
        def run20():
            for _ in range(20):
                run()
        g, _ = eng.capture(run20)  # HIP graph: GPU-bound timing, no host launch overhead
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name:16s} {'fp8' if F8 else 'bf16'} M={M} K={K} N={N} flags={flags} splitk={sk} rows={rz}: {us:7.1f} us  "
              f"{flops / us / 1e6:7.1f} TF/s", flush=True)
