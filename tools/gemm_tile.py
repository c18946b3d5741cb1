"""Launch time of the linear GEMM (csrc/gemm.hip gemm_glds) per tile height: each setting of STZS_GEMM_TILE (read once
per process by the launcher) in its own child process, the denoiser's linear shapes at several row counts.

    python tools/gemm_tile.py            (env: M=3200,6400,12800; TILES=0,64,128)
"""
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if "--child" not in sys.argv:
    tiles = os.environ.get("TILES", "0,64,128").split(",")
    for t in tiles:
        env = dict(os.environ, STZS_GEMM_TILE=t)
        r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, timeout=120)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402
from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402
from stzs.weights import Arena, pack_conv  # noqa: E402

eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
cases = {"ffn1": (512, 2048, torch.bfloat16, L.ACT_GELU, False), "qkv": (512, 1536, torch.bfloat16, L.ACT_NONE, False),
         "out": (512, 512, torch.float32, L.ACT_NONE, True), "ffn2": (2048, 512, torch.float32, L.ACT_NONE, True)}
tile = os.environ.get("STZS_GEMM_TILE", "0")
line = []
for M in [int(v) for v in os.environ.get("M", "3200,6400,12800").split(",")]:
    for name, (K, N, odt, act, gated) in cases.items():
        w = torch.randn(N, K) / math.sqrt(K)
        A = Arena()
        cw = pack_conv(A, "g", w, torch.zeros(N))
        A.finalize("cuda:0")
        cw.w, cw.b = A[cw.w], A[cw.b]
        x = Act(torch.randn(M // 50, 50, K, device="cuda:0").to(torch.bfloat16))
        y = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt))
        res = Act(torch.zeros(M // 50, 50, N, device="cuda:0", dtype=odt)) if gated else None
        gate = torch.ones(M // 50, N, device="cuda:0")

        def run():
            eng.conv(cw, x, y, epi_act=act, res=res, gate=gate.data_ptr() if gated else None, gate_bs=N)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        # 20 launches captured in one graph: the replay is GPU time only (one eager launch from Python is host-bound)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                run()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
        ts.sort()
        us = ts[len(ts) // 2]
        tf = 2.0 * M * K * N / (us * 1e-6) / 1e12
        line.append(f"{name}@{M}:{us:.1f}us/{tf:.0f}TF")
print(f"tile {tile:>3s}: " + "  ".join(line), flush=True)
