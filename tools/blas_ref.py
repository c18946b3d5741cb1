"""Reference point for the denoiser linears: the vendor GEMM (torch.matmul -> hipBLASLt) on the same shapes as
tools/gemm_bench.py (M = 6400 CFG-batched rows), bf16 in / bf16 out, no epilogue.  Not a product path: a yardstick
for what a tuned library tile reaches at these short-K shapes.   python tools/blas_ref.py  (env M, REPS)"""
import os

import torch

M = int(os.environ.get("M", 6400))
REPS = int(os.environ.get("REPS", 200))
for name, K, N in (("ffn1", 512, 2048), ("qkv", 512, 1536), ("out", 512, 512), ("ffn2", 2048, 512)):
    a = torch.randn(M, K, device="cuda:0", dtype=torch.bfloat16)
    w = torch.randn(K, N, device="cuda:0", dtype=torch.bfloat16)
    for _ in range(10):
        c = a @ w
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            c = a @ w
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS // 20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (REPS // 20 * 20)
    print(f"blas {name:5s} M {M} K {K} N {N}: {us:7.2f} us  {2 * M * K * N / us / 1e6:7.1f} TFLOP/s")
