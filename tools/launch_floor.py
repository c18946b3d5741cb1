"""Per-launch cost of a dependent kernel chain replayed from one HIP graph (tiny kernels): the floor under
every launch of the batch-1 latency path."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import ctypes as C  # noqa: E402

import torch  # noqa: E402

from stzs import _lib as L  # noqa: E402

lib = L.load()
x = torch.randn(1, 50, 256, device="cuda:0")
y = torch.empty(1, 256, device="cuda:0")
z = torch.zeros(4096, device="cuda:0")


def chain(n):
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(n):
        L.check(lib.stzs_mean_rows(x.data_ptr(), y.data_ptr(), 1, 50, 256, 50 * 256, 0, 256, 256, s))


for n in (1, 100):
    chain(n)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain(n)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 20
    print(f"graph of {n} dependent tiny launches: {el * 1e6:.1f} us per replay, {el * 1e6 / n:.2f} us per launch")

# two independent chains captured on two streams: do graph branches run concurrently on replay?
x2 = torch.randn(1, 50, 256, device="cuda:0")
y2 = torch.empty(1, 256, device="cuda:0")
side = torch.cuda.Stream()


def chain2(n):
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    s = C.c_void_p(cur.cuda_stream)
    s2 = C.c_void_p(side.cuda_stream)
    for _ in range(n):
        L.check(lib.stzs_mean_rows(x.data_ptr(), y.data_ptr(), 1, 50, 256, 50 * 256, 0, 256, 256, s))
        L.check(lib.stzs_mean_rows(x2.data_ptr(), y2.data_ptr(), 1, 50, 256, 50 * 256, 0, 256, 256, s2))
    cur.wait_stream(side)


chain2(100)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    chain2(100)
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 20
print(f"graph of 2 x 100 launches on two captured streams: {el * 1e6:.1f} us per replay")
