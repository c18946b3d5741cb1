"""Do the forked branches of ONE captured HIP graph run concurrently on this runtime?  Two spin kernels of `SPIN`
cycles, one on the capture stream and one on a forked side stream, joined; replay wall time ~1x the spin = concurrent,
~2x = the branches ran one after the other.  Variants: which branch is enqueued first, and a 3-branch form.
    python tools/graph_branch_probe.py          (env SPIN=400000 cycles, REPS=20)"""
import os
import time

import torch

dev = "cuda:0"
spin = int(os.environ.get("SPIN", 400000))
reps = int(os.environ.get("REPS", 20))


def capture(order, nside=1, nk=1):
    side = [torch.cuda.Stream(dev) for _ in range(nside)]
    g = torch.cuda.CUDAGraph()
    tiny = torch.zeros(1, device=dev)
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        tiny.add_(1)
        for s in side:
            s.wait_stream(cur)
        if order == "main_first":
            for _ in range(nk):
                torch.cuda._sleep(spin // nk)
        for s in side:
            with torch.cuda.stream(s):
                for _ in range(nk):
                    torch.cuda._sleep(spin // nk)
        if order == "side_first":
            for _ in range(nk):
                torch.cuda._sleep(spin // nk)
        for s in side:
            cur.wait_stream(s)
        tiny.add_(1)
    return g


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


one = timeit(lambda: torch.cuda._sleep(spin))
print(f"env DEBUG_HIP_FORCE_GRAPH_QUEUES={os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES')} "
      f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')}: one spin {one:.0f} us")
for order in ("main_first", "side_first"):
    g = capture(order)
    print(f"  2 branches, {order}: replay {timeit(g.replay):.0f} us ({timeit(g.replay) / one:.2f}x one spin)")
for nk in (4, 16):
    for order in ("main_first", "side_first"):
        g = capture(order, 1, nk)
        print(f"  2 branches of {nk} kernels, {order}: replay {timeit(g.replay):.0f} us ({timeit(g.replay) / one:.2f}x)")
g = capture("main_first", 2)
print(f"  3 branches: replay {timeit(g.replay):.0f} us ({timeit(g.replay) / one:.2f}x one spin)")
# two graphs on two streams (what bench's shards do)
ga, gb = capture("main_first", 0), capture("main_first", 0)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def two():
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    with torch.cuda.stream(sa):
        ga.replay()
    with torch.cuda.stream(sb):
        gb.replay()
    cur.wait_stream(sa)
    cur.wait_stream(sb)


print(f"  two 1-branch graphs on two streams: {timeit(two):.0f} us ({timeit(two) / one:.2f}x one spin)")
