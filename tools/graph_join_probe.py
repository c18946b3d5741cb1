"""Does work enqueued on a stream after a HIP graph replay wait for EVERY leaf of the graph?

A captured fork whose side branch is the last thing in the graph (no node on the capture stream after the join)
leaves the graph with two leaves.  This probe replays such a graph (side branch: a spin, then out <- src) and
reads `out` on the same stream right behind the replay; stale reads mean the replay's completion only covered the
capture stream's leaf (engine.fork() then needs a node on the capture stream after the join).

    python tools/graph_join_probe.py        (env: REPS=200, SPIN=200000 cycles)
"""
import os

import torch

dev = "cuda:0"
reps = int(os.environ.get("REPS", 200))
spin = int(os.environ.get("SPIN", 200000))
n = 1 << 20


def build(join_node: bool):
    src = torch.zeros(n, device=dev)
    out = torch.zeros(n, device=dev)
    tiny = torch.zeros(1, device=dev)
    side = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        tiny.add_(1)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            torch.cuda._sleep(spin)
            out.copy_(src)
        cur.wait_stream(side)
        if join_node:
            tiny.add_(1)
    return g, src, out


for join_node in (False, True):
    res = torch.zeros(reps, device=dev)
    torch.cuda.synchronize()
    g, src, out = build(join_node)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for r in range(reps):
            src.fill_(float(r + 1))
            out.fill_(-1.0)
            g.replay()
            res[r:r + 1].copy_(out[n - 1:n])  # the last element: written last by the copy
    torch.cuda.synchronize()
    want = torch.arange(1, reps + 1, device=dev, dtype=torch.float32)
    bad = int((res != want).sum().item())
    idx = (res != want).nonzero().flatten().tolist()
    print(f"join node after the fork: {join_node}: {bad} of {reps} replays read a stale side-branch output"
          f" (replays {idx[:10]}, read {[res[i].item() for i in idx[:10]]})", flush=True)
