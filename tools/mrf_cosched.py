"""Does running the three resblocks' convs of one MRF layer SIDE BY SIDE pay?  The stage-1 c1 convs of the k3 / k7 / k11
resblocks (B = 64, T 24 001, 128 channels, dilation d) timed one after another on one stream vs. each on its own
stream at once (the hardware queues interleave their workgroups on the CUs) -- an upper-bound probe for a one-launch
"trio" form.  python tools/mrf_cosched.py   (env: B, D, REPS, STAGE=1|0, GRAPH=1: both orders captured in a HIP graph
-- at batch 1 the eager launches are host-bound)"""
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
B = int(os.environ.get("B", 64))
D = int(os.environ.get("D", 1))
REPS = int(os.environ.get("REPS", 10))
T, C = (24001, 128) if os.environ.get("STAGE", "1") == "1" else (4000, 256)
g = torch.Generator().manual_seed(0)
engs, convs = [], []
x = Act(torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16))
mean = (torch.randn(B, C, generator=g) * 0.1).to(dev)
rstd = (torch.rand(B, C, generator=g) + 0.5).to(dev)
gb = (torch.randn(B, 2 * C, generator=g) * 0.2).to(dev)
al = (torch.rand(C, generator=g) + 0.5).to(dev)
for k in (3, 7, 11):
    e = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device=dev)
    w = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    A = Arena()
    cw = pack_conv(A, "b", w, torch.zeros(C), frag32=True)
    A.finalize(dev)
    cw.w, cw.b = A[cw.w], A[cw.b]
    y = Act(torch.zeros(B, T, C, device=dev, dtype=torch.bfloat16))
    kw = dict(pad=D * (k - 1) // 2, dil=D, pro=(mean, rstd, C, gb.data_ptr(), 2 * C, C), pro_act=L.ACT_SNAKE,
              pro_alpha=al, stats_key=f"cs.{k}")
    engs.append(e)
    convs.append((e, cw, y, kw, k))


def run(i):
    e, cw, y, kw, k = convs[i]
    e.conv(cw, x, y, **kw)


for i in range(3):
    run(i)
torch.cuda.synchronize()
if os.environ.get("GRAPH", "0") == "1":
    cur = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(3)]

    def seq_body():
        for i in range(3):
            run(i)

    def conc_body():
        c = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(c)
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                run(i)
        for s in streams:
            c.wait_stream(s)

    def timed(body):
        g = torch.cuda.CUDAGraph()
        sg = torch.cuda.Stream()
        sg.wait_stream(cur)
        with torch.cuda.stream(sg):
            with torch.cuda.graph(g, stream=sg):
                for _ in range(REPS):
                    body()
        cur.wait_stream(sg)
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / (5 * REPS) * 1e3

    singles = []
    for i in range(3):
        singles.append(timed(lambda i=i: run(i)))
    tseq, tconc = timed(seq_body), timed(conc_body)
    print(f"[graph] stage T={T} C={C} B={B} d={D}: k3 / k7 / k11 alone {singles[0]:.1f} / {singles[1]:.1f} / "
          f"{singles[2]:.1f} us (conv + statistics); one stream {tseq:.1f} us per layer; three branches {tconc:.1f} us "
          f"({tseq / tconc:.3f}x)", flush=True)
    sys.exit(0)
ev = lambda: torch.cuda.Event(enable_timing=True)
single = []
for i in range(3):
    a, b = ev(), ev()
    a.record()
    for _ in range(REPS):
        run(i)
    b.record()
    torch.cuda.synchronize()
    single.append(a.elapsed_time(b) / REPS * 1e3)
a, b = ev(), ev()
a.record()
for _ in range(REPS):
    for i in range(3):
        run(i)
b.record()
torch.cuda.synchronize()
seq = a.elapsed_time(b) / REPS * 1e3
streams = [torch.cuda.Stream() for _ in range(3)]
cur = torch.cuda.current_stream()
for _ in range(2):
    a, b = ev(), ev()
    a.record()
    for s in streams:
        s.wait_stream(cur)
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            for _ in range(REPS):
                run(i)
    for s in streams:
        cur.wait_stream(s)
    b.record()
    torch.cuda.synchronize()
conc = a.elapsed_time(b) / REPS * 1e3
print(f"stage T={T} C={C} B={B} d={D}: k3 / k7 / k11 alone {single[0]:.1f} / {single[1]:.1f} / {single[2]:.1f} us; "
      f"one stream {seq:.1f} us per layer; three streams at once {conc:.1f} us per layer ({seq / conc:.3f}x)", flush=True)
