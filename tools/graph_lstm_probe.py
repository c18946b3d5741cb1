"""Does a forked graph branch run beside the exchange LSTM (csrc/lstm.hip) in one captured graph?  Branch A: one
v0-width BiLSTM recurrence (B = 1, T = 200); branch B: spin kernels of about the same total time.  Replay time vs
the two alone.    python tools/graph_lstm_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

dev = "cuda:0"
eng = StyleTTSZS(S, init_params(S, 0), device=dev)
lw = eng.W.pr_shared
x = Act(torch.randn(1, 200, S.pr_in, device=dev).to(torch.bfloat16))
y = Act(torch.zeros(1, 200, S.pr_hid, device=dev, dtype=torch.bfloat16))
side = torch.cuda.Stream(dev)
nk = int(os.environ.get("NK", 8))
spin = int(os.environ.get("SPIN", 600000))


def timeit(fn, reps=20):
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


def cap(parts):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        if "lstm" in parts:
            eng.lstm(lw, x, y, "probe")
        if "spin" in parts:
            with torch.cuda.stream(side) if "lstm" in parts else torch.cuda.stream(cur):
                for _ in range(nk):
                    torch.cuda._sleep(spin // nk)
        cur.wait_stream(side)
    return g


eng.lstm(lw, x, y, "probe")
torch.cuda.synchronize()
ga, gs, gb = cap(("lstm",)), cap(("spin",)), cap(("lstm", "spin"))
ta, ts_, tb = timeit(ga.replay), timeit(gs.replay), timeit(gb.replay)
print(f"lstm alone {ta:.0f} us, {nk} spins alone {ts_:.0f} us, both forked in one graph {tb:.0f} us "
      f"(serial would be {ta + ts_:.0f}); status {eng.check_status()}")
