"""Diagnostic: is the exchange LSTM (csrc/lstm.hip) deterministic call to call?  Runs the same stzs_lstm call
repeatedly on fixed inputs and reports how many distinct outputs it produced, with the exchange slab left as
the previous call left it, or zeroed before every call; eager and graph-replayed.

    python tools/lstm_det.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0  # noqa: E402

S = SPEC_V0
dev = torch.device("cuda:0")
eng = StyleTTSZS(S, init_params(S, 0), device=dev)
g = torch.Generator().manual_seed(0)
for (B, T, name) in ((8, 80, "te_lstm"), (64, 80, "te_lstm"), (8, 200, "pr_shared"), (1, 80, "te_lstm")):
    lw = getattr(eng.W, name)
    Ci = lw.ih.Ci
    x = eng.act(f"x{B}_{T}_{Ci}", B, T, Ci)
    x.t[:, :, :Ci] = (torch.randn(B, T, Ci, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    y = eng.act(f"y{B}_{T}", B, T, S.pr_hid)
    nx = eng.lib.stzs_lstm_workspace(B, lw.H, 2)
    xchg = eng.buf("lstm.xchg", (max(nx, 16),), torch.uint8, zero=True)
    for zero in (False, True):
        outs = []
        for i in range(12):
            if zero:
                xchg.zero_()
            eng.lstm(lw, x, y, "probe")
            torch.cuda.synchronize()
            outs.append(y.t.clone())
        distinct = len({o.view(torch.int16).cpu().numpy().tobytes() for o in outs})
        dmax = max((o.float() - outs[0].float()).abs().max().item() for o in outs)
        print(f"B={B:3d} T={T:3d} {name:10s} eager, slab {'zeroed' if zero else 'kept  '}: {distinct} distinct of 12,"
              f" max |dy| {dmax:.3e}, status {eng.check_status()}", flush=True)
    # graph-replayed
    gr, _ = eng.capture(lambda: eng.lstm(lw, x, y, "probe"))
    outs = []
    for i in range(12):
        gr.replay()
        torch.cuda.synchronize()
        outs.append(y.t.clone())
    distinct = len({o.view(torch.int16).cpu().numpy().tobytes() for o in outs})
    dmax = max((o.float() - outs[0].float()).abs().max().item() for o in outs)
    print(f"B={B:3d} T={T:3d} {name:10s} graph replay: {distinct} distinct of 12, max |dy| {dmax:.3e}, "
          f"status {eng.check_status()}", flush=True)
