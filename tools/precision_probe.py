"""What the north-star log-mel L1 <= 1e-3 demands of each stage (CPU oracle, v0 dims, configs[1] inputs).

1. sensitivity: a random relative perturbation of ONE stage's output (codes, F0, N, aligned text, text features)
   -> end-to-end log-mel L1 vs the unperturbed oracle;
2. arithmetic: every conv / linear / attention matmul / LSTM matmul of the oracle emulated with bf16x3 split
   operands (hi*hi + hi*lo + lo*hi, fp32 accumulate, fp32 activations), with the WEIGHT operand rounded to bf16 and
   the activation split (hi*hi + lo*hi: two products; attention keeps three), and with bf16 operands (hi*hi only).

    python tools/precision_probe.py        (~1-2 min on 8 threads; env MODES=3,2,1, SENS=0 skips part 1)
Oracle use: this is a measurement tool (tools/), not product code.
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from oracle import stzs_ref as R  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0  # noqa: E402

torch.set_num_threads(int(os.environ.get("THREADS", 8)))
S = SPEC_V0
P = init_params(S, seed=0)
tok, ref, eps, dur = bench.make_inputs(S, 1, seed=1000)
o = R.synth(P, S, tok, ref, bench.STEPS_LATENCY, bench.CFG, eps, dur, seeds=[7])
g = torch.Generator().manual_seed(3)


def mel(a, b):
    return (R.log_mel(a, S) - R.log_mel(b, S)).abs().mean().item()


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def pert(x, d):
    return x * (1 + d * torch.randn(x.shape, generator=g))


base = o["wav"]
SENS = os.environ.get("SENS", "1") != "0"
print("== sensitivity: relative perturbation of one stage -> end-to-end log-mel L1")
for d in ((1e-6, 1e-5, 1e-4) if SENS else ()):
    c2 = pert(o["codes"], d)
    pr = R.predict_prosody(P, S, o["h_txt"], c2, dur)
    print(f"codes {d:.0e}: F0 {rel(pr['F0'], o['F0']):.2e} mel "
          f"{mel(R.decode(P, S, pr['asr'], pr['F0'], pr['N'], c2, [7]), base):.2e}", flush=True)
for d in ((1e-6, 1e-5, 1e-4) if SENS else ()):
    print(f"F0 {d:.0e}: mel {mel(R.decode(P, S, o['asr'], pert(o['F0'], d), o['N'], o['codes'], [7]), base):.2e}")
for d in ((1e-5, 1e-4) if SENS else ()):
    print(f"N {d:.0e}: mel {mel(R.decode(P, S, o['asr'], o['F0'], pert(o['N'], d), o['codes'], [7]), base):.2e}")
    print(f"asr {d:.0e}: mel {mel(R.decode(P, S, pert(o['asr'], d), o['F0'], o['N'], o['codes'], [7]), base):.2e}")
for d in ((1e-5, 1e-4) if SENS else ()):
    h2 = pert(o["h_txt"], d)
    c2 = R.sample_style(P, S, h2, o["prompt"], eps, bench.STEPS_LATENCY, bench.CFG)
    pr = R.predict_prosody(P, S, h2, c2, dur)
    w = R.decode(P, S, pr["asr"], pr["F0"], pr["N"], c2, [7])
    print(f"h_txt {d:.0e}: codes {rel(c2, o['codes']):.2e} F0 {rel(pr['F0'], o['F0']):.2e} mel {mel(w, base):.2e}",
          flush=True)

# ---- split-operand emulation
_lin, _conv, _convT, _mm = F.linear, F.conv1d, F.conv_transpose1d, torch.matmul
MODE = {"n": 3}


def _split(x):
    h = x.to(torch.bfloat16).float()
    return h, (x - h).to(torch.bfloat16).float()


def x3(op, a, b, bias=None, *args, w_op=True, **kw):
    """op(a, b) on split operands; b is the weight (w_op) except in the attention products."""
    ah, al = _split(a)
    bh, bl = _split(b)
    if MODE["n"] == 1:
        return op(ah, bh, bias, *args, **kw) if bias is not None or args or kw else op(ah, bh)
    r = op(ah, bh, bias, *args, **kw) if bias is not None or args or kw else op(ah, bh)
    lo = (lambda u, v: op(u, v, None, *args, **kw)) if bias is not None or args or kw else op
    if MODE["n"] == 2 and w_op:  # bf16 weight, split activation: two products
        return r + lo(al, bh)
    return r + lo(ah, bl) + lo(al, bh)


F.linear = lambda x, w, b=None: x3(_lin, x, w, b)
F.conv1d = lambda x, w, b=None, *a, **k: x3(_conv, x, w, b, *a, **k)
F.conv_transpose1d = lambda x, w, b=None, *a, **k: x3(_convT, x, w, b, *a, **k)


def mha(q, k, v, heads):
    Rr, Lq, D = q.shape
    dh = D // heads
    q = q.view(Rr, Lq, heads, dh).transpose(1, 2)
    k = k.view(Rr, k.shape[1], heads, dh).transpose(1, 2)
    v = v.view(Rr, v.shape[1], heads, dh).transpose(1, 2)
    a = torch.softmax(x3(_mm, q, k.transpose(-1, -2), w_op=False) / math.sqrt(dh), dim=-1)
    return x3(_mm, a, v, w_op=False).transpose(1, 2).reshape(Rr, Lq, D)


def bilstm(x, P_, name):
    B, T, _ = x.shape
    H = P_[name + ".w_hh"].shape[1]
    outs = []
    for sfx, rev in (("", False), ("_rev", True)):
        gx = F.linear(x, P_[name + ".w_ih" + sfx], P_[name + ".b_ih" + sfx] + P_[name + ".b_hh" + sfx])
        h, c = torch.zeros(B, H), torch.zeros(B, H)
        ys = [None] * T
        for t in (range(T - 1, -1, -1) if rev else range(T)):
            gt = gx[:, t] + x3(_mm, h, P_[name + ".w_hh" + sfx].t())
            i, f, gg, oo = gt.chunk(4, dim=-1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(oo) * torch.tanh(c)
            ys[t] = h
        outs.append(torch.stack(ys, 1))
    return torch.cat(outs, -1)


R._mha, R.bilstm = mha, bilstm
print("== split-operand emulation, every GEMM-like op, fp32 activations (prompt codes teacher-forced)")
for n in [int(v) for v in os.environ.get("MODES", "3,2,1").split(",")]:
    MODE["n"] = n
    o2 = R.synth(P, S, tok, ref, bench.STEPS_LATENCY, bench.CFG, eps, dur, seeds=[7], prompt_idx=o["prompt_idx"])
    print(f"{ {3: 'bf16x3', 2: 'w-bf16 x-split', 1: 'bf16'}[n] }: h {rel(o2['h_txt'], o['h_txt']):.2e} codes {rel(o2['codes'], o['codes']):.2e} "
          f"F0 {rel(o2['F0'], o['F0']):.2e} N {rel(o2['N'], o['N']):.2e} wav {rel(o2['wav'], o['wav']):.2e} "
          f"log-mel L1 {mel(o2['wav'], o['wav']):.2e}", flush=True)
for n in (3, 2):
    MODE["n"] = n
    w = R.decode(P, S, o["asr"], o["F0"], o["N"], o["codes"], [7])
    print(f"{ {3: 'bf16x3', 2: 'w-bf16 x-split'}[n] } decoder only (teacher-forced): wav {rel(w, o['wav']):.2e} "
          f"log-mel L1 {mel(w, o['wav']):.2e}", flush=True)
