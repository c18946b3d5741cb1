"""Per-launch rates of the 36 MRF convs of one configs[2] step (batch 64, eager, one stream, HIP events).

Prints one line per launch: tag, (ks, dil, T_out, Co), µs, TFLOP/s, algorithmic GB/s, and a summary per
(ks, dil) class.  B from $B (default 64)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from bench import CFG, STEPS_THROUGHPUT, make_inputs  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

B = int(os.environ.get("B", 64))
eng = StyleTTSZS(S, init_params(S, 0), device="cuda:0")
tok, ref, eps, dur = (t.cuda() for t in make_inputs(S, B, 7))
nf = int(dur[0].sum())


def step():
    return eng.synth(tok, ref, steps=STEPS_THROUGHPUT, cfg_scale=CFG, noise=eps, durations=dur,
                     seeds=list(range(B)), n_frames=nf)


step()
step()
torch.cuda.synchronize()
rows = []
for rep in range(int(os.environ.get("REPS", 3))):
    eng.start_timer({"rb.c1", "rb.c2"})
    step()
    rows.append(eng.stop_timer())
cls = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0])
for i, r in enumerate(rows[0]):
    t = min(rr[i][1] for rr in rows)  # best of REPS per launch
    w, _, f, b, (ks, dil, T, Co) = r
    print(f"{w:6s} k{ks:<2d} d{dil} T{T:6d} C{Co:4d}  {t * 1e6:8.1f} us  {f / t / 1e12:7.1f} TF/s  {b / t / 1e9:7.1f} GB/s")
    c = cls[(ks, dil, Co, w)]
    c[0] += t
    c[1] += f
    c[2] += b
    c[3] += 1
print("class (ks, dil, Co, tag): launches, total us, TF/s, GB/s")
tt = ff = 0.0
for k, (t, f, b, n) in sorted(cls.items()):
    tt += t
    ff += f
    print(k, n, f"{t * 1e6:9.1f}", f"{f / t / 1e12:7.1f}", f"{b / t / 1e9:7.1f}")
print(f"all: {tt * 1e6:.1f} us, {ff / tt / 1e12:.1f} TF/s")
