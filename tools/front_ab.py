"""Front stages of the throughput engine at the bench batch (text + prompt encoders, sampler, prosody; B = 64) timed
eagerly with HIP events -- for A/B runs of two library builds (STZS_LIB=<path>): median of REPS passes.

    STZS_LIB=... python tools/front_ab.py            (env: B=64, REPS=15)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

B = int(os.environ.get("B", 64))
reps = int(os.environ.get("REPS", 15))
eng = StyleTTSZS(S, init_params(S, 0), device="cuda:0")
tok, ref, eps, dur, seeds = bench.rank_inputs(S, B, 0)
tok, ref, eps, dur = (t.cuda() for t in (tok, ref, eps, dur))
nf = int(dur[0].sum())


def front():
    h, pr = eng.encode_inputs(tok, ref)
    codes = eng.sample_style(h, pr, eps, bench.STEPS_THROUGHPUT, bench.CFG)
    return eng.predict_prosody(h, codes, dur, nf)


front()
torch.cuda.synchronize()
g, _ = eng.capture(front)
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
print(f"lib={os.environ.get('STZS_LIB', 'in-tree')} B={B}: front graph median {statistics.median(ts):.1f} us "
      f"(min {min(ts):.1f})", flush=True)
