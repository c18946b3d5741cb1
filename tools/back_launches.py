"""Per-launch times of the decoder (the pipe schedule's back stage) at the bench batch: one eager pass with HIP events
around every modelled launch, grouped by tag -> time, achieved TFLOP/s, algorithmic GB/s, fraction of its roofline.

    python tools/back_launches.py            (env: B=64)
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

B = int(os.environ.get("B", 64))
eng = StyleTTSZS(S, init_params(S, 0), device="cuda:0")
tok, ref, eps, dur, seeds = bench.rank_inputs(S, B, 0)
tok, ref, eps, dur = (t.cuda() for t in (tok, ref, eps, dur))
nf = int(dur[0].sum())
h, pr = eng.encode_inputs(tok, ref)
codes = eng.sample_style(h, pr, eps, bench.STEPS_THROUGHPUT, bench.CFG)
pro = eng.predict_prosody(h, codes, dur, nf)
eng.decode(pro, codes, seeds)  # warm: buffers
torch.cuda.synchronize()
for rep in range(2):
    bench.gpu_ahead()
    eng.start_timer("*")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.decode(pro, codes, seeds)
    e1.record()
    rec = eng.stop_timer()
span = e0.elapsed_time(e1) * 1e3
agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
for (w, t, f, b, shp, stg) in rec:
    a = agg[w]
    a[0] += 1
    a[1] += t
    a[2] += f
    a[3] += b
    a[4] += max(f / (bench.PEAK_BF16_TFLOPS * 1e12), b / (bench.PEAK_HBM_GBS * 1e9))
tot = sum(a[1] for a in agg.values())
print(f"decoder at B = {B}: span {span:.0f} us, modelled launches {len(rec)} = {tot * 1e6:.0f} us")
for w, (n, t, f, b, tr) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{w:28s} {n:3d} x {t / n * 1e6:8.1f} us = {t * 1e6:8.1f} us  {f / t / 1e12:7.1f} TF/s  {b / t / 1e9:7.1f} GB/s  "
          f"frac {tr / t:.3f}")
