"""Throughput of the precise modes (split-operand decoder; whole pipeline) vs the bf16 path on the bench
workload shape.      python tools/precise_bench.py [B] [modes]     -> one JSON line"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from bench import CFG, STEPS_THROUGHPUT, make_inputs  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
P = init_params(S, seed=0)
res = {}
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["bf16", "precise_decoder", "precise"]
for mode in modes:
    eng = StyleTTSZS(S, P, device="cuda:0", precise_decoder=(mode == "precise_decoder"), precise=(mode == "precise"))
    tok, ref, eps, dur = (t.cuda() for t in make_inputs(S, B, 0))
    nf = int(dur[0].sum())
    step = lambda: eng.synth(tok, ref, steps=STEPS_THROUGHPUT, cfg_scale=CFG, noise=eps, durations=dur,
                             seeds=list(range(B)), n_frames=nf)
    step()
    g, _ = eng.capture(step)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / n
    res[mode] = dict(ms_per_step=round(el * 1e3, 2), audio_s_per_s=round(B * 5.0 / el, 1))
    del g, eng
    torch.cuda.empty_cache()
print(json.dumps(dict(batch=B, workload="5-s targets, 2-step CFG-5", **res)))
