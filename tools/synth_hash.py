"""Whole-pipeline bit check across two library builds: synthesize fixed v0 inputs on the throughput engine (B = 3),
the latency engine (B = 1), the fp8-denoiser engine (B = 1) and the precise engine (B = 2), and print the sha256 of
every output (waveform, style codes, durations).  Run once per build (STZS_LIB=<lib.so>), compare the printed lines.

    STZS_LIB=<lib.so> python tools/synth_hash.py > a.txt
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from bench import CFG, make_inputs  # noqa: E402
from stzs.engine import StyleTTSZS, latency_engine  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402


def h(t):
    return hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


P = init_params(S, 0)
base = StyleTTSZS(S, P, device="cuda:0")
cases = [("throughput", base, 3, 2), ("latency", latency_engine(S, base.W), 1, 10),
         ("fp8", StyleTTSZS(S, P, device="cuda:0", fp8_denoiser=True), 1, 2),
         ("precise", StyleTTSZS(S, P, device="cuda:0", precise=True), 2, 2)]
for name, eng, B, steps in cases:
    tok, ref, eps, dur = (t.cuda() for t in make_inputs(S, B, 7))
    for dur_in in (dur, None):
        n = B if dur_in is not None else 1  # (predicted durations: one utterance -- a batch shares its frame count)
        out = eng.synth(tok[:n], ref[:n], steps=steps, cfg_scale=CFG, noise=eps[:n], durations=dur_in,
                        seeds=list(range(n)))
        torch.cuda.synchronize()
        tag = "forced" if dur_in is not None else "predicted"
        print(f"{name:10s} {tag:9s} " + " ".join(f"{k}={h(v)}" for k, v in sorted(out.items())
                                                   if isinstance(v, torch.Tensor)), flush=True)
