"""configs[1] latency probe: batch 1, 10-step CFG-5, 5-s target, graph-replayed N times (for rocprofv3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from bench import CFG, STEPS_LATENCY, make_inputs  # noqa: E402
from stzs.engine import LATENCY_BLK_SPLITK, LATENCY_DN_ROWS, LATENCY_DN_SPLITK, LATENCY_TE_SPLITK, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

sk = os.environ.get("STZS_DN_SPLITK")  # "0": split-K off, "ff2=4,...": a table; unset: the bench's latency engine
rw = os.environ.get("STZS_DN_ROWS")  # "0": whole-chip small-M linears off, "qkv=1,...": a table; unset: the latency table
te = os.environ.get("STZS_TE_SPLITK")  # text-encoder conv split-K slices; unset: the latency engine's LATENCY_TE_SPLITK
bk = os.environ.get("STZS_BLK_SPLITK")  # AdaIN-block conv split-K slices; unset: the latency engine's LATENCY_BLK_SPLITK
eng = StyleTTSZS(S, init_params(S, 0), device="cuda:0", dn_splitk=None if sk is not None else LATENCY_DN_SPLITK,
                 dn_rows=None if rw is not None else LATENCY_DN_ROWS, te_splitk=None if te is not None else LATENCY_TE_SPLITK,
                 blk_splitk=None if bk is not None else LATENCY_BLK_SPLITK,
                 branch_streams=(lambda v: v != "0" if v in ("0", "1") else set(v.split(",")))(
                     os.environ.get("STZS_BRANCH_STREAMS", "0")))  # "1": text || prompt and F0 || N forked; "f0n" / "enc"
tok, ref, eps, dur = (t.cuda() for t in make_inputs(S, 1, 1000))
nf = int(dur[0].sum())
one = lambda: eng.synth(tok, ref, steps=STEPS_LATENCY, cfg_scale=CFG, noise=eps, durations=dur, seeds=[7], n_frames=nf)
one()
g, _ = eng.capture(one)
n = int(os.environ.get("N", 20))
ts = []
for _ in range(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
ts.sort()
print(f"STZS_DN_SPLITK={sk} STZS_DN_ROWS={rw} STZS_TE_SPLITK={te} STZS_BLK_SPLITK={bk} branch_streams={eng.branch_streams} dur_overlap={int(eng.dur_overlap)} latency p50 {ts[len(ts) // 2]:.3f} ms  min {ts[0]:.3f}  launches/synth {eng.launches // 2}")
