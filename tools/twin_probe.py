"""Diagnostic: which stage of two engine twins differs when their captured graphs replay concurrently on two
streams (tests/test_gpu_configs.py::test_two_shard_streams_match_eager).  Prints, per variant and twin, whether
each intermediate buffer equals its sequential-replay value.

    python tools/twin_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0  # noqa: E402

S = SPEC_V0
dev = torch.device("cuda:0")
eng = StyleTTSZS(S, init_params(S, 0), device=dev)
nb = int(os.environ.get("NB", 8))
tok, ref, eps, dur, seeds = bench.rank_inputs(S, 2 * nb, 0)
tok_d, ref_d, eps_d, dur_d = (t.to(dev) for t in (tok, ref, eps, dur))
nf = int(dur[0].sum())
KEYS = ["te.e", "te.h", "prompt.z", "prompt", "dn.x", "pr.xin", "pr.hd", "pr.xs", "pr.F0", "gen.x0", "gen.xs0",
        "gen.x1", "gen.xs1", "gen.wav"]
tws, graphs = [], []
for i in range(2):
    tw = eng.twin()
    sl = slice(i * nb, (i + 1) * nb)
    st = {}

    def front(tw=tw, sl=sl, st=st):
        h = tw.text_encode(tok_d[sl])
        pr = tw.prompt_encode(ref_d[sl])
        codes = tw.sample_style(h, pr, eps_d[sl], 2, 5.0)
        st["codes"], st["pro"] = codes, tw.predict_prosody(h, codes, dur_d[sl], nf)

    def back(tw=tw, sl=sl, st=st):
        return tw.decode(st["pro"], st["codes"], seeds[sl])
    front()
    back()
    graphs.append((tw.capture(front)[0], tw.capture(back)[0]))
    tws.append(tw)


def snap(tw):
    out = {}
    for key, t in tw._bufs.items():
        if isinstance(key, tuple) and key[0] in KEYS:
            out[key[0]] = t.clone()
    return out


def seq():
    for ga, gb in graphs:
        ga.replay()
        gb.replay()
    torch.cuda.synchronize()
    return [snap(t) for t in tws]


ref_state = seq()


def compare(tag):
    torch.cuda.synchronize()
    for i, tw in enumerate(tws):
        cur = snap(tw)
        bad = [k for k in KEYS if k in cur and not torch.equal(cur[k], ref_state[i][k])]
        print(f"{tag:32s} twin {i}: differs in {bad if bad else 'nothing'}  status {tw.check_status()}", flush=True)


def run(plan, tag, reps=3):
    """plan: list per stream of graph lists"""
    streams = [torch.cuda.Stream(dev) for _ in plan]
    cur = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(cur)
    for _ in range(reps):
        for s, gl in zip(streams, plan):
            with torch.cuda.stream(s):
                for g in gl:
                    g.replay()
    for s in streams:
        cur.wait_stream(s)
    compare(tag)


(fa0, fb0), (fa1, fb1) = graphs
seq()
compare("sequential again")
run([[fa0], [fa1]], "fronts concurrently")
seq()
run([[fb0], [fb1]], "backs concurrently")
seq()
run([[fa0], [fb1]], "front0 || back1")
seq()
run([[fa0, fb0], [fa1, fb1]], "front+back concurrently")
