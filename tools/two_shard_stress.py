"""Stress the bench's two-shard concurrent graph replay (tests/test_gpu_configs.py test_two_shard_streams_match_eager)
many times in one process and say WHICH output of which shard diverges from the sequential replay (codes, F0, N,
decoder wav), to localise a timing-dependent mismatch.

    python tools/two_shard_stress.py      (env: ITERS=40, BRANCH=1 (branch_streams), NB=8, SWEEP_US=0, BUFS=1)
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

dev = "cuda:0"
iters = int(os.environ.get("ITERS", 40))
branch = os.environ.get("BRANCH", "1") == "1"
nb = int(os.environ.get("NB", 8))
sweep = float(os.environ.get("SWEEP_US", 0))  # shard-1 start offset step per iteration (us, 32 steps; tools/pk_bisect.py)
S = SPEC_V0
eng = StyleTTSZS(S, init_params(S, seed=0), device=dev)
tok, ref, eps, dur, seeds = bench.rank_inputs(S, 2 * nb, 0)
tok_d, ref_d, eps_d, dur_d = (t[:2 * nb].to(dev) for t in (tok, ref, eps, dur))
nf = int(dur[0].sum())
pairs, sts, tws, wavs = [], [], [], []
for i in range(2):
    tw = eng.twin()
    tw.branch_streams = branch
    sl = slice(i * nb, (i + 1) * nb)
    st = {}

    def front(tw=tw, sl=sl, st=st):
        h, pr = tw.encode_inputs(tok_d[sl], ref_d[sl])
        codes = tw.sample_style(h, pr, eps_d[sl], bench.STEPS_THROUGHPUT, bench.CFG)
        st["codes"], st["pro"] = codes, tw.predict_prosody(h, codes, dur_d[sl], nf)

    def back(tw=tw, sl=sl, st=st):
        return tw.decode(st["pro"], st["codes"], seeds[sl])
    ga = tw.capture(front)[0]
    gb, wav = tw.capture(back)
    pairs.append((ga, gb))
    sts.append(st)
    tws.append(tw)
    wavs.append(wav)


def snap(i):
    st = sts[i]
    d = dict(codes=st["codes"].clone(), F0=st["pro"]["F0"].clone(), N=st["pro"]["N"].clone(), wav=wavs[i].clone())
    if i == 0 and os.environ.get("BUFS", "1") == "1":  # every cached buffer of shard 0's twin
        for k, ent in tws[0]._bufs.items():
            if isinstance(k, tuple):
                d["buf:" + k[0]] = ent[2].clone()
    return d


for ga, gb in pairs:
    ga.replay()
    gb.replay()
torch.cuda.synchronize()
want = [snap(i) for i in range(2)]
for ga, gb in pairs:  # a second sequential pass must agree with the first
    ga.replay()
    gb.replay()
torch.cuda.synchronize()
for i in range(2):
    s = snap(i)
    print("sequential repeat shard", i, {k: torch.equal(s[k], want[i][k]) for k in s}, flush=True)
streams = [torch.cuda.Stream(dev) for _ in range(2)]
cur = torch.cuda.current_stream(dev)
bad = {}
for it in range(iters):
    for s in streams:
        s.wait_stream(cur)
    ev = torch.cuda.Event()
    for rep in range(3):
        for j, (s, (ga, gb)) in enumerate(zip(streams, pairs)):
            with torch.cuda.stream(s):
                if rep == 0 and j == 1:
                    s.wait_event(ev)
                    if sweep:
                        torch.cuda._sleep(int((it % 32) * sweep * 1e-6 * 2.4e9))
                ga.replay()
                if rep == 0 and j == 0:
                    ev.record(s)
                gb.replay()
    for s in streams:
        cur.wait_stream(s)
    torch.cuda.synchronize()
    for i in range(2):
        s = snap(i)
        diff = [k for k in s if not torch.equal(s[k], want[i][k])]
        if diff:
            bad[(it, i)] = diff
            print(f"iter {it} shard {i}: differs in {diff}; max |d| " +
                  ", ".join(f"{k} {(s[k].float() - want[i][k].float()).abs().max().item():.3e}" for k in diff) +
                  f"; status {tws[i].check_status()}", flush=True)
            if "buf:gen.har" in diff:
                h1, h0 = s["buf:gen.har"].float(), want[i]["buf:gen.har"].float()
                dd = (h1 != h0)
                idx = dd.nonzero()
                print(f"   gen.har {tuple(h1.shape)}: {idx.shape[0]} elements differ; utt {idx[:, 0].unique().tolist()[:8]} "
                      f"rows {idx[:, 1].min().item()}..{idx[:, 1].max().item()} ch {idx[:, 2].unique().tolist()}", flush=True)
                for r in idx[:6].tolist():
                    print(f"     {r}: got {h1[tuple(r)].item():.5f} want {h0[tuple(r)].item():.5f}", flush=True)
                u0, r0 = idx[0, 0].item(), idx[0, 1].item()
                print("     got  row:", " ".join(f"{v:.5f}" for v in h1[u0, r0, :22].tolist()), flush=True)
                print("     want row:", " ".join(f"{v:.5f}" for v in h0[u0, r0, :22].tolist()), flush=True)
                print(f"   first utt rows differing: {dd[idx[0, 0]].any(1).nonzero().flatten()[:20].tolist()}", flush=True)
            if "wav" in diff:
                d = (s["wav"].float() - want[i]["wav"].float()).abs() > 0
                for u in d.any(1).nonzero().flatten().tolist()[:4]:
                    nzi = d[u].nonzero().flatten()
                    print(f"   utt {u}: {nzi.numel()} samples differ, first {nzi[0].item()} last {nzi[-1].item()} "
                          f"of {d.shape[1]}", flush=True)
print(f"branch_streams={branch}: {len(bad)} shard mismatches in {iters} iterations x 2 shards", flush=True)
