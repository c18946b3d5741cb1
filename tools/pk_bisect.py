"""Two-shard root-cause bisection: run the bench's concurrent two-shard graph replay (as
tools/two_shard_stress.py) once per code-object variant of the harmonic-source kernel (tools/probe/pk_variants.py),
swapping ONLY stzs_harmonic_source in both engine twins (tools/probe/pk_shim.so), and count the passes whose
harmonic-source rows (gen.har) or waveform differ from a sequential replay of the same variant.

    python tools/pk_bisect.py            (env: ITERS=24, NB=8, VARIANTS=pk,pk_nop,pk_unswap,nopk, SWEEP_US=0)
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from stzs import _lib as L  # noqa: E402
from stzs.engine import StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0  # noqa: E402

PROBE = os.path.join(ROOT, "tools", "probe")
dev = "cuda:0"
iters = int(os.environ.get("ITERS", 24))
nb = int(os.environ.get("NB", 8))
variants = os.environ.get("VARIANTS", "pk,pk_nop,pk_unswap,nopk").split(",")
sweep = float(os.environ.get("SWEEP_US", 0))  # shard-1 start offset step per iteration (us), 32 steps
stop_clean = int(os.environ.get("STOP_CLEAN", 0))  # give up on the remaining variants when pk shows nothing
shim = C.CDLL(os.path.join(PROBE, "pk_shim.so"))
shim.shim_load.argtypes = [C.c_char_p]
shim.shim_harmonic_source.argtypes = [C.POINTER(L.SourceArgs), C.c_void_p]
shim.shim_harmonic_source.restype = C.c_int


class LibProxy:
    """the engine's library handle with stzs_harmonic_source redirected to the loaded variant"""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, k):
        if k == "stzs_harmonic_source":
            return shim.shim_harmonic_source
        return getattr(self._lib, k)


S = SPEC_V0
eng = StyleTTSZS(S, init_params(S, seed=0), device=dev)
tok, ref, eps, dur, seeds = bench.rank_inputs(S, 2 * nb, 0)
tok_d, ref_d, eps_d, dur_d = (t[:2 * nb].to(dev) for t in (tok, ref, eps, dur))
nf = int(dur[0].sum())
tws = []
for i in range(2):
    tw = eng.twin()
    tw.lib = LibProxy(tw.lib)
    tws.append(tw)


def capture():
    pairs, sts, wavs = [], [], []
    for i, tw in enumerate(tws):
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
        wavs.append(wav)
    return pairs, wavs


def har(i):
    for k, ent in tws[i]._bufs.items():
        if isinstance(k, tuple) and k[0] == "gen.har":
            return ent[2]
    raise KeyError("gen.har")


def snap(wavs):
    return [(har(i).clone(), wavs[i].clone()) for i in range(2)]


summary = {}
for var in variants:
    rc = shim.shim_load(os.path.join(PROBE, f"pk_{var}.hsaco").encode())
    assert rc == 0, (var, rc)
    pairs, wavs = capture()
    for ga, gb in pairs:
        ga.replay()
        gb.replay()
    torch.cuda.synchronize()
    want = snap(wavs)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    cur = torch.cuda.current_stream(dev)
    nbad, where = 0, []
    t0 = time.time()
    for it in range(iters):
        for s in streams:
            s.wait_stream(cur)
        ev = torch.cuda.Event()
        for rep in range(3):
            for j, (s, (ga, gb)) in enumerate(zip(streams, pairs)):
                with torch.cuda.stream(s):
                    if rep == 0 and j == 1:
                        s.wait_event(ev)
                        if sweep:  # slide shard 1 against shard 0 so the source kernel meets every phase of it
                            torch.cuda._sleep(int((it % 32) * sweep * 1e-6 * 2.4e9))
                    ga.replay()
                    if rep == 0 and j == 0:
                        ev.record(s)
                    gb.replay()
        for s in streams:
            cur.wait_stream(s)
        torch.cuda.synchronize()
        got = snap(wavs)
        for i in range(2):
            h1, h0 = got[i][0], want[i][0]
            if not torch.equal(h1, h0) or not torch.equal(got[i][1], want[i][1]):
                nbad += 1
                idx = (h1 != h0).nonzero()
                if idx.numel():
                    rows = idx[:, 1]
                    lanes = sorted(set(((rows % 256) // 16).tolist()))
                    where.append(f"it{it} shard{i}: {idx.shape[0]} el, utt {idx[:, 0].unique().tolist()[:4]}, "
                                 f"frame%256 16-lane groups {lanes}, ch {idx[:, 2].unique().tolist()}")
                else:
                    where.append(f"it{it} shard{i}: wav only")
    summary[var] = (nbad, iters * 2)
    print(f"variant {var}: {nbad} of {2 * iters} shard passes differ ({time.time() - t0:.1f} s)", flush=True)
    for w in where[:12]:
        print("   ", w, flush=True)
    if stop_clean and var == "pk" and nbad == 0:
        print("pk clean: no reproduction on this box; stopping", flush=True)
        break
print("SUMMARY", {k: f"{v[0]}/{v[1]}" for k, v in summary.items()}, flush=True)
