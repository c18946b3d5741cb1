#!/usr/bin/env python3
"""Benchmark of the MI355X StyleTTS-ZS synthesis hot path (BASELINE.json metric).

metric  : synthesized audio-seconds per wall-second (whole job, all GPUs) + p50 utterance latency,
          3-s reference -> 5-s target.
workload: one "step" = one synth() of a batch of 64 utterances per GPU (BASELINE.json configs[2],
          "batch=64, 2-step distilled diffusion, bf16" -- the throughput config whose 8-GPU form is
          configs[3]), CFG scale 5, HOTPATH spec v0 dims, seeded random-init weights, synthetic
          fixed-length inputs (16 tokens/s, durations forced to [3,2] -> exactly 5.000 s).
latency : configs[1] (batch 1, 10-step CFG-5 sampling) timed per utterance HOST TO HOST (inputs
          H2D from pinned memory, graph replay, waveform D2H, synchronize); p50/p90 reported, and the device-resident
          p50 beside it.
timing  : W warm-up steps, then K steps bracketed by barrier + synchronize, max over ranks.
          The synth() of a step is replayed from one captured HIP graph (all ~1000 launches).
roofline: the dominant kernel (the generator MRF convs -- mrfv_conv at stage 1, mrf_conv at stage 0 -- 89% of decoder FLOPs) timed
          per launch with HIP events on its own stream in an instrumented eager pass right after
          the timed region; achieved = algorithmic FLOP / average launch time (bound: MFMA).
          roofline.stages: sum t_roof / sum t_meas per synth() stage and per kernel family (stage_roofline).
cpu     : the CPU oracle (oracle/stzs_ref.py, torch fp32) on a bounded sample of the same
          workload (rank 0, N=1 only), threads = the process's affinity cores (capped by OMP_NUM_THREADS, the
          job's CPU share, when set); core counts and the host ISA are reported.
h2h     : the same steps timed host to host as well (tokens / reference / noise / durations copied in from
          pinned host memory, the waveform copied back, on per-shard copy streams overlapping the other phase) --
          reported beside `value`, which the driver contract fixes as device-resident (inputs in HBM when the
          timed region starts; the PCIe-inclusive rate is never `value`).

    python bench.py [--gpus N] [--steps K] [--warmup W]        (N > 1: starts N rank processes itself)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "styletts-zs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TARGET_S = 5.0
TOK_PER_S = 16
REF_S = 3.0
B_THROUGHPUT = 64
STEPS_THROUGHPUT = 2
CFG = 5.0
STEPS_LATENCY = 10
CHUNK_HALO = 10   # configs[4] chunked decoder: aligned frames of context each side of a 1-s chunk
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
PEAK_HBM_GBS = 8000.0


def make_inputs(S, B, seed):
    g = torch.Generator().manual_seed(1234 + seed)
    T = int(TOK_PER_S * TARGET_S)
    tok = torch.randint(1, S.n_symbols, (B, T), generator=g, dtype=torch.int64).to(torch.int32)
    ref = torch.randn(B, int(REF_S * S.sr), generator=torch.Generator().manual_seed(4321 + seed)) * 0.1
    eps = torch.randn(B, S.L_s, S.code_dim, generator=torch.Generator().manual_seed(seed))
    dur = torch.tensor([[3, 2] * (T // 2)] * B, dtype=torch.int32)
    return tok, ref, eps, dur


def rank_weights(S, rank, world, dev):
    """The packed weights every rank synthesizes with.  Rank 0 owns the parameters (seeded init); every other
    rank packs a placeholder arena of the same layout (seed 1: different bytes) and receives rank 0's with
    ONE broadcast of the arena (RCCL over xGMI on the GPU node; gloo in tests/test_dist.py).
    -> (PackedModel, broadcast wall ms)"""
    from stzs.params import init_params
    from stzs.weights import PackedModel
    W = PackedModel(S, init_params(S, seed=0 if rank == 0 else 1), dev)
    ms = 0.0
    if world > 1:
        from stzs.dist import broadcast_weights
        ms = broadcast_weights(W, src=0)
    return W, ms


def rank_inputs(S, B, rank):
    """this rank's shard of the global batch: utterances [rank*B, (rank+1)*B), their inputs and seeds."""
    tok, ref, eps, dur = make_inputs(S, B, seed=rank)
    seeds = [rank * B + i for i in range(B)]
    return tok, ref, eps, dur, seeds


def host_isa():
    """the host CPU's model and the vector ISA torch's CPU kernels dispatch to."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        cap = torch.backends.cpu.get_cpu_capability()
    except Exception:  # older torch
        cap = "unknown"
    return f"{model} ({cap})" if model else cap


def cpu_baseline(S, P, budget_s=15.0, lat_runs=5):
    from oracle import stzs_ref as R
    # every core of this process's affinity, unless the job's CPU share is pinned (OMP_NUM_THREADS: the GPU box
    # sets it to the share one GPU may use; both numbers are reported)
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    nthr = min(aff, share) if share > 0 else aff
    torch.set_num_threads(nthr)
    tok, ref, eps, dur = make_inputs(S, 1, 0)
    n, t0 = 0, time.perf_counter()
    while True:
        R.synth(P, S, tok, ref, STEPS_THROUGHPUT, CFG, eps, dur, seeds=[0])
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 64:
            break
    # configs[1] beside the GPU p50 (BASELINE.md c2 "CPU oracle latency, same inputs"): the latency leg's own inputs
    # (batch 1, 10-step CFG 5, seed 1000 of rank 0), p50 over a few runs after one warm-up
    tok1, ref1, eps1, dur1 = make_inputs(S, 1, seed=1000)
    lat = []
    for i in range(lat_runs + 1):
        a = time.perf_counter()
        R.synth(P, S, tok1, ref1, STEPS_LATENCY, CFG, eps1, dur1, seeds=[7])
        if i:
            lat.append((time.perf_counter() - a) * 1e3)
    return dict(value=n * TARGET_S / el, unit="audio-s/s", cores=nthr, affinity_cores=aff, isa=host_isa(), kind="port",
                sample=f"{n} x 1 utterance of the bench workload (5-s target, {STEPS_THROUGHPUT}-step CFG-{CFG:g}), "
                       f"CPU oracle torch fp32, {el:.1f} s",
                latency_ms=round(float(np.percentile(lat, 50)), 1),
                latency_sample=f"configs[1] on the latency leg's inputs (batch 1, 5-s target, {STEPS_LATENCY}-step "
                               f"CFG-{CFG:g}): p50 of {lat_runs} runs after one warm-up, {nthr} threads")


def longform(S, P, dev, runs=7):
    """configs[4] latency: one 30-s target (T_txt 480), 2-step CFG-5 sampling on fp8 e4m3 denoiser linears,
    waveform emitted by the streaming iSTFT in 1-s chunks.  Eager launches (no graph); p50 over runs."""
    from stzs.engine import StyleTTSZS
    e8 = StyleTTSZS(S, P, device=dev, fp8_denoiser=True)
    T = int(TOK_PER_S * 30)
    g = torch.Generator().manual_seed(99)
    tok = torch.randint(1, S.n_symbols, (1, T), generator=g).to(dev, torch.int32)
    ref = (torch.randn(1, int(REF_S * S.sr), generator=g) * 0.1).to(dev)
    eps = torch.randn(1, S.L_s, S.code_dim, generator=g).to(dev)
    dur = torch.tensor([[3, 2] * (T // 2)], dtype=torch.int32).to(dev)
    nf = int(40 * 30)

    def timed(halo, eng=None):
        eng = e8 if eng is None else eng
        first, total = [], []
        for i in range(runs + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 0
            for j, (_, w) in enumerate(eng.synth_stream(tok, ref, steps=STEPS_THROUGHPUT, cfg_scale=CFG, noise=eps,
                                                       durations=dur, seeds=[3], n_frames=nf, chunk_s=1.0,
                                                       check=False, chunked_halo=halo)):
                if j == 0:
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                n += w.shape[1]
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            assert n == 30 * S.sr
            if i:
                first.append((t1 - t0) * 1e3)
                total.append((t2 - t0) * 1e3)
        return round(float(np.percentile(first, 50)), 3), round(float(np.percentile(total, 50)), 3)
    f_w, t_w = timed(None)
    f_c, t_c = timed(CHUNK_HALO)
    lstm_to = int(int(e8.status.item()) != 0)
    del e8
    # the long-form mode at tolerance: fp8 sampler, precise text encoder / prosody predictor / decoder
    # (StyleTTSZS(precise=True, fp8_denoiser=True); tests/test_gpu_stream.py::test_longform_30s_precise_prosody)
    ep = StyleTTSZS(S, P, device=dev, precise=True, fp8_denoiser=True)
    f_p, t_p = timed(None, ep)
    lstm_to += int(int(ep.status.item()) != 0)
    del ep
    torch.cuda.empty_cache()
    return dict(lstm_timeouts=lstm_to, config="configs[4]: batch 1, 30-s target, 2-step CFG-5, fp8 e4m3 denoiser linears, "
                       "streaming iSTFT in 1-s chunks, eager", audio_s=30.0,
                p50_first_chunk_ms=f_w, p50_total_ms=t_w, realtime_factor=round(30.0 / (t_w * 1e-3), 1),
                chunked=dict(halo_frames=CHUNK_HALO, p50_first_chunk_ms=f_c, p50_total_ms=t_c,
                             note="chunked decoder (engine.decode_chunked): 1-s chunks decoded over +-halo windows with "
                                  "window-local statistics; parity vs oracle decode_chunked (tests/test_gpu_stream.py)"),
                precise_prosody=dict(p50_first_chunk_ms=f_p, p50_total_ms=t_p,
                                     realtime_factor=round(30.0 / (t_p * 1e-3), 1),
                                     note="fp8 denoiser sampler, precise (split-operand, fp32 activations) text encoder, "
                                          "prosody predictor and decoder: the configs[4] mode whose 30-s log-mel L1 "
                                          "vs the oracle is flat per 5-s window (tests/test_gpu_stream.py)"))


def gpu_ahead(ms=60.0):
    """a spinning kernel at the head of an instrumented eager pass: the host enqueues the pass's launches and events
    while it runs, so the pass then executes back to back (per-launch events would otherwise time host gaps
    wherever enqueueing is slower than the kernels)."""
    torch.cuda._sleep(int(ms * 1e-3 * 2.4e9))


def _family(w, shp):
    """kernel family of a recorded launch (stage-roofline breakdown)."""
    if w in ("rb.c1", "rb.c2"):
        return f"mrf k{shp[0]} stage {0 if shp[3] > 128 else 1}"
    if w.startswith("ups"):
        return f"ConvT {w}"
    if w.endswith(".rec"):
        return "lstm recurrence"
    if w in ("attention",):
        return "attention"
    if w.endswith(".ln") or w.startswith("te.ln") or w in ("ln1", "rowln"):
        return "row LayerNorm"
    if w in ("chan_stats", "harmonic_source", "istft", "quant"):
        return w
    if shp is not None and shp[0] == 1:
        return "linears (ks=1: gemm_glds / rows)"
    return "other convs (k>1)"


def stage_roofline(eng, S, tok_d, ref_d, eps_d, dur_d, seeds, n_frames):
    """SURVEY.md §8(d) per stage: sum t_roof / sum t_meas, one eager pass of the bench workload (batch B on one
    stream, enqueued behind gpu_ahead()).  t_meas = the stage's span between HIP events on the launching stream;
    t_roof = sum over the stage's modelled launches (every conv / linear, attention, LSTM recurrence, LayerNorm rows, statistics, harmonic source,
    iSTFT; each timed with its own events) of max(FLOP / P_bf16, bytes / BW_hbm).  Unmodelled launches (CFG + Euler,
    statistics finalize, gathers, duration head, copies) count in t_meas with no t_roof: the fractions are lower
    bounds.  Families: the same over every launch of one kernel family, t_meas = their own event times."""
    stages = {}
    W = eng.W

    def mark(name, fn):
        eng.stage = name
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        stages[name] = (e0, e1)
        return r

    def gen(gen_in, F0, gbd):
        har = eng.sine_gen(F0, seeds)
        x = gen_in
        for i in range(len(S.up_rates)):
            x = eng.mrf(eng.upsample(x, har, i), i, gbd, W.dec_norm)
        return x

    gpu_ahead()
    eng.start_timer("*")
    try:
        h, pr = mark("text+prompt", lambda: eng.encode_inputs(tok_d, ref_d))
        codes = mark("sampler", lambda: eng.sample_style(h, pr, eps_d, STEPS_THROUGHPUT, CFG))
        pro = mark("predictor", lambda: eng.predict_prosody(h, codes, dur_d, n_frames))
        gen_in, gbd = mark("decoder_pre", lambda: eng.decoder_pre(pro, codes))
        x = mark("generator", lambda: gen(gen_in, pro["F0"], gbd))
        mark("conv_post+istft", lambda: eng.istft(eng.conv_post(x)))
    finally:
        eng.stage = ""
        rec = eng.stop_timer()
    roof = lambda f, b: max(f / (PEAK_BF16_TFLOPS * 1e12), b / (PEAK_HBM_GBS * 1e9))
    out, fam = {}, {}
    for name, (e0, e1) in stages.items():
        rs = [r for r in rec if r[5] == name]
        tm = e0.elapsed_time(e1) * 1e-3
        tr = sum(roof(r[2], r[3]) for r in rs)
        out[name] = dict(t_meas_us=round(tm * 1e6, 1), t_roof_us=round(tr * 1e6, 1), frac=round(tr / tm, 4),
                         modelled_us=round(sum(r[1] for r in rs) * 1e6, 1), launches_modelled=len(rs),
                         gflop=round(sum(r[2] for r in rs) / 1e9, 2), gbytes=round(sum(r[3] for r in rs) / 1e9, 3))
    for r in rec:
        f = fam.setdefault(_family(r[0], r[4]), [0, 0.0, 0.0, 0.0, 0.0])
        f[0] += 1
        f[1] += r[1]
        f[2] += roof(r[2], r[3])
        f[3] += r[2]
        f[4] += r[3]
    fams = {k: dict(launches=v[0], t_meas_us=round(v[1] * 1e6, 1), t_roof_us=round(v[2] * 1e6, 1),
                    frac=round(v[2] / v[1], 4) if v[1] > 0 else None,
                    tflops=round(v[3] / v[1] / 1e12, 1) if v[1] > 0 else None,
                    alg_gbs=round(v[4] / v[1] / 1e9, 1) if v[1] > 0 else None)
            for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])}
    tags = {}
    for r in rec:  # by launch tag: where a stage's time goes
        t = tags.setdefault(r[0], [0, 0.0, 0.0])
        t[0] += 1
        t[1] += r[1]
        t[2] += roof(r[2], r[3])
    top = {k: dict(launches=v[0], t_meas_us=round(v[1] * 1e6, 1), frac=round(v[2] / v[1], 4) if v[1] > 0 else None)
           for k, v in sorted(tags.items(), key=lambda kv: -kv[1][1])[:16]}
    tm_all = sum(v["t_meas_us"] for v in out.values())
    tr_all = sum(v["t_roof_us"] for v in out.values())
    return dict(method="eager pass, one stream, batch %d; HIP events per stage and per modelled launch" % tok_d.shape[0],
                total=dict(t_meas_us=round(tm_all, 1), t_roof_us=round(tr_all, 1), frac=round(tr_all / tm_all, 4)),
                stages=out, families=fams, top_tags=top)


def precise_mode(S, P, dev, B=64, steps=5, nstream=2, stagger=1, schedule="pipe"):
    """throughput of the PRECISE mode -- the whole pipeline (text encoder, style diffusion, predictor, decoder) on
    fp32 activations and split-operand bf16x3 products, the mode that meets the north-star log-mel L1 <= 1e-3
    END TO END (tests/test_gpu_precise.py: 4.2e-4 at configs[1]) -- on the throughput workload (batch 64, 5-s
    targets, 2-step CFG 5): replayed as the main leg is (schedule "pipe": pipe_runner, the front of batch i + 1 beside
    the decoder of batch i; "shards": `nstream` shards on their own streams, shard_runner), and as one graph on one
    stream beside it."""
    from stzs.engine import StyleTTSZS
    ep = StyleTTSZS(S, P, device=dev, precise=True)
    host_src = make_inputs(S, B, 7)
    tok, ref, eps, dur = (t.to(dev) for t in host_src)
    nf = int(dur[0].sum())
    seeds = list(range(B))
    fn = lambda: ep.synth(tok, ref, steps=STEPS_THROUGHPUT, cfg_scale=CFG, noise=eps, durations=dur,
                          seeds=seeds, n_frames=nf, check=False)
    o = fn()
    nwav = o["wav"].shape[1]
    g, _ = ep.capture(fn)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    el1 = (time.perf_counter() - t0) / steps
    del g
    if schedule == "pipe":
        run_steps, twins, _ = pipe_runner(ep, S, dev, tok, ref, eps, dur, seeds, nf, None, host_src, nwav)
    else:
        run_steps, twins, _ = shard_runner(ep, S, dev, tok, ref, eps, dur, seeds, nf, nstream, stagger, None, host_src,
                                           nwav)
    run_steps(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(steps)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    lstm_to = int(ep.status.item()) + sum(int(t.status.item()) for t in twins)
    # where the precise step goes: the per-stage / per-family roofline of one eager pass, conv / linear FLOP counted
    # bf16x3-equivalent (3 bf16 MFMA products per fp32 product), so frac is against the bf16 MFMA peak
    st = stage_roofline(ep, S, tok, ref, eps, dur, seeds, nf)
    del run_steps, twins, ep
    torch.cuda.empty_cache()
    return dict(config=f"batch {B}, 5-s targets, 2-step CFG-5, precise mode (fp32 activations, split-operand "
                       f"bf16x3 convs / linears / LSTM / attention in every stage); " +
                       ("front of batch i + 1 beside the decoder of batch i (pipe_runner)" if schedule == "pipe" else
                        f"{nstream} shards on {nstream} streams (stagger {stagger})"),
                audio_s_per_s=round(B * TARGET_S / el, 1), ms_per_step=round(el * 1e3, 2),
                single_stream_audio_s_per_s=round(B * TARGET_S / el1, 1), lstm_status=lstm_to, stages=st)


def shard_runner(eng, S, dev, tok_d, ref_d, eps_d, dur_d, seeds, n_frames, nstream, stagger, pidx, host_src, nwav,
                 steps=STEPS_THROUGHPUT, cfg=CFG):
    """the per-GPU batch as `nstream` (near-)equal shards on engine twins (shared weights, own buffers), each captured
    as two graphs -- front (text, prompt, style diffusion, prosody) and back (decoder) -- replayed on its own stream;
    shard j > 0 starts one front phase behind shard 0 (stagger 1) or behind shard j - 1 (stagger 2: the first
    fronts chain, spreading the shards' phases), so one shard's latency-bound front (LSTM recurrences, small GEMMs) runs beside another's decoder convs.  A step is one front + one back of every shard; steps are not
    joined, the timed region ends with a synchronize after the last one.
    Host-to-host steps (h2h=True): per shard one H2D and one D2H copy stream, ordered by events so the copies overlap
    the shard's other phase -- step i+1's inputs go in once step i's front graph has read them (during its back graph),
    step i's waveform comes out during step i+1's front graph, and back graph i+1 waits for that D2H.
    -> (run_steps(k, h2h=False), twins, host buffers {tok, ref, eps, dur, wav} (pinned))"""
    B = tok_d.shape[0]
    sizes = [B // nstream + (1 if i < B % nstream else 0) for i in range(nstream)]
    pairs, twins = [], []
    for i in range(nstream):
        tw = eng.twin()
        twins.append(tw)
        sl = slice(sum(sizes[:i]), sum(sizes[:i + 1]))
        st_ = {}

        def front(tw=tw, sl=sl, st_=st_):
            h, pr = tw.encode_inputs(tok_d[sl], ref_d[sl], pidx)
            if pr.shape[0] == 1 and sl.stop - sl.start > 1:  # shared speaker: one prompt for the shard
                pe = tw.buf("prompt.bc", (sl.stop - sl.start, S.L_s, S.code_dim), pr.dtype)
                pe.copy_(pr.expand(pe.shape[0], -1, -1))
                pr = pe
            codes = tw.sample_style(h, pr, eps_d[sl], steps, cfg)
            st_["codes"], st_["pro"] = codes, tw.predict_prosody(h, codes, dur_d[sl], n_frames)

        def back(tw=tw, sl=sl, st_=st_):
            return tw.decode(st_["pro"], st_["codes"], seeds[sl])
        front()
        back()
        ga = tw.capture(front)[0]
        gb, wv = tw.capture(back)
        pairs.append((ga, gb, sl, wv))
    streams = [torch.cuda.Stream(dev) for _ in range(nstream)]
    h2d_streams = [torch.cuda.Stream(dev) for _ in range(nstream)]
    d2h_streams = [torch.cuda.Stream(dev) for _ in range(nstream)]
    host = dict(zip(("tok", "ref", "eps", "dur"), (t.pin_memory() for t in host_src)))
    host["wav"] = torch.empty(B, nwav, dtype=torch.float32).pin_memory()

    def run_steps(k, h2h=False):
        cur = torch.cuda.current_stream(dev)
        for st in streams + (h2d_streams + d2h_streams if h2h else []):
            st.wait_stream(cur)
        ev = torch.cuda.Event()
        evs = [torch.cuda.Event() for _ in range(nstream)]  # stagger 2: shard j waits for shard j - 1's first front
        front_done = [torch.cuda.Event() for _ in range(nstream)]
        back_done = [torch.cuda.Event() for _ in range(nstream)]
        in_ready = [torch.cuda.Event() for _ in range(nstream)]
        out_done = [torch.cuda.Event() for _ in range(nstream)]
        for i in range(k):
            for j, (st, (ga, gb, sl, wv)) in enumerate(zip(streams, pairs)):
                if h2h:  # this shard's inputs in from pinned host memory
                    with torch.cuda.stream(h2d_streams[j]):
                        if i > 0:
                            h2d_streams[j].wait_event(front_done[j])
                        for d_, h_ in ((tok_d, host["tok"]), (ref_d, host["ref"]), (eps_d, host["eps"]),
                                       (dur_d, host["dur"])):
                            d_[sl].copy_(h_[sl], non_blocking=True)
                        in_ready[j].record(h2d_streams[j])
                with torch.cuda.stream(st):
                    if i == 0 and j > 0 and stagger:
                        st.wait_event(evs[j - 1] if stagger == 2 else ev)
                    if h2h:
                        st.wait_event(in_ready[j])
                    ga.replay()
                    if h2h:
                        front_done[j].record(st)
                    if i == 0 and j == 0:
                        ev.record(st)
                    if i == 0:
                        evs[j].record(st)
                    if h2h and i > 0:
                        st.wait_event(out_done[j])
                    gb.replay()
                    if h2h:
                        back_done[j].record(st)
                if h2h:  # and its waveform back
                    with torch.cuda.stream(d2h_streams[j]):
                        d2h_streams[j].wait_event(back_done[j])
                        host["wav"][sl].copy_(wv, non_blocking=True)
                        out_done[j].record(d2h_streams[j])
        for st in streams + (h2d_streams + d2h_streams if h2h else []):
            cur.wait_stream(st)
    return run_steps, twins, host


def pipe_runner(eng, S, dev, tok_d, ref_d, eps_d, dur_d, seeds, n_frames, pidx, host_src, nwav, nback=1,
                steps=STEPS_THROUGHPUT, cfg=CFG):
    """the per-GPU batch as a two-stage pipeline: the front graph (text, prompt, style diffusion, prosody) of the WHOLE
    batch on one stream, the back graphs (decoder; `nback` utterance shards, each on its own stream) on others, so batch
    i's decoder runs beside batch i + 1's front (the latency-bound recurrences and small GEMMs of the front fill what
    the decoder convs leave).  Two front twins and two sets of back twins alternate by step parity (front i + 2 waits
    for every back of step i, the readers of its outputs).  Every step is one front + the backs of the full batch; the
    first front of a timed run is not overlapped (pipeline fill).  Host-to-host steps: the inputs go in on the front
    stream before each front, each back shard's waveform comes out on its stream after it.
    The front ends at the prosody: moving the decoder pre-blocks + harmonic source into it measured slower (18.3k vs
    19.2k audio-s/s), the harmonic source alone flat (profiles/r06y, r06z).
    -> (run_steps(k, h2h=False), twins, host buffers {tok, ref, eps, dur, wav} (pinned))"""
    B = tok_d.shape[0]
    sizes = [B // nback + (1 if i < B % nback else 0) for i in range(nback)]
    offs = [sum(sizes[:j]) for j in range(nback)]
    fr, st, twins, graphs = [eng.twin(), eng.twin()], [{}, {}], [], []
    for p in range(2):
        def front(tw=fr[p], s=st[p]):
            h, pr = tw.encode_inputs(tok_d, ref_d, pidx)
            codes = tw.sample_style(h, pr, eps_d, steps, cfg)
            s["codes"], s["pro"] = codes, tw.predict_prosody(h, codes, dur_d, n_frames)
        front()
        backs = []
        for j in range(nback):
            tw, b0, nb = eng.twin(), offs[j], sizes[j]
            twins.append(tw)

            def back(tw=tw, s=st[p], b0=b0, nb=nb):
                pro = s["pro"]
                if nb < B:  # this shard's utterances of the front's outputs
                    pro = dict(pro, asr_buf=pro["asr_buf"].rows(b0, nb), F0=pro["F0"][b0:b0 + nb],
                               N=pro["N"][b0:b0 + nb])
                return tw.decode(pro, s["codes"][b0:b0 + nb], seeds[b0:b0 + nb])
            back()
            gb, wv = tw.capture(back)
            backs.append((gb, wv, b0, nb))
        ga = fr[p].capture(front)[0]
        graphs.append((ga, backs))
    # (equal priorities: a high-priority decoder stream measured 12.7k audio-s/s, a high-priority front stream 15.6k,
    # against 19.0k -- profiles/r06y_*prio*; the front on a CU-masked stream (every 2nd / 4th / 8th CU) 13.4-14.4k
    # against 19.3k -- profiles/r06af: the front is not latency-bound enough to live on a fraction of the chip)
    sF, sD = torch.cuda.Stream(dev), [torch.cuda.Stream(dev) for _ in range(nback)]
    host = dict(zip(("tok", "ref", "eps", "dur"), (t.pin_memory() for t in host_src)))
    host["wav"] = torch.empty(B, nwav, dtype=torch.float32).pin_memory()

    def run_steps(k, h2h=False):
        cur = torch.cuda.current_stream(dev)
        for x in [sF] + sD:
            x.wait_stream(cur)
        fdone = [torch.cuda.Event() for _ in range(k)]
        bdone = [[torch.cuda.Event() for _ in range(nback)] for _ in range(k)]
        for i in range(k):
            ga, backs = graphs[i & 1]
            with torch.cuda.stream(sF):
                if i >= 2:  # this twin's codes / prosody were read by the backs of step i - 2
                    for e in bdone[i - 2]:
                        sF.wait_event(e)
                if h2h:
                    for d_, h_ in ((tok_d, host["tok"]), (ref_d, host["ref"]), (eps_d, host["eps"]), (dur_d, host["dur"])):
                        d_.copy_(h_, non_blocking=True)
                ga.replay()
                fdone[i].record(sF)
            for j, (gb, wv, b0, nb) in enumerate(backs):
                with torch.cuda.stream(sD[j]):
                    sD[j].wait_event(fdone[i])
                    gb.replay()
                    if h2h:
                        host["wav"][b0:b0 + nb].copy_(wv, non_blocking=True)
                    bdone[i][j].record(sD[j])
        for x in [sF] + sD:
            cur.wait_stream(x)
    return run_steps, fr + twins, host


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) without an outside launcher: start N rank processes of this script, one per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), exactly as
    `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N` would.  This
    process makes no GPU call (no HIP runtime initialised here): the ranks own the GPUs, rank 0 prints the JSON line on
    the shared stdout.  If any rank fails, the others are stopped (by their own PIDs) and its exit code is returned, so
    a missing GPU or a failed rendezvous ends the run loudly instead of reporting fewer GPUs."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    print(f"[bench] rank process {p.pid} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for q in procs:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


def dry_run(world, rank):
    """--dry-run: the N-rank set-up path on CPU under gloo with the tiny spec, up to the first GPU call -- process
    group, rank 0's weights broadcast to every rank (rank_weights), this rank's input shard (rank_inputs), the max
    reduction of the timings -- and rank 0 prints one JSON line (tests/test_dist.py runs `bench.py --gpus 2
    --dry-run` through launch_ranks)."""
    from stzs.dist import arena_digest, reduce_max
    from stzs.spec import SPEC_TINY
    if world > 1:
        dist.init_process_group("gloo")
    dev = torch.device("cpu")
    W, bcast_ms = rank_weights(SPEC_TINY, rank, world, dev)
    tok, ref, eps, dur, seeds = rank_inputs(SPEC_TINY, 4, rank)
    info = dict(rank=rank, digest=arena_digest(W), seeds=seeds, pid=os.getpid(),
                env=dict(LOCAL_RANK=os.environ.get("LOCAL_RANK"), MASTER_ADDR=os.environ.get("MASTER_ADDR")))
    allinfo = [None] * world
    if world > 1:
        dist.all_gather_object(allinfo, info)
        bcast_ms = reduce_max([bcast_ms], dev)[0]
    else:
        allinfo = [info]
    if rank == 0:
        print(json.dumps(dict(dry_run=True, n_gpus=world, weight_broadcast_ms=round(bcast_ms, 3), ranks=allinfo)))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= rank processes) of this node; > 1 without WORLD_SIZE in the environment starts the "
                         "ranks itself (launch_ranks); under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank set-up only (gloo, CPU, tiny spec): process group, weight broadcast, input shards")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=B_THROUGHPUT)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-longform", action="store_true")
    ap.add_argument("--no-precise", action="store_true")
    ap.add_argument("--no-stages", action="store_true", help="skip the per-stage roofline pass")
    ap.add_argument("--streams", type=int, default=4,
                    help="split the per-GPU batch over this many concurrently replayed graphs (engine twins)")
    ap.add_argument("--schedule", choices=("shards", "pipe"), default="pipe",
                    help="shards: --streams concurrent front+back graphs of batch shards (shard_runner); pipe: the whole "
                         "batch's front beside the previous batch's decoder (pipe_runner)")
    ap.add_argument("--pipe-backs", type=int, default=1, help="--schedule pipe: decoder shards (streams) per step")
    ap.add_argument("--precise-schedule", choices=("shards", "pipe"), default="pipe",
                    help="the precise leg's schedule (shards: 2 shards, stagger 1)")
    ap.add_argument("--stagger", type=int, default=2,
                    help="1: shards j > 0 start one front phase late; 2: shard j starts after shard j - 1's first front")
    ap.add_argument("--branch-streams", default="0",
                    help="fork independent branches onto side streams inside the graphs: 0 / 1 (all sites) / a comma "
                         "list of sites (enc = text || prompt encoder, f0n = F0 || N)")
    ap.add_argument("--shared-speaker", action="store_true",
                    help="one reference speaker for the whole job: rank 0 encodes the prompt once and broadcasts its "
                         "discrete codes (stzs.dist.broadcast_prompt_codes); every step then skips the prompt front "
                         "end (reported in config; off by default: each utterance has its own reference)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus < 1:
            sys.exit(f"[bench] --gpus {args.gpus}: need at least one GPU")
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))  # (this process never touches a GPU)
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            sys.exit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run(world, rank)
        return
    # rehearsal knobs for the N-rank path on a box with fewer GPUs (never set by the driver): STZS_BENCH_DEVICE pins
    # every rank to one device index, STZS_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU); the
    # line then reports rehearsal: true and its timing is not a scaling measurement
    rehearsal = "STZS_BENCH_DEVICE" in os.environ or os.environ.get("STZS_DIST_BACKEND", "nccl") != "nccl"
    dev = torch.device(f"cuda:{int(os.environ.get('STZS_BENCH_DEVICE', local))}")
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("STZS_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from stzs.engine import LATENCY_DN_ROWS, LATENCY_DN_SPLITK, LATENCY_TE_SPLITK, StyleTTSZS, latency_engine
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    # rank 0 owns the weights; every other rank receives them with ONE RCCL broadcast of the arena
    W, bcast_ms = rank_weights(S, rank, world, dev)
    bsv = args.branch_streams
    bs = (bsv == "1") if bsv in ("0", "1") else frozenset(v for v in bsv.split(",") if v)
    eng = StyleTTSZS(S, None, device=dev, packed=W, branch_streams=bs)
    P = init_params(S, seed=0) if rank == 0 and world == 1 else None  # host params: CPU baseline / extra modes

    B = args.batch
    tok, ref, eps, dur, seeds = rank_inputs(S, B, rank)
    tok_d, ref_d, eps_d, dur_d = (t.to(dev) for t in (tok, ref, eps, dur))
    n_frames = int(dur[0].sum())
    pidx = None  # shared-speaker mode: the job's one prompt, as discrete codes broadcast from rank 0
    if args.shared_speaker:
        from stzs.dist import broadcast_prompt_codes
        G = S.code_dim // S.vq_group
        src_idx = None
        if rank == 0:
            _, ref0, _, _ = make_inputs(S, 1, seed=0)
            eng.prompt_encode(ref0.to(dev))
            src_idx = eng.prompt_idx.clone()
        pidx = broadcast_prompt_codes(src_idx, (1, S.L_s, G), dev) if world > 1 else src_idx

    def step():
        return eng.synth(tok_d, ref_d, steps=STEPS_THROUGHPUT, cfg_scale=CFG, noise=eps_d, durations=dur_d,
                         seeds=seeds, n_frames=n_frames, prompt_idx=pidx, check=False)

    out = step()  # eager warm-up: allocates every cached buffer
    torch.cuda.synchronize()
    audio_s = out["wav"].shape[1] / S.sr
    graph = None
    if not args.no_graph:
        try:
            graph, out = eng.capture(step)
        except Exception as e:  # capture failure -> eager replay, reported in the JSON
            print(f"[bench] graph capture failed ({type(e).__name__}: {e}); eager", file=sys.stderr)
            graph = None
    run = graph.replay if graph is not None else step
    nstream = min(args.streams, B) if (graph is not None and args.streams > 1) else 1
    twins = [eng]
    pipe = graph is not None and args.schedule == "pipe"
    if pipe:
        nstream = 1 + args.pipe_backs
        run_steps, tws, host = pipe_runner(eng, S, dev, tok_d, ref_d, eps_d, dur_d, seeds, n_frames, pidx,
                                           (tok, ref, eps, dur), out["wav"].shape[1], nback=args.pipe_backs)
        twins += tws
    elif nstream > 1:
        run_steps, tws, host = shard_runner(eng, S, dev, tok_d, ref_d, eps_d, dur_d, seeds, n_frames, nstream,
                                            int(args.stagger), pidx, (tok, ref, eps, dur), out["wav"].shape[1])
        twins += tws
    else:
        host = {}

        def run_steps(k, h2h=False):
            for _ in range(k):
                if h2h:
                    for d_, h_ in ((tok_d, host["tok"]), (ref_d, host["ref"]), (eps_d, host["eps"]),
                                   (dur_d, host["dur"])):
                        d_.copy_(h_, non_blocking=True)
                run()
                if h2h:
                    host["wav"].copy_(out["wav"], non_blocking=True)
    run_steps(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # the same steps host to host (inputs from pinned host memory, waveform back): reported beside `value`
    if not host:
        host.update(zip(("tok", "ref", "eps", "dur"), (t.pin_memory() for t in (tok, ref, eps, dur))))
        host["wav"] = torch.empty(B, out["wav"].shape[1], dtype=torch.float32).pin_memory()
    run_steps(1, h2h=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run_steps(args.steps, h2h=True)
    torch.cuda.synchronize()
    el_h2h = time.perf_counter() - t1
    h2d_bytes = sum(t.numel() * t.element_size() for t in (tok, ref, eps, dur))
    if world > 1:
        from stzs.dist import reduce_max
        el, el_h2h = reduce_max([el, el_h2h], dev)
    total_audio = world * B * audio_s * args.steps
    value = total_audio / el  # whole job: every rank's utterances over the slowest rank's clock
    # the LSTM exchange's spin-timeout words of every engine that ran (a timeout = wrong prosody, reported);
    # the latency / long-form / precise engines are added below
    lstm_timeouts = sum(1 for tw in twins if int(tw.status.item()) != 0)

    # ---- roofline of the dominant kernel: instrumented eager pass, events on the kernel's stream ----
    gpu_ahead()
    eng.start_timer({"rb.c1", "rb.c2"})
    step()
    rec = eng.stop_timer()
    tsum = sum(r[1] for r in rec)
    fsum = sum(r[2] for r in rec)
    bsum = sum(r[3] for r in rec)
    nl = max(len(rec), 1)
    achieved = (fsum / nl) / (tsum / nl) / 1e12 if tsum > 0 else 0.0
    # per launch t_roof = max(F / P_mfma, B_alg / BW_hbm); aggregate = sum t_roof / sum t_meas
    # (the k3 convs are HBM-bound at 128 channels, the k7 / k11 ones MFMA-bound)
    t_roof = sum(max(r[2] / (PEAK_BF16_TFLOPS * 1e12), r[3] / (PEAK_HBM_GBS * 1e9)) for r in rec)
    n_hbm = sum(1 for r in rec if r[3] / (PEAK_HBM_GBS * 1e9) > r[2] / (PEAK_BF16_TFLOPS * 1e12))
    # HBM bytes per launch from the committed PMC passes of this workload (tools/pmc_bench.sh)
    traffic, tsrc = None, None
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_mrf.json")))
    if pmcs:  # the newest round's PMC passes (tools/pmc_bench.sh)
        with open(pmcs[-1]) as f:
            traffic, tsrc = json.load(f).get("traffic_bytes_per_launch"), "profiles/" + os.path.basename(pmcs[-1])
    roof = dict(bound="mfma", achieved=round(achieved, 2), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                frac=round(achieved / PEAK_BF16_TFLOPS, 4), traffic=traffic, traffic_src=tsrc,
                alg_bytes_per_launch=round(bsum / nl),
                kernel="generator MRF convs: mrfv_conv (csrc/mrfv.hip; stage 1 narrow, stage 0 the wide 256-channel form)",
                launches=len(rec),
                avg_launch_us=round(tsum / nl * 1e6, 2), alg_gflop_per_launch=round(fsum / nl / 1e9, 3),
                time_frac=round(t_roof / tsum, 4) if tsum > 0 else None, hbm_bound_launches=n_hbm,
                alg_hbm_gbs=round(bsum / tsum / 1e9, 1) if tsum > 0 else None)
    if not args.no_stages:  # SURVEY.md §8(d) aggregate per stage (sum t_roof / sum t_meas) + per kernel family
        roof["stages"] = stage_roofline(eng, S, tok_d, ref_d, eps_d, dur_d, seeds, n_frames)

    # ---- p50 latency, configs[1]: batch 1, 10-step CFG-5 ----
    lat = None
    if not args.no_latency:
        # host to host, as the metric defines the latency: tokens / reference / noise / durations
        # copied in from pinned host memory, the graph replayed, the waveform copied back, then a synchronize
        host1 = [t.pin_memory() for t in make_inputs(S, 1, seed=1000 + rank)]
        tok1, ref1, eps1, dur1 = dev1 = [t.to(dev) for t in host1]
        # the batch-1 serving engine: same packed weights, whole-chip small-M denoiser linears (stzs/engine.py
        # latency_engine: LATENCY_DN_ROWS, LATENCY_DN_SPLITK)
        elat = latency_engine(S, W, dev)

        def one():
            return elat.synth(tok1, ref1, steps=STEPS_LATENCY, cfg_scale=CFG, noise=eps1, durations=dur1, seeds=[7],
                              n_frames=n_frames, check=False)
        o1 = one()
        g1 = None
        if graph is not None:
            try:
                g1, o1 = elat.capture(one)
            except Exception:
                g1 = None
        wav1_h = torch.empty(o1["wav"].shape, dtype=torch.float32).pin_memory()

        def r1(h2h):
            if h2h:
                for d_, h_ in zip(dev1, host1):
                    d_.copy_(h_, non_blocking=True)
            o = g1.replay() if g1 is not None else one()
            if h2h:
                wav1_h.copy_((o1 if g1 is not None else o)["wav"], non_blocking=True)
        ts, tsd = [], []
        for i in range(45):
            h2h = i % 2 == 0
            torch.cuda.synchronize()
            a = time.perf_counter()
            r1(h2h)
            torch.cuda.synchronize()
            if i >= 5:
                (ts if h2h else tsd).append((time.perf_counter() - a) * 1e3)
        lstm_timeouts += int(int(elat.status.item()) != 0)
        lat = dict(p50_ms=round(float(np.percentile(ts, 50)), 3), p90_ms=round(float(np.percentile(ts, 90)), 3),
                   p50_device_resident_ms=round(float(np.percentile(tsd, 50)), 3),
                   timing="host to host: inputs H2D from pinned memory + graph replay + waveform D2H, then synchronize "
                          "(p50_device_resident_ms: the replay alone, inputs already in HBM)",
                   config="batch 1, 10-step sampling, CFG 5, 5-s target, 3-s reference",
                   dn_splitk=dict(LATENCY_DN_SPLITK), dn_rows=dict(LATENCY_DN_ROWS),
                   te_splitk=LATENCY_TE_SPLITK, forks=sorted(elat.branch_streams))

    # ---- configs[4]: 30-s target, batch 1, fp8 denoiser linears, streaming iSTFT (1-s chunks) ----
    lf = None
    if not args.no_longform and world == 1:
        lf = longform(S, P, dev)
        lstm_timeouts += lf.pop("lstm_timeouts")
    pr = None
    if not args.no_precise and world == 1:
        # (shards: 2 -- 4 measured slower in the fp32-activation mode, r05_j 6 491 vs 7 756)
        pr = precise_mode(S, P, dev, schedule=args.precise_schedule)
        lstm_timeouts += int(pr["lstm_status"] != 0)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(S, P)

    if rank == 0:
        line = {
            # BASELINE.json's metric; `value` is the WHOLE-JOB rate (all n_gpus), the per-GPU rate is
            # audio_s_per_s_per_gpu (= value at n_gpus 1)
            # (p50_latency_ms right behind value: the driver's stdout tail keeps the line's first ~200 characters)
            "metric": "synthesized audio-sec/sec (whole job) + p50 utterance latency, 3-s ref -> 5-s target",
            "value": round(value, 2),
            "p50_latency_ms": lat["p50_ms"] if lat else None,
            "unit": "audio-s/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded tokens 16/s, 3-s noise reference, forced [3,2] durations); random-init weights",
            "config": {"workload": "configs[2]: batch 64/GPU, 5-s targets, 2-step distilled style diffusion, CFG 5",
                       "global_batch": world * B, "seq_len": n_frames, "parallelism": f"dp{world} (utterance shards)",
                       "spec": S.name, "graph": graph is not None, "branch_streams": bs if isinstance(bs, bool) else sorted(bs), "streams": nstream,
                       "schedule": "pipe" if pipe else ("shards" if nstream > 1 else "one"),
                       "stagger": int(args.stagger) if nstream > 1 and not pipe else 0, "shared_speaker": bool(args.shared_speaker)},
            "audio_s_per_s_per_gpu": round(value / world, 2),
            "latency": lat,
            "roofline": roof,
            "cpu_baseline": cpu,
            "weight_broadcast_ms": round(bcast_ms, 3),
            "rehearsal": rehearsal,
            "lstm_timeouts": lstm_timeouts,
            "host_to_host": {"value": round(world * B * audio_s * args.steps / el_h2h, 2), "unit": "audio-s/s",
                             "ms_per_step": round(el_h2h / args.steps * 1e3, 3), "h2d_bytes_per_step": h2d_bytes,
                             "d2h_bytes_per_step": int(host["wav"].numel() * 4),
                             "note": "inputs copied in from pinned host memory and the waveform copied back inside "
                                     "every step, on the shard streams"},
            "longform": lf,
            "precise": pr,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
