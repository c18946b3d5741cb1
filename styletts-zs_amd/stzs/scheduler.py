"""Variable-length batching for the synthesis hot path (length bucketing).

The kernels take uniform [B, T, C] batches (per-utterance InstanceNorm statistics, LSTM recurrences and
attention are computed per row, never across rows).  Real requests differ in token count, reference length
and -- known only after the duration head -- frame count.  BucketScheduler runs them in two phases:

  phase 1  requests grouped by (token count, reference length), chunks of <= max_batch:
           text encoder, prompt front end, style diffusion, duration head (a1-a6)  -> per-utterance durations
  phase 2  utterances regrouped by their aligned frame count T40 (the quantity every decoder buffer is sized
           by), chunks of <= max_batch: alignment, prosody (a7-a8) and the decoder (a9-a13).  Token rows of a
           phase-2 batch are zero-padded to its longest text with duration 0 for the padding tokens, which the
           alignment scan never references -- so padding changes no output value.

Every row is computed exactly as it would be alone (tests/test_gpu_scheduler.py compares against
per-request synth() calls), so bucketing is a pure scheduling decision.  Regrouping copies a few small
per-utterance tensors (text rows, duration-encoder rows, codes) with torch indexing on the device: data
movement only, no compute.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional

import torch

from .engine import Act, StyleTTSZS


@dataclass
class Request:
    tokens: torch.Tensor            # int [T_txt]
    ref_wav: torch.Tensor           # fp32 [N] (24 kHz reference)
    noise: torch.Tensor             # fp32 [L_s, code_dim] style noise
    seed: int = 0                   # harmonic-source noise seed
    durations: Optional[torch.Tensor] = None  # optional forced int [T_txt]


class BucketScheduler:
    def __init__(self, engine: StyleTTSZS, max_batch: int = 64, steps: int = 2, cfg_scale: float = 5.0):
        self.eng, self.max_batch, self.steps, self.cfg = engine, max_batch, steps, cfg_scale
        self.stats = {}

    def _chunks(self, ids):
        for i in range(0, len(ids), self.max_batch):
            yield ids[i:i + self.max_batch]

    def synth(self, reqs: List[Request]) -> List[torch.Tensor]:
        """-> one fp32 waveform [600 * T40_i] per request, in request order (device tensors)."""
        eng, S, dev = self.eng, self.eng.spec, self.eng.device
        # ---- phase 1: text / prompt / style / durations, grouped by (T_txt, N_ref) ----
        g1 = OrderedDict()
        for i, r in enumerate(reqs):
            g1.setdefault((int(r.tokens.shape[0]), int(r.ref_wav.shape[0]), r.durations is not None), []).append(i)
        per = [None] * len(reqs)
        n1 = 0
        for (_, _, forced), ids in g1.items():
            for ch in self._chunks(ids):
                n1 += 1
                tok = torch.stack([reqs[i].tokens for i in ch]).to(dev, torch.int32)
                ref = torch.stack([reqs[i].ref_wav for i in ch]).to(dev, torch.float32)
                eps = torch.stack([reqs[i].noise for i in ch]).to(dev, torch.float32)
                h = eng.text_encode(tok)
                prompt = eng.prompt_encode(ref)
                codes = eng.sample_style(h, prompt, eps, self.steps, self.cfg)
                dur_ov = torch.stack([reqs[i].durations for i in ch]) if forced else None
                du = eng.predict_durations(h, codes, dur_ov)
                tot = du["dur"].to(torch.int64).sum(1).cpu()  # host sync: frame counts decide phase 2
                eng.check_status()  # a timed-out LSTM exchange would make these durations wrong: raise
                for j, i in enumerate(ch):
                    per[i] = dict(h=h.t[j].clone(), d=du["d"].t[j].clone(), dur=du["dur"][j].clone(),
                                  codes=codes[j].clone(), T40=int(tot[j]), seed=reqs[i].seed)
        # ---- phase 2: prosody + decoder, grouped by aligned frame count ----
        g2 = OrderedDict()
        for i, p in enumerate(per):
            g2.setdefault(p["T40"], []).append(i)
        out = [None] * len(reqs)
        n2 = 0
        for T40, ids in g2.items():
            for ch in self._chunks(ids):
                n2 += 1
                Tm = max(per[i]["h"].shape[0] for i in ch)
                b = len(ch)
                h = torch.zeros(b, Tm, per[ch[0]]["h"].shape[1], dtype=per[ch[0]]["h"].dtype, device=dev)
                d = torch.zeros(b, Tm, per[ch[0]]["d"].shape[1], dtype=per[ch[0]]["d"].dtype, device=dev)
                dur = torch.zeros(b, Tm, dtype=torch.int32, device=dev)
                for j, i in enumerate(ch):
                    T = per[i]["h"].shape[0]
                    h[j, :T], d[j, :T], dur[j, :T] = per[i]["h"], per[i]["d"], per[i]["dur"]
                codes = torch.stack([per[i]["codes"] for i in ch]).contiguous()
                pro = eng.prosody_frames(Act(h, 0, S.d_txt), codes, Act(d, 0, S.pr_in), dur, T40)
                wav = eng.decode(pro, codes, [per[i]["seed"] for i in ch])
                for j, i in enumerate(ch):
                    out[i] = wav[j].clone()
        eng.check_status()  # the phase-2 prosody LSTMs
        self.stats = dict(requests=len(reqs), phase1_batches=n1, phase2_batches=n2,
                          frame_buckets=sorted(g2.keys()))
        return out
