"""The oracle's own floating-point floor on configs[4]: the CPU oracle (oracle/stzs_ref.py) run in
float64 -- parameters, inputs and the harmonic source cast / restated in fp64 -- against the same oracle in fp32, on the
30-s input of tests/test_gpu_stream.py::test_longform_30s_precise_prosody, downstream of one fixed set of style codes
(the fp32 oracle's own 2-step CFG-5 codes, fed to both: the comparison is text encoder -> predictor -> decoder, the part
the GPU's precise long-form mode computes after its fp8 sampler).  Reports log-mel L1 (whole, per 5-s window), waveform
rel-L2, F0 / N rel-L2, and the fp32 decoder teacher-forced on the fp64 F0 / N / aligned features (what is left once the
F0 difference is taken out).  Test infrastructure: CPU only, imports the oracle.

    python tools/oracle_floor.py [--seconds 30] [--threads 8] [--out profiles/r06_oracle_floor.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

from oracle import stzs_ref as R  # noqa: E402


def run(P, S, tok, codes, dur, seeds):
    """text encoder -> prosody predictor (given durations) -> decoder, on fixed codes; fp64 params / codes run every
    oracle op in fp64 (the harmonic source through R.harmonic_source64)."""
    with torch.no_grad():
        h = R.text_encoder(P, S, tok)
        pro = R.predict_prosody(P, S, h, codes, dur)
        wav = R.decode(P, S, pro["asr"], pro["F0"], pro["N"], codes, seeds)
    return dict(wav=wav, F0=pro["F0"], N=pro["N"], asr=pro["asr"])


def logmel_l1(a, b, S):
    return (R.log_mel(a.float(), S) - R.log_mel(b.float(), S)).abs().mean().item()


def windows(a, b, S, sec=5):
    n = sec * S.sr
    return [round(logmel_l1(a[:, i:i + n], b[:, i:i + n], S), 6) for i in range(0, a.shape[1], n)]


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=int, default=30)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    from stzs.params import init_params
    from stzs.spec import SPEC_V0
    S = SPEC_V0
    P = init_params(S, seed=0)
    T = 16 * args.seconds
    g = torch.Generator().manual_seed(77)  # tests/test_gpu_stream.py::test_longform_30s_precise_prosody inputs
    tok = torch.randint(1, S.n_symbols, (1, T), generator=g)
    ref = torch.randn(1, 3 * S.sr, generator=g) * 0.1
    eps = torch.randn(1, S.L_s, S.code_dim, generator=g)
    dur = torch.tensor([[3, 2] * (T // 2)], dtype=torch.int32)
    seeds = [7]
    t0 = time.time()
    codes = R.synth(P, S, tok, ref, 2, 5.0, eps, dur, seeds=seeds)["codes"]
    t1 = time.time()
    o32 = run(P, S, tok, codes, dur, seeds)
    t2 = time.time()
    P64 = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in P.items()}
    o64 = run(P64, S, tok, codes.double(), dur, seeds)
    t3 = time.time()
    # the fp32 decoder on the fp64 predictor's outputs: the decoder's own fp32 floor, F0 difference taken out
    with torch.no_grad():
        wtf = R.decode(P, S, o64["asr"].float(), o64["F0"].float(), o64["N"].float(), codes, seeds)
    t4 = time.time()
    res = dict(
        what="fp32 oracle vs the same oracle in float64 (params, inputs, harmonic source), 2-step CFG-5 codes of the fp32 "
             "oracle fed to both; configs[4] input of test_longform_30s_precise_prosody",
        seconds=args.seconds, threads=args.threads,
        logmel_l1=round(logmel_l1(o32["wav"], o64["wav"], S), 7),
        logmel_l1_per_5s=windows(o32["wav"], o64["wav"], S),
        wav_rel_l2=rel(o32["wav"], o64["wav"]),
        F0_rel_l2=rel(o32["F0"], o64["F0"]), N_rel_l2=rel(o32["N"], o64["N"]), asr_rel_l2=rel(o32["asr"], o64["asr"]),
        decoder_fp32_on_fp64_prosody=dict(logmel_l1=round(logmel_l1(wtf, o64["wav"], S), 7),
                                          logmel_l1_per_5s=windows(wtf, o64["wav"], S)),
        wall_s=dict(codes=round(t1 - t0, 1), fp32=round(t2 - t1, 1), fp64=round(t3 - t2, 1), tf=round(t4 - t3, 1)))
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
