"""Generate the golden fixtures under tests/golden/ from the CPU oracle (oracle/stzs_ref.py).

    python tests/golden/make_golden.py

The upstream reference has no code, weights or vectors (`/root/reference/README.md:15-16`), so the
fixtures freeze OUR oracle's outputs for HOTPATH spec v0: they catch oracle drift (tests/test_oracle.py)
and give the GPU tests a committed target (tests/test_gpu_golden.py).  Weights are NOT stored: they are
regenerated from (spec, seed) by stzs.params.init_params and fingerprinted by `param_checksum`.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]

import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from oracle import stzs_ref as R  # noqa: E402
from stzs.params import init_params, param_checksum  # noqa: E402
from stzs.spec import SPEC_TINY, SPEC_V0  # noqa: E402


def inputs(S, B, T, seed=1234):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(1, S.n_symbols, (B, T), generator=g)
    ref = torch.randn(B, S.sr // 2, generator=g) * 0.1
    eps = torch.randn(B, S.L_s, S.code_dim, generator=g)
    dur = torch.tensor([[3, 2] * (T // 2)] * B, dtype=torch.int32)
    return tok, ref, eps, dur


def main():
    torch.set_num_threads(8)
    # tiny spec: full synth with forced durations, 2-step CFG-5, and the predicted-duration path
    S = SPEC_TINY
    P = init_params(S, 0)
    tok, ref, eps, dur = inputs(S, 2, 8)
    o = R.synth(P, S, tok, ref, 2, 5.0, eps, dur, seeds=[0, 1])
    pr = R.predict_prosody(P, S, o["h_txt"], o["codes"], None)
    t = {"tok": tok.to(torch.int32), "ref": ref, "eps": eps, "dur": dur, "h_txt": o["h_txt"], "prompt": o["prompt"],
         "prompt_idx": o["prompt_idx"], "prompt_margin": o["prompt_margin"], "codes": o["codes"], "F0": o["F0"], "N": o["N"], "wav": o["wav"], "dur_pred": pr["dur_pred"],
         "dur_sum": pr["dur_sum"]}
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, "tiny_synth.safetensors"),
              metadata={"spec": S.name, "seed": "0", "param_checksum": param_checksum(P), "steps": "2", "cfg": "5.0",
                        "seeds": "0,1"})
    # full v0 dims: 1-s utterance (T_txt 16 -> T40 40), keep outputs only (weights ~98M from the seed)
    S = SPEC_V0
    P = init_params(S, 0)
    tok, ref, eps, dur = inputs(S, 1, 16, seed=99)
    o = R.synth(P, S, tok, ref, 1, 1.0, eps, dur, seeds=[5])
    t = {"tok": tok.to(torch.int32), "ref": ref, "eps": eps, "dur": dur, "prompt_idx": o["prompt_idx"],
         "prompt_margin": o["prompt_margin"], "codes": o["codes"], "F0": o["F0"], "N": o["N"], "wav": o["wav"]}
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(HERE, "v0_synth_1s.safetensors"),
              metadata={"spec": S.name, "seed": "0", "param_checksum": param_checksum(P), "steps": "1", "cfg": "1.0",
                        "seeds": "5"})
    print("wrote golden fixtures")


if __name__ == "__main__":
    main()
