"""Attention kernel A/B across two library builds: the bf16 and precise attention on the denoiser shapes, output hashes saved
(bit comparison) and time per launch (graph-replayed chain of launches, so the batch-1 dependent-launch cost shows).

    STZS_LIB=<lib.so> OUT=<file.json> python tools/attn_ab.py
    python tools/attn_ab.py --compare a.json b.json
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "--compare":
    import json
    a, b = json.load(open(sys.argv[2])), json.load(open(sys.argv[3]))
    for k in a:
        print(f"{k:28s} {'bit-identical' if a[k] == b[k] else 'DIFFERS'}")
    sys.exit(0)

from stzs.engine import Act, StyleTTSZS  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_TINY  # noqa: E402

eng = StyleTTSZS(SPEC_TINY, init_params(SPEC_TINY, 0), device="cuda:0")
out = {}
g = torch.Generator().manual_seed(0)
D, dh = 512, 64
for R, Lq, Lk, prec in [(2, 50, 50, False), (2, 50, 130, False), (128, 50, 50, False), (128, 50, 130, False),
                        (3, 50, 530, False), (2, 50, 50, True), (2, 50, 130, True), (128, 50, 130, True)]:
    dt = torch.float32 if prec else torch.bfloat16
    q = Act((torch.randn(R, Lq, D, generator=g)).to("cuda:0", dt))
    kv = Act((torch.randn(R, Lk, 2 * D, generator=g)).to("cuda:0", dt))
    o = Act(torch.zeros(R, Lq, D, dtype=dt, device="cuda:0"))
    a = eng._attn_args(q, kv.sl(0, D), kv.sl(D, D), o)
    if prec:
        a.precise = 1

    def run(a=a):
        eng._call(eng.lib.stzs_attention, a, "attention")
    run()
    torch.cuda.synchronize()
    key = f"R{R}_Lk{Lk}_{'x3' if prec else 'bf16'}"
    out[key] = hashlib.sha256(o.t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()
    n = 50
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(n):
                run()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{key:28s} {e0.elapsed_time(e1) / (5 * n) * 1e3:7.2f} us per launch (chain of {n}, graph)", flush=True)
json.dump(out, open(os.environ.get("OUT", "attn_out.json"), "w"), indent=1)
