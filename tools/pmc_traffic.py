"""HBM traffic per launch of the dominant kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md 'HBM' prescribes: FETCH_SIZE (KB) reports 1/2 of the bytes of wide
streaming reads on gfx950 -> x2; WRITE_SIZE (KB) exact for 16-B-per-lane stores.

Besides the average over every matching dispatch, the generator MRF convs (mrfv_conv<PACT, HR, HA, KS, NCH, AL, WPW>)
are broken out per shape -- stage (NCH 1: 128 channels x 24 001 rows; WPW 2: 256 x 4 000), kernel width, residual /
accumulate operands and batch (from the grid: one workgroup per (utterance, 128-row tile[, 256-channel tile])) --
each against its algorithmic bytes (input once, output once, + residual, + accumulate; bf16; weights once).
`traffic_bytes_per_launch` is the average over the B = 64 dispatches when there are any (the bench's roofline pass
runs the 64-utterance batch; the timed shards are 32 each).
usage: python tools/pmc_traffic.py <dir with FETCH_SIZE/ and WRITE_SIZE/> <kernel substring[|substring...]> > out.json"""
import csv
import glob
import json
import os
import re
import sys

d, sub = sys.argv[1], sys.argv[2]
subs = sub.split("|")
STAGE = {1: (128, 24001), 2: (256, 4000)}  # stage-1 (NCH 1) / stage-0 (wide, WPW 2) channels, rows at configs[2]


def per_dispatch(counter):
    vals = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(x in r["Kernel_Name"] for x in subs) and r["Counter_Name"] == counter:
                key = (r.get("Dispatch_Id", r.get("Correlation_Id")), r["Kernel_Name"], int(r["Grid_Size"]))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals


def shape(name, grid):
    m = re.search(r"mrfv_conv<(\d+), (true|false), (true|false), (\d+), (\d+), (true|false), (\d+)(?:, (\d+))?>", name)
    if not m:
        return None
    pact, hr, ha, ks, nch, _, wpw, bt = m.groups()
    ks, nch, wpw, bt = int(ks), int(nch), int(wpw), int(bt or 128)
    st = 1 if nch == 1 else (2 if wpw == 2 else 0)
    if st == 0 or pact != "2":
        return None
    C, T = STAGE[st]
    wgs = grid // 256
    B = wgs // ((T + bt - 1) // bt)  # (mrfv_conv<..., BT>: 128- or 64-row tiles)
    nop = 2 + (hr == "true") + (ha == "true")
    alg = B * T * C * 2 * nop + ks * C * C * 2
    form = "c1" if hr == "false" else ("c2+acc" if ha == "true" else "c2")
    return (f"stage {1 if st == 1 else 0} k{ks} {form} B{B}", B, alg)


fetch, write = per_dispatch("FETCH_SIZE"), per_dispatch("WRITE_SIZE")
if not fetch or not write:
    sys.exit(f"no dispatches of {sub!r} in {d}")
groups = {}
for cnt, vals in (("f", fetch), ("w", write)):
    for (_, name, grid), v in vals.items():
        sh = shape(name, grid)
        if sh is None:
            continue
        g = groups.setdefault(sh[0], dict(B=sh[1], alg=sh[2], f=[], w=[]))
        g[cnt].append(v)
by_shape = {}
for k in sorted(groups):
    g = groups[k]
    if not g["f"] or not g["w"]:
        continue
    t = (2.0 * sum(g["f"]) / len(g["f"]) + sum(g["w"]) / len(g["w"])) * 1024.0
    by_shape[k] = dict(dispatches=len(g["f"]), traffic_bytes=round(t), alg_bytes=g["alg"],
                       ratio=round(t / g["alg"], 3), B=g["B"])
f_kb = sum(fetch.values()) / len(fetch)
w_kb = sum(write.values()) / len(write)
traffic = (2.0 * f_kb + w_kb) * 1024.0
b64 = [v for v in by_shape.values() if v["B"] == 64]
out = dict(kernel=sub, dispatches=[len(fetch), len(write)], fetch_size_kb_avg=round(f_kb, 1),
           write_size_kb_avg=round(w_kb, 1), correction="FETCH_SIZE x 2 (gfx950 wide-read tally)",
           traffic_bytes_all_dispatches=round(traffic))
if b64:
    n = sum(v["dispatches"] for v in b64)
    tb = sum(v["traffic_bytes"] * v["dispatches"] for v in b64) / n
    ab = sum(v["alg_bytes"] * v["dispatches"] for v in b64) / n
    out.update(traffic_bytes_per_launch=round(tb), alg_bytes_per_launch_b64=round(ab), ratio_b64=round(tb / ab, 3),
               traffic_scope="the B = 64 generator MRF dispatches (the bench's roofline pass)")
else:
    out.update(traffic_bytes_per_launch=round(traffic), traffic_scope="every matching dispatch")
out["by_shape"] = by_shape
print(json.dumps(out, indent=1))
