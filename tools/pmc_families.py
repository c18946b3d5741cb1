"""Per-kernel-family HBM traffic and MFMA utilisation of one workload from rocprofv3 PMC passes (each pass in its own
run, --kernel-trace only, as MI355X_MICROARCH.md prescribes; tools/pmc_families.sh collects them).

    python tools/pmc_families.py <dir> [--n-cu 256] > profiles/<tag>_pmc_families.json

<dir>/<pass>/**/run_counter_collection.csv for passes holding FETCH_SIZE, WRITE_SIZE, the MFMA op counters
(SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F8, units of 512 FLOP), SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE; and the
kernel trace of each pass (run_kernel_trace.csv) for the dispatch durations.

Per family (the kernel's base name: mrf_conv, mrfv_conv, ups_conv, gemm_glds, gemm_rows, lstm_xchg, ...):
  * traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE tallies 1/2 of the bytes of wide streaming reads), KB
    -> bytes, summed over the family's dispatches, and as GB/s over their summed duration (vs 8 TB/s);
  * mfma_tflops = MOPS x 512 / duration, frac_bf16 = that / 2500 TFLOP/s (dense bf16; fp8 ops priced at the bf16
    rate: the non-scaled fp8 MFMA runs at the bf16 rate on gfx950);
  * mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x n_CU x 4 SIMDs): the fraction of SIMD cycles the
    matrix pipe was busy (GRBM_GUI_ACTIVE is summed over the 8 XCDs).
Durations come from the pass with the most dispatches; a counter's per-dispatch values are summed over its
instances (per-XCD / per-SE rows)."""
import argparse
import collections
import csv
import glob
import json
import os
import re

PEAK_TF = 2500.0
PEAK_GBS = 8000.0


def family(name):
    m = re.search(r"(?:::|^)(?:void )?(?:\(anonymous namespace\)::)?(\w+)(?:<|\()", name)
    if m:
        return m.group(1)
    return name.split("(")[0].split("<")[0].strip()[-48:]


def load_pass(pdir):
    """-> ({dispatch: {counter: value}}, {dispatch: (family, duration_ns)})"""
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            cnt[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = family(r["Kernel_Name"])
    dur = {}
    for f in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        cf = f.replace("kernel_trace.csv", "counter_collection.csv")
        for r in csv.DictReader(open(f)):
            dur[(cf, r.get("Dispatch_Id") or r.get("Correlation_Id"))] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return cnt, meta, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--n-cu", type=int, default=256)
    a = ap.parse_args()
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(lambda: collections.defaultdict(int))
    durs = collections.defaultdict(dict)
    for pdir in sorted(glob.glob(os.path.join(a.dir, "*"))):
        if not os.path.isdir(pdir):
            continue
        cnt, meta, dur = load_pass(pdir)
        p = os.path.basename(pdir)
        for d, cs in cnt.items():
            f = meta[d]
            for c, v in cs.items():
                fam[f][c] += v
                ndisp[f][c] += 1
            if d in dur:
                durs[p].setdefault(f, []).append(dur[d])
    # durations: the pass that traced the most dispatches of the family
    out = {}
    for f, cs in fam.items():
        best = max((v for v in (durs[p].get(f) for p in durs) if v), key=len, default=None)
        ns = float(sum(best)) if best else 0.0
        n = len(best) if best else max(ndisp[f].values())
        e = dict(dispatches=n, total_us=round(ns / 1e3, 1))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            nf, nw = ndisp[f]["FETCH_SIZE"], ndisp[f]["WRITE_SIZE"]
            byt = (2.0 * cs["FETCH_SIZE"] / nf + cs["WRITE_SIZE"] / nw) * 1024.0 * n
            e["traffic_mb"] = round(byt / 1e6, 1)
            if ns:
                e["hbm_gbs"] = round(byt / ns, 1)
                e["hbm_frac"] = round(byt / ns / PEAK_GBS, 4)
        mops = sum(cs.get(k, 0.0) / max(ndisp[f][k], 1) for k in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F8",
                                                                   "SQ_INSTS_VALU_MFMA_MOPS_F16") if k in cs) * n
        if mops and ns:
            e["mfma_gflop"] = round(mops * 512 / 1e9, 2)
            e["mfma_tflops"] = round(mops * 512 / ns / 1e3, 1)
            e["mfma_frac_bf16"] = round(mops * 512 / ns / 1e3 / PEAK_TF, 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs and cs["GRBM_GUI_ACTIVE"] > 0:
            busy = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / ndisp[f]["SQ_VALU_MFMA_BUSY_CYCLES"]
            act = cs["GRBM_GUI_ACTIVE"] / ndisp[f]["GRBM_GUI_ACTIVE"]
            e["mfma_busy"] = round(busy / (act / 8.0 * a.n_cu * 4), 4)
        out[f] = e
    tot_us = sum(e["total_us"] for e in out.values())
    res = dict(source=a.dir, total_kernel_us=round(tot_us, 1),
               corrections="FETCH_SIZE x 2 (gfx950 wide-read tally, MI355X_MICROARCH.md); MOPS x 512 FLOP",
               families=dict(sorted(out.items(), key=lambda kv: -kv[1]["total_us"])))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
