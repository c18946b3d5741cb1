"""Summarise tools/sq_pmc.sh output: per mrfv_conv template, each SQ counter averaged over dispatches, the MFMA-busy
fraction (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1 024 SIMDs)), wait / issue shares of SQ_WAVE_CYCLES, the
LDS bank-conflict share, and the effective clock from GRBM_GUI_ACTIVE / 8 over the kernel-trace duration.
    python tools/sq_summary.py gpurun_out/sq_<tag> > out.json"""
import collections
import csv
import json
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")):
        if "mrfv_conv" in r["Kernel_Name"]:
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for r in csv.DictReader(open(f"{d}/{p}/run_kernel_trace.csv")):
        if "mrfv_conv" in r["Kernel_Name"]:
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for n, c in vals.items():
    a = {k: sum(v) / len(v) for k, v in c.items()}
    wc, gui = a.get("SQ_WAVE_CYCLES", 1.0), a.get("GRBM_GUI_ACTIVE", 1.0)
    t_ns = sorted(dur[n])[len(dur[n]) // 2] if dur[n] else None
    out[n.replace("void (anonymous namespace)::", "").split("(")[0]] = dict(
        mfma_busy=round(a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 1024), 3),
        clock_ghz=round(gui / 8 / t_ns, 3) if t_ns else None,
        wait_inst_any=round(a.get("SQ_WAIT_INST_ANY", 0) / wc, 3), wait_inst_lds=round(a.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
        active_valu=round(a.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3), active_lds=round(a.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3),
        lds_bank_conflict_share=round(a.get("SQ_LDS_BANK_CONFLICT", 0) / max(a.get("SQ_LDS_IDX_ACTIVE", 1), 1), 3),
        kernel_us_median=round(t_ns / 1e3, 1) if t_ns else None)
print(json.dumps(out, indent=1))
