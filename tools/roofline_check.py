"""Cross-check of bench.py's roofline line against a rocprofv3 kernel trace of the same command (tools/prof.sh):
the 36 MRF resblock convs of the instrumented eager batch-64 pass (the LAST 36 Snake-prologue MRF dispatches in the
trace: mrf_conv<2,...> stage 0, mrfv_conv<2,...> stage 1) -> their average duration, to compare with the bench
line's roofline.avg_launch_us (which bench.py measures with HIP events on the launching stream).

    python tools/roofline_check.py gpurun_out/<prof dir>/run_kernel_trace.csv [bench log]
"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if r["Kernel_Name"].startswith(("void (anonymous namespace)::mrf_conv<2,", "void (anonymous namespace)::mrfv_conv<2,"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-36:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
out = dict(source=sys.argv[1], mrf_dispatches_in_trace=len(rows), last_pass_launches=len(last),
           avg_launch_us_rocprof=round(sum(dur) / len(dur), 2),
           grid_x_first_last=[int(last[0]["Grid_Size_X"]), int(last[-1]["Grid_Size_X"])])
if len(sys.argv) > 2:
    line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
    rf = json.loads(line)["roofline"]
    out["avg_launch_us_bench_events"] = rf["avg_launch_us"]
    out["ratio"] = round(out["avg_launch_us_rocprof"] / rf["avg_launch_us"], 3)
print(json.dumps(out, indent=1))
