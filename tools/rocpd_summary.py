"""Per-kernel summary of a rocprofv3 SQLite output (`rocprofv3 --kernel-trace -d DIR -o p`): calls, average and
total duration per (kernel, grid), largest total first.

    python tools/rocpd_summary.py gpurun_out/DIR/p_results.db [name regex] [--per N]   (--per: divide totals by N)
"""
import re
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
per = 1.0
if "--per" in sys.argv:
    per = float(sys.argv[sys.argv.index("--per") + 1])
    args = [a for a in args if a != sys.argv[sys.argv.index("--per") + 1]]
db, flt = args[0], (args[1] if len(args) > 1 else "")
c = sqlite3.connect(db)
q = """select s.kernel_name, count(*), sum(k.end - k.start), k.grid_size_x / k.workgroup_size_x, k.grid_size_y,
       k.grid_size_z from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s on k.kernel_id = s.id
       group by s.kernel_name, k.grid_size_x, k.grid_size_y, k.grid_size_z order by sum(k.end - k.start) desc"""
tot = 0
for n, cnt, t, gx, gy, gz in c.execute(q):
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n).replace("Ev14stzs_conv_args.kd", "").replace(".kd", "")[:64]
    if flt and not re.search(flt, n):
        continue
    tot += t
    print(f"{short:64s} {cnt / per:8.1f} x {t / cnt / 1e3:8.2f} us = {t / per / 1e3:9.1f} us  grid {gx}x{gy}x{gz}")
print(f"total {tot / per / 1e3:.1f} us")
