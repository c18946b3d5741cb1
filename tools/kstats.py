"""Summarise a rocprofv3 kernel_stats.csv per synth step: python tools/kstats.py <csv> [passes]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 18]:
    print(f"{float(r['TotalDurationNs'])/1e6/n:8.2f} ms/pass {float(r['Percentage']):6.2f}% n/pass={int(r['Calls'])/n:>6.1f} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:96]}")
print(f"total {tot/1e6/n:.2f} ms/pass")
