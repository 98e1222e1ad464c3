#!/usr/bin/env python3
"""Print a compact table from a rocprofv3 *_kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>5s}")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r["Name"].replace("twtml::", "")
    name = name[:70]
    print(f"{name:70s} {r['Calls']:>6s} {float(r['TotalDurationNs'])/1e6:9.2f} "
          f"{float(r['AverageNs'])/1e3:9.1f} {100*float(r['TotalDurationNs'])/tot:5.1f}")
