#!/usr/bin/env python3
"""Average PMC counters per kernel over rocprofv3 counter_collection CSVs."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        continue
    for r in rows:
        name = r.get("Kernel_Name", r.get("Kernel-Name", "?")).replace("twtml::", "")[:60]
        cnt = r.get("Counter_Name", "?")
        acc[name][cnt].append(float(r.get("Counter_Value", "nan")))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
