"""Per-batch busy / idle time of the LR engine's compute stream.

python tools/diag/compute_gaps.py run_kernel_trace.csv

From a rocprofv3 ``--kernel-trace`` CSV: the compute stream (the one
carrying ``k_sgd_*``) is cut into batches at each ``k_batch_init``; per batch
it prints the span (first kernel start .. last kernel end), the kernel-busy
time inside it, the idle gap before the next batch's first kernel, and what
ran on the other streams during that gap -- where a step goes that is not GD.
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::|twtml::", "", name)
    name = re.sub(r"\(.*$", "", name).replace("void ", "")
    return re.sub(r"<.*$", "", name)


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["k"] = short(r["Kernel_Name"])
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    streams = collections.defaultdict(list)
    for r in rows:
        streams[r["Stream_Id"]].append(r)
    for v in streams.values():
        v.sort(key=lambda r: r["t0"])
    comp = max(streams, key=lambda s: sum(1 for r in streams[s] if r["k"].startswith("k_sgd_")))
    seq = streams[comp]
    starts = [i for i, r in enumerate(seq) if r["k"] == "k_batch_init"]
    others = [r for s, v in streams.items() if s != comp for r in v]
    print(f"compute stream {comp}: {len(starts)} batches")
    print(f"{'batch':>5} {'span_us':>9} {'busy_us':>9} {'gap_after_us':>12}  other streams during the gap")
    for b, (a, z) in enumerate(zip(starts, starts[1:] + [len(seq)])):
        ks = seq[a:z]
        span = (ks[-1]["t1"] - ks[0]["t0"]) / 1e3
        # busy: union of kernel intervals
        busy, cur0, cur1 = 0, None, None
        for r in ks:
            if cur1 is None or r["t0"] > cur1:
                if cur1 is not None:
                    busy += cur1 - cur0
                cur0, cur1 = r["t0"], r["t1"]
            else:
                cur1 = max(cur1, r["t1"])
        busy += cur1 - cur0
        gap = (seq[z]["t0"] - ks[-1]["t1"]) / 1e3 if z < len(seq) else float("nan")
        desc = ""
        if z < len(seq):
            g0, g1 = ks[-1]["t1"], seq[z]["t0"]
            ov = collections.Counter(o["k"] for o in others if o["t0"] < g1 and o["t1"] > g0)
            desc = ", ".join(f"{k} x{v}" for k, v in ov.most_common(5))
        print(f"{b:5d} {span:9.1f} {busy / 1e3:9.1f} {gap:12.1f}  {desc}")


if __name__ == "__main__":
    main(sys.argv[1])
