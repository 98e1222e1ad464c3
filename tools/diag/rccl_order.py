"""Where the RCCL kernels run in a forced-DP (or multi-rank) engine trace.

python tools/diag/rccl_order.py run_kernel_trace.csv

From a rocprofv3 ``--kernel-trace`` CSV: the compute stream (the one carrying
``k_sgd_*``), the kernel sequence of a typical GD iteration on it, the RCCL
kernels there with per-call time, and for every RCCL kernel on that stream that
is not between ``k_sgd_reduce`` and ``k_sgd_update`` (the prep-packet
all-gather / the stats all-reduce) the prep-stream kernels that overlap it in
time.
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*$", "", name).replace("void ", "").replace("twtml::", "")
    return re.sub(r"<.*$", "", name)


def is_rccl(name: str) -> bool:
    return bool(re.search(r"nccl|rccl", name, re.I))


def is_copy(name: str) -> bool:
    # a world-1 communicator: RCCL's all-gather is a device copy, its in-place
    # all-reduce does nothing on the device
    return name.startswith("__amd_rocclr_copyBuffer")


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
    print(f"compute stream {comp}: {len(seq)} dispatches")
    names = collections.Counter(r["k"] for r in seq)
    for k, v in names.most_common(12):
        print(f"    {v:6d}  {k}")
    # iteration pattern: the kernels from one k_sgd_iter* to the next
    pats = collections.Counter()
    idx = [i for i, r in enumerate(seq) if r["k"].startswith("k_sgd_iter")]
    for a, b in zip(idx, idx[1:]):
        pats[" -> ".join(r["k"] for r in seq[a:b])] += 1
    print("GD iteration patterns on the compute stream (count: sequence):")
    for p, c in pats.most_common(4):
        print(f"  {c:5d}: {p}")
    # RCCL on the compute stream: in-loop (between reduce and update) vs other
    inloop, other = [], []
    for i, r in enumerate(seq):
        if not is_rccl(r["k"]):
            continue
        prev = seq[i - 1]["k"] if i else ""
        nxt = seq[i + 1]["k"] if i + 1 < len(seq) else ""
        (inloop if prev == "k_sgd_reduce" and nxt.startswith("k_sgd_update") else other).append((i, r))
    def us(r):
        return (r["t1"] - r["t0"]) / 1e3
    if inloop:
        d = sorted(us(r) for _, r in inloop)
        print(f"RCCL between k_sgd_reduce and k_sgd_update: {len(inloop)} calls, kernel "
              f"{inloop[0][1]['k']}, median {d[len(d) // 2]:.2f} us, p90 {d[int(0.9 * (len(d) - 1))]:.2f} us")
        # gap reduce-end -> update-start: the collective's whole cost on the stream
        gaps = sorted((seq[i + 1]["t0"] - seq[i - 1]["t1"]) / 1e3 for i, _ in inloop)
        print(f"  k_sgd_reduce end -> k_sgd_update start: median {gaps[len(gaps) // 2]:.2f} us")
    print(f"other RCCL kernels on the compute stream: {len(other)}")
    # what the gradient collective costs the stream: k_sgd_reduce end -> k_sgd_update start
    gaps = sorted((seq[i + 1]["t0"] - r["t1"]) / 1e3 for i, r in enumerate(seq[:-1])
                  if r["k"] == "k_sgd_reduce" and seq[i + 1]["k"].startswith("k_sgd_update") or
                  (r["k"] == "k_sgd_reduce" and i + 2 < len(seq) and seq[i + 2]["k"].startswith("k_sgd_update")))
    if gaps:
        print(f"k_sgd_reduce end -> next kernel (all-reduce on the stream) over {len(gaps)} iterations: "
              f"median {gaps[len(gaps) // 2]:.2f} us, p90 {gaps[int(0.9 * (len(gaps) - 1))]:.2f} us")
    # copies inside the GD loop (between an update and the next iteration
    # kernel): the world-1 packet all-gather issued mid-loop
    mid = [(i, r) for i, r in enumerate(seq) if is_copy(r["k"]) and 0 < i < len(seq) - 1
           and seq[i - 1]["k"].startswith("k_sgd_update") and seq[i + 1]["k"].startswith("k_sgd_iter")]
    print(f"device copies between a GD update and the next iteration (mid-loop all-gather at world 1): {len(mid)}")
    for i, r in mid[:8]:
        ov = collections.Counter(o["k"] for s2, v in streams.items() if s2 != comp for o in v
                                 if o["t0"] < r["t1"] and o["t1"] > r["t0"])
        print(f"  {(r['t1'] - r['t0']) / 1e3:8.2f} us; overlapping other-stream kernels: "
              + (", ".join(f"{k} x{v}" for k, v in ov.most_common(4)) or "none"))
    others = [r for s, v in streams.items() if s != comp for r in v]
    for i, r in other:
        ov = collections.Counter(o["k"] for o in others if o["t0"] < r["t1"] and o["t1"] > r["t0"])
        ctx = f"{seq[i - 1]['k'] if i else '-'} -> [{r['k']}] -> {seq[i + 1]['k'] if i + 1 < len(seq) else '-'}"
        print(f"  {us(r):8.2f} us  {ctx}; overlapping other-stream kernels: "
              + (", ".join(f"{k} x{v}" for k, v in ov.most_common(4)) or "none"))


if __name__ == "__main__":
    main(sys.argv[1])
