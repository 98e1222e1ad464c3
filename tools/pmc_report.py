#!/usr/bin/env python3
"""Roofline-style per-kernel table from tools/pmc_r2.sh output.

For every case directory pair <case>_kt (kernel trace) / <case>_p<k> (counter
passes) it prints, per kernel (template instance): calls, mean duration,
VGPR / SGPR / LDS per workgroup, workgroup size, HBM bytes per call
(FETCH_SIZE + WRITE_SIZE, KiB in rocprofv3), the achieved bandwidth, L2 hit
rate, LDS bank-conflict cycles per LDS-active cycle, VALU / MFMA instruction
counts and the mean resident waves per SIMD.

Occupancy: SQ_WAVE_CYCLES accumulates resident waves per quad-cycle over
the whole device and SQ_BUSY_CYCLES is summed over the 32 shader engines
(8 XCDs x 4), so 4 * 32 * SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / 1024 SIMDs is the
mean number of resident waves per SIMD while the SQs were busy.  The scale
checks out on a kernel whose occupancy is fixed by its resources
(k_sgd_iter_hyb: one 1024-thread workgroup per CU = 4 waves per SIMD;
measured 3.8 -- the tail of the last workgroups).
"""
import collections
import csv
import glob
import os
import re
import sys

NUM_SIMD = 256 * 4
NUM_SE = 32


def short(name: str) -> str:
    n = name.replace("twtml::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    depth, out = 0, []
    for ch in n:          # drop the parameter list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()[:58]


def kernel_trace(path):
    rows = list(csv.DictReader(open(path)))
    acc = collections.defaultdict(lambda: {"n": 0, "ns": 0.0})
    for r in rows:
        k = short(r.get("Kernel_Name", "?"))
        a = acc[k]
        a["n"] += 1
        a["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for col, key in (("VGPR_Count", "vgpr"), ("Arch_VGPR_Count", "vgpr"), ("Accum_VGPR_Count", "agpr"),
                         ("SGPR_Count", "sgpr"), ("LDS_Block_Size", "lds"), ("Scratch_Size", "scratch"),
                         ("Workgroup_Size", "wg"), ("Workgroup_Size_X", "wg")):
            if col in r and r[col] not in ("", None):
                a[key] = r[col]
    return acc


def counters(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            acc[short(r.get("Kernel_Name", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def fmt(x, spec):
    return "-" if x is None else format(x, spec)


def report(root):
    cases = sorted({os.path.basename(d).rsplit("_", 1)[0] for d in glob.glob(os.path.join(root, "*_kt"))})
    for case in cases:
        kt_files = glob.glob(os.path.join(root, f"{case}_kt", "**", "*kernel_trace.csv"), recursive=True)
        if not kt_files:
            continue
        kt = kernel_trace(kt_files[0])
        cc = counters(glob.glob(os.path.join(root, f"{case}_p*", "**", "*counter_collection.csv"), recursive=True))
        print(f"\n### {case}\n")
        print("| kernel | calls | mean us | VGPR/AGPR/SGPR | LDS B/WG | WG | HBM MB/call | GB/s | L2 hit | "
              "LDS confl/active | VALU inst/call | MFMA inst/call | waves/SIMD |")
        print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
        for k, c in sorted(cc.items(), key=lambda kv: -kt.get(kv[0], {"ns": 0})["ns"]):
            t = kt.get(k)
            if not t:
                continue
            us = t["ns"] / t["n"] / 1e3
            hbm = None
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hbm = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            gbs = hbm / (us * 1e-6) / 1e9 if hbm is not None and us > 0 else None
            hit = None
            if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
                tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
                hit = c["TCC_HIT_sum"] / tot if tot else None
            confl = None
            if c.get("SQ_ACTIVE_INST_LDS"):
                confl = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_ACTIVE_INST_LDS"]
            occ = None
            if c.get("SQ_BUSY_CYCLES"):
                occ = 4.0 * NUM_SE * c.get("SQ_WAVE_CYCLES", 0.0) / c["SQ_BUSY_CYCLES"] / NUM_SIMD
            regs = f"{t.get('vgpr', '-')}/{t.get('agpr', '-')}/{t.get('sgpr', '-')}"
            print(f"| `{k}` | {t['n']} | {us:.1f} | {regs} | {t.get('lds', '-')} | {t.get('wg', '-')} | "
                  f"{fmt(hbm / 1e6 if hbm is not None else None, '.1f')} | {fmt(gbs, '.0f')} | {fmt(hit, '.2f')} | "
                  f"{fmt(confl, '.3f')} | {fmt(c.get('SQ_INSTS_VALU'), '.3g')} | "
                  f"{fmt(c.get('SQ_INSTS_MFMA'), '.3g')} | {fmt(occ, '.2f')} |")


if __name__ == "__main__":
    report(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_r2")
