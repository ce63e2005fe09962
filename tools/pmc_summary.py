#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs (kernel trace stats + PMC passes) per kernel.

Usage: pmc_summary.py <profile dir> [--last K]

For every kernel: the --stats average over all dispatches, and (with --last K) the
average over the last K dispatches of the kernel trace -- bench.py times its last K
launches (the steady-state window after burn-in and warmup), so that is the figure
that must agree with bench.py's HIP-event kernel_ms.  PMC counters are averaged the
same two ways.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads 1/2
of the bytes of a wide coalesced stream (128-B requests tallied at 64 B), so the read
side is doubled; WRITE_SIZE is taken as is.  Both are in KiB.  (The doubling is
calibrated for 16 B/lane streams -- the step kernels' bulk loads are 16 B/lane
global_load_lds or 128-B row segments -- so treat the absolute as approximate.)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def derive(d):
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
        d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        ns = d.get("avg_ns")
        if ns:
            d["hbm_GBps"] = d["hbm_bytes_per_launch"] / ns
    if "SQ_INSTS_VALU" in d and d.get("SQ_WAVES"):
        d["valu_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        d["salu_per_wave"] = d.get("SQ_INSTS_SALU", 0) / d["SQ_WAVES"]
    # wave-cycle attribution (MI355X_MICROARCH.md, PMC slots): WAVE_CYCLES = WAIT_ANY
    # (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue-stalled) + ACTIVE_INST_ANY
    # (issuing), all in quad-cycles; ACTIVE_INST_<unit> split the issuing part
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        att = {}
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_FLAT", "SQ_ACTIVE_INST_MISC"):
            if k in d:
                att[k[3:].lower() + "_frac"] = round(d[k] / wc, 4)
        if d.get("SQ_WAVES"):
            att["wave_life_cycles"] = round(4 * wc / d["SQ_WAVES"], 1)
        d["wave_cycle_attribution"] = att


def main(out, last=0):
    summ = {"kernels": {}, "last_k": last}
    st = glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        for r in rows(st[0]):
            summ["kernels"].setdefault(r["Name"], {}).update(
                {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                 "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                 "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])})
    tr = glob.glob(os.path.join(out, "kt", "**", "*kernel_trace.csv"), recursive=True)
    if tr and last:
        per = defaultdict(list)
        for r in rows(tr[0]):
            per[r["Kernel_Name"]].append((int(r["Dispatch_Id"]),
                                          int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for k, v in per.items():
            v.sort()
            tail = [x[1] for x in v[-last:]]
            summ["kernels"].setdefault(k, {})["last_k_avg_ns"] = sum(tail) / len(tail)
    for p in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(lambda: defaultdict(list))
        for r in rows(p):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or "?"
            acc[name][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for k, cs in acc.items():
            d = summ["kernels"].setdefault(k, {})
            for c, v in cs.items():
                d[c] = sum(x[1] for x in v) / len(v)     # per-dispatch average
                if last:
                    v.sort()
                    tail = [x[1] for x in v[-last:]]
                    d.setdefault("last_k", {})[c] = sum(tail) / len(tail)
    for k, d in summ["kernels"].items():
        derive(d)
        if "last_k" in d:
            lk = d["last_k"]
            lk["avg_ns"] = d.get("last_k_avg_ns")
            derive(lk)
    print(json.dumps(summ, indent=1, sort_keys=True))


if __name__ == "__main__":
    a = sys.argv[1:]
    k = 0
    if "--last" in a:
        i = a.index("--last")
        k = int(a[i + 1])
        del a[i:i + 2]
    main(a[0], k)
