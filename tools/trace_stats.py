#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace run (its rocpd SQLite output, <dir>/*.db) as
a CSV like rocprofv3's kernel_stats.csv: name, calls, total / mean / min / max duration (ns),
percentage, VGPRs, LDS bytes, grid size.

usage: python tools/trace_stats.py <trace dir> [out.csv]
"""
import csv
import glob
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(d, "kernel_stats.csv")
    rows = {}
    for db in glob.glob(os.path.join(d, "*.db")):
        con = sqlite3.connect(db)
        for name, dur, vgpr, lds, gx in con.execute("select name, duration, vgpr_count, lds_size, grid_x from kernels"):
            r = rows.setdefault(name, {"durs": [], "vgpr": vgpr, "lds": lds, "grid": gx})
            r["durs"].append(float(dur))
    total = sum(sum(r["durs"]) for r in rows.values()) or 1.0
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage", "VGPRs",
                    "LdsBytes", "GridX"])
        for name, r in sorted(rows.items(), key=lambda kv: -sum(kv[1]["durs"])):
            ds = r["durs"]
            w.writerow([name, len(ds), round(sum(ds), 1), round(sum(ds) / len(ds), 1), round(min(ds), 1),
                        round(max(ds), 1), round(100.0 * sum(ds) / total, 3), r["vgpr"], r["lds"], r["grid"]])
    print(open(out).read())


if __name__ == "__main__":
    main()
