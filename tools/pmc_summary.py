#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV runs per kernel (mean per dispatch) -> profiles/pmc_summary.json.

HBM bytes follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and
WRITE_SIZE are KiB (TCC_EA0_RDREQ/WRREQ x 64 B); on gfx950 FETCH_SIZE reads 1/2 of the bytes
of wide (16 B/lane) reads, so the read side is doubled ("gfx950 x2 correction").  Our loads
are 16-B per lane (global_load_dwordx4), the calibrated case.

usage: tools/pmc_summary.py <config> <prof_dir> [<out.json>] [<kernel-key suffix>]
(the suffix, e.g. "_batch16_fma", names the launch profiled; entries of other kernels / suffixes
of the same config are kept)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {k: k for k in ("ceres_fused", "ceres_primary", "ceres_finalize", "ceres_assemble")}


def short(name):
    for k in SHORT:
        if k in name:
            return k
    return None


def load(prof_dir):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(prof_dir, "*", "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                acc[k][(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    out = {}
    for k, d in acc.items():
        per = defaultdict(list)
        for (cname, _), vals in d.items():
            per[cname].append(sum(vals))            # sum over instances (XCDs / channels) per dispatch
        out[k] = {c: sum(v) / len(v) for c, v in per.items()}
        out[k]["dispatches"] = max(len(v) for v in per.values())
    return out


def main():
    cfg, prof = sys.argv[1], sys.argv[2]
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_summary.json")
    suffix = sys.argv[4] if len(sys.argv) > 4 else ""
    data = load(prof)
    summ = json.load(open(dst)) if os.path.exists(dst) else {}
    entry = {}
    for k, c in data.items():
        e = {"counters_mean_per_dispatch": {n: round(v, 1) for n, v in sorted(c.items())}}
        if "FETCH_SIZE" in c:
            rd = c["FETCH_SIZE"] * 1024 * 2
            wr = c.get("WRITE_SIZE", 0.0) * 1024
            e["hbm_read_bytes_per_launch"] = int(rd)
            e["hbm_write_bytes_per_launch"] = int(wr)
            e["hbm_bytes_per_launch"] = int(rd + wr)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) > 0:
            e["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU", 0) > 0:
            e["valu_lane_utilisation"] = round(c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64), 4)
        g = c.get("GRBM_GUI_ACTIVE", 0)
        if g > 0:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs, the TA / TD / TCP sums over the 256 CUs'
            # instances: busy fraction = sum / (256 x GRBM / 8)
            for n, key in (("TA_TA_BUSY_sum", "ta_busy_frac"), ("TD_TD_BUSY_sum", "td_busy_frac")):
                if n in c:
                    e[key] = round(c[n] / (32.0 * g), 4)
        if "TCC_REQ_sum" in c:
            e["l2_requests_per_launch"] = int(c["TCC_REQ_sum"])
        if "TCP_TCC_READ_REQ_sum" in c and c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) > 0:
            e["l1_to_l2_read_frac"] = round(c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
        if c.get("SQ_WAVE_CYCLES", 0) > 0:
            for n, key in (("SQ_WAIT_INST_ANY", "issue_stall_frac"), ("SQ_WAIT_ANY", "waitcnt_parked_frac"),
                           ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
                if n in c:
                    e[key] = round(c[n] / c["SQ_WAVE_CYCLES"], 4)
        entry[k + suffix] = e
    summ.setdefault(cfg, {}).update(entry)
    with open(dst, "w") as f:
        json.dump(summ, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
