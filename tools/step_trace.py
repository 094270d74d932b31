#!/usr/bin/env python3
"""The timed regime of bench.py under rocprofv3: from a kernel trace of

    rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o run -- \\
        python3 bench.py --steps K --warmup W --no-orbit --no-roofline --no-cpu-baseline

(the same timed loop as the default run; those flags only drop the untimed extra loops that come
after it, so the last K x L render launches of the trace ARE the K timed steps, L launches per
step), report per step: the wall span of those launches, the time the GPU had at least one of
them running (union of their intervals), and their summed durations (> span when the step streams
overlap), next to the bench line's own ms_per_step from the same run.

usage: python tools/step_trace.py <trace dir> <bench log> <out.json> [kernel prefix, default ceres_fused]
"""
import csv
import glob
import json
import os
import sys


def kernel_rows(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows, key=lambda r: r[1])


def union_ns(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def summarize(rows, line, prefix="ceres_fused"):
    K = line["steps"]
    F = line["config"]["frames_per_step"]
    per_launch = 56                                  # kFramesPerLaunch: frames per kernel launch
    L = (F + per_launch - 1) // per_launch if line["n_gpus"] == 1 else None
    ren = [r for r in rows if prefix + "<" in r[0] or r[0].startswith(prefix)]
    timed = ren[-K * L:]
    t0, t1 = timed[0][1], max(r[2] for r in timed)
    # every kernel of any name inside the window (assembly, collectives) counts for the busy time
    window = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    busy = union_ns([(r[1], r[2]) for r in window])
    ksum = sum(r[2] - r[1] for r in timed)
    return {"steps": K, "launches_per_step": L, "kernel": prefix, "frames_per_step": F,
            "render_launches": len(timed), "names_in_window": sorted({r[0].split("(")[0][:60] for r in window}),
            "span_ms_per_step": round((t1 - t0) / 1e6 / K, 5), "busy_ms_per_step": round(busy / 1e6 / K, 5),
            "kernel_ms_per_step": round(ksum / 1e6 / K, 5), "mean_launch_ms": round(ksum / 1e6 / len(timed), 5),
            "overlap": round(ksum / busy, 3) if busy else None,
            "bench_ms_per_step": line["ms_per_step"], "bench_value": line["value"],
            "config": line["config"]["workload"].split(":")[0], "arith": line.get("arith"),
            "streams": line["config"].get("streams")}


def main():
    d, log, out = sys.argv[1:4]
    prefix = sys.argv[4] if len(sys.argv) > 4 else "ceres_fused"
    with open(log) as f:
        line = json.loads([ln for ln in f if ln.startswith("{") and '"metric"' in ln][-1])
    res = summarize(kernel_rows(d), line, prefix)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
