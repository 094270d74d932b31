#!/usr/bin/env python3
"""Diagnostic: per-wavefront timeline of the persistent frame kernel (stats scene).

Prints the distribution of wave start/end times, chunks fetched, shadow batches, fetch
clocks and node-pair work, to tell load imbalance / tail effects from throughput limits.
usage: python tools/wave_diag.py [config] [frames]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    mesh, bvh, cam = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    out = {}
    for stats in (False, True):
        sc = pkg.Scene(mesh, bvh, stats=stats)
        ms = []
        for _ in range(frames):
            _, _, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], want_pixels=True)
            ms.append(st["ms"])
        out["stats" if stats else "plain"] = {"ms_median": float(np.median(ms)), "ms_min": float(np.min(ms)),
                                             "rays": st["rays"], "pairs": st["node_pairs"], "tests": st["tri_tests"]}
        if stats:
            log = sc.wave_log().astype(np.int64)
            t0 = log[:, 0].min()
            start = (log[:, 0] - t0) / 100.0    # us (100 MHz)
            end = (log[:, 1] - t0) / 100.0
            life = end - start
            q = lambda a: [float(np.percentile(a, p)) for p in (0, 10, 50, 90, 99, 100)]  # noqa: E731
            out["waves"] = int(log.shape[0])
            out["start_us_pct"] = q(start)
            out["end_us_pct"] = q(end)
            out["life_us_pct"] = q(life)
            out["chunks_pct"] = q(log[:, 2])
            out["batches_pct"] = q(log[:, 3])
            out["fetch_clk_pct"] = q(log[:, 4])
            out["pairs_pct"] = q(log[:, 5])
            out["shadow_traced_pct"] = q(log[:, 7])
            out["sum_fetch_clk_over_sum_life_clk"] = float(log[:, 4].sum() / max(1.0, (life.sum() * 2400)))
            np.save(os.path.join(REPO, "gpurun_out", f"wave_log_{name}.npy"), log)
        sc.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
