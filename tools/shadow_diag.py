#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of ceres_shadow (stats scene): per-iteration time per wave."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    mesh, bvh, cam = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    sc = pkg.Scene(mesh, bvh, stats=True)
    for _ in range(3):
        _, _, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"])
    log = sc.wave_log().astype(np.int64)
    log = log[log[:, 0] > 0]
    act = log[log[:, 2] > 0]
    t0 = log[:, 0].min()
    start = (act[:, 0] - t0) / 100.0
    end = (act[:, 1] - t0) / 100.0
    life = end - start
    per_iter = life / act[:, 2]
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (0, 10, 50, 90, 99, 100)]  # noqa: E731
    it = np.maximum(act[:, 3], 1)
    out0 = {"box_clk_per_iter": q(act[:, 4] / it), "leaf_clk_per_iter": q(act[:, 5] / it),
            "next_clk_per_iter": q(act[:, 6] / it), "iters_vs_maxchain": q(act[:, 3] / act[:, 2]),
            "sum_box_leaf_next_clk_over_life_clk": round(float((act[:, 4] + act[:, 5] + act[:, 6]).sum() / (life.sum() * 100 * 24)), 4)}
    out = {**out0,"ms": st["ms"], "waves_logged": int(log.shape[0]), "active_waves": int(act.shape[0]),
           "start_us": q(start), "end_us": q(end), "life_us": q(life), "max_chain": q(act[:, 2]),
           "us_per_iter": q(per_iter), "lane_util": round(float(act[:, 7].sum() / (act[:, 2] * 64).sum()), 4)}
    # corr: long waves
    idx = np.argsort(-life)[:10]
    out["slowest"] = [[round(float(start[i]), 2), round(float(life[i]), 2), int(act[i, 2]), round(float(per_iter[i]), 3)] for i in idx]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
