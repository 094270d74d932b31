#!/usr/bin/env python3
"""A/B kernel variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/ab.py [config] [rounds] [variant ...]   (variants: wave twopass frame)
Prints per-variant device ms per frame (HIP events around the launches), median and min,
and checks every variant renders the reference PPM.
"""
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    variants = sys.argv[3:] or ["wave", "twopass", "frame"]
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    mesh, bvh, cam = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    mode = pkg.MODE_PRIMARY if cfg["mode"] == "primary" else pkg.MODE_FULL
    scenes = {}
    for v in variants:
        # "kernel[:tiles_per_wave[:pf_bits]]", e.g. "wave:1:01" = wave variant, prefetch in shadow only
        parts = v.split(":")
        os.environ["CERES_KERNEL"] = parts[0]
        os.environ["CERES_TPW"] = parts[1] if len(parts) > 1 and parts[1] else "1"
        if len(parts) > 2:
            os.environ["CERES_PF"] = parts[2]
        else:
            os.environ.pop("CERES_PF", None)
        scenes[v] = pkg.Scene(mesh, bvh)
    res = {v: [] for v in variants}
    ok = {}
    for v, sc in scenes.items():
        _, rgb, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode, want_pixels=False)
        ok[v] = hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"]["exact"]
    want_px = os.environ.get("AB_FLOAT", "1") == "1"
    for _ in range(rounds):
        for v, sc in scenes.items():
            _, _, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode, want_pixels=want_px, want_rgb8=True)
            res[v].append(st["ms"])
    out = {v: {"median_ms": round(float(np.median(r)), 4), "min_ms": round(float(np.min(r)), 4),
               "mrays_s_median": round(meta["exact"]["rays"] / (np.median(r) * 1e3), 1), "parity": ok[v]}
           for v, r in res.items()}
    print(json.dumps({"config": name, "rounds": rounds, "results": out}))


if __name__ == "__main__":
    main()
