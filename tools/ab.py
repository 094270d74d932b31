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
        kern, _, tpw = v.partition(":")          # e.g. "wave:4" = wave variant, 4 tiles per wave
        os.environ["CERES_KERNEL"] = kern
        os.environ["CERES_TPW"] = tpw or "1"
        scenes[v] = pkg.Scene(mesh, bvh)
    res = {v: [] for v in variants}
    ok = {}
    for v, sc in scenes.items():
        _, rgb, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode, want_pixels=False)
        ok[v] = hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"]["exact"]
    for _ in range(rounds):
        for v, sc in scenes.items():
            _, _, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode, want_pixels=True, want_rgb8=True)
            res[v].append(st["ms"])
    out = {v: {"median_ms": round(float(np.median(r)), 4), "min_ms": round(float(np.min(r)), 4),
               "mrays_s_median": round(meta["exact"]["rays"] / (np.median(r) * 1e3), 1), "parity": ok[v]}
           for v, r in res.items()}
    print(json.dumps({"config": name, "rounds": rounds, "results": out}))


if __name__ == "__main__":
    main()
