#!/usr/bin/env python3
"""Diagnostic: is a C3 frame throughput- or latency(tail)-bound?

1. Per-kernel device time (HIP events) for the full frame and for 1/2, 1/4, 1/8 of its rows
   (ceres_tiling rank 0 of world w): a throughput-bound kernel scales with the work.
2. Shadow-kernel wavefront timeline (stats scene wave log): life of each wave vs its longest
   per-lane chain of node visits -> per-step latency of the critical waves.
usage: python tools/tail_diag.py [config]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    sun = np.asarray(cfg["sun"], np.float32)
    out = {"scaling": {}}
    sc = pkg.Scene(mesh, bvh)
    rgb = torch.empty(3 * W * H, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for world in (1, 2, 4, 8, 16):
        t = pkg.Tiling(16 if world > 1 else H, 0, world)
        for _ in range(5):
            sc.render_device(basis, sun, W, H, tiling=t, d_rgb8=rgb.data_ptr(), stream=st)
        sc.read_timing()
        sc.set_timing(True)
        for _ in range(30):
            sc.render_device(basis, sun, W, H, tiling=t, d_rgb8=rgb.data_ptr(), stream=st)
        p, s, n = sc.read_timing()
        sc.set_timing(False)
        out["scaling"][f"1/{world}"] = {"primary_ms": round(p / n, 4), "shadow_ms": round(s / n, 4)}
    # batched frames for comparison
    for F in (2, 4):
        b12 = np.tile(basis, (F, 1)).astype(np.float32)
        s3 = np.tile(sun, (F, 1)).astype(np.float32)
        big = torch.empty(F * 3 * W * H, dtype=torch.uint8, device="cuda")
        sc.set_timing(True)
        for _ in range(30):
            sc.render_batch_device(b12, s3, W, H, d_rgb8=big.data_ptr(), stream=st)
        p, s, n = sc.read_timing()
        sc.set_timing(False)
        out["scaling"][f"x{F}"] = {"primary_ms": round(p / n, 4), "shadow_ms": round(s / n, 4)}
    sc.close()
    ss = pkg.Scene(mesh, bvh, stats=True)
    ss.render(basis, sun, W, H, want_pixels=False)
    try:
        log = ss.wave_log().astype(np.int64)
    except pkg.CeresError:                      # the fused kernel keeps no wave log
        print(json.dumps(out, indent=1))
        return
    log = log[log[:, 1] > 0]
    if log.shape[0] == 0:
        print(json.dumps(out, indent=1))
        return
    t0 = log[:, 0].min()
    start = (log[:, 0] - t0) / 100.0
    end = (log[:, 1] - t0) / 100.0
    life = end - start
    mp = log[:, 2]
    q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 99, 100)]  # noqa: E731
    busy = mp > 0
    out["shadow_waves"] = int(log.shape[0])
    out["shadow_waves_with_rays"] = int(busy.sum())
    out["span_us"] = round(float(end.max()), 2)
    out["start_us_pct"] = q(start)
    out["life_us_pct"] = q(life[busy])
    out["max_chain_pct"] = q(mp[busy])
    out["us_per_step_pct"] = q(life[busy] / mp[busy])
    top = np.argsort(-life)[:10]
    out["slowest"] = [{"start": round(float(start[i]), 1), "life": round(float(life[i]), 1), "max_chain": int(mp[i]),
                       "wave_tests": int(log[i, 3]), "wave_pairs": int(log[i, 7])} for i in top]
    ss.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
