#!/usr/bin/env python3
"""Where a batch's wave-time goes: primary phase vs shadow phase of the fused kernel.

Stats scene (diagnostic build of the same kernel, s_memrealtime per wave at 100 MHz), bench.py's
8-frame orbit batch in ONE launch (the throughput path: one shadow ray per lane over the BVH4).
Sums resident wave-time over all waves: primary (start -> after the closest-hit pass) and
shadow + shading (-> end), and the same split for waves with and without shadow rays.
usage: python tools/phase_split.py [config] [frames]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
from conftest import import_package  # noqa: E402
import bench  # noqa: E402


def main():
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta = bench.load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    sc = pkg.Scene(mesh, bvh, stats=True)
    b12, s3 = bench.step_views(pkg, cfg, meta, cam, F, F)
    out = torch.empty(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        sc.render_batch_device(b12, s3, W, H, mode=pkg.cfg_mode(cfg), d_rgb8=out.data_ptr())
    torch.cuda.synchronize()
    log = sc.wave_log(1 << 22).astype(np.int64)
    t0, tp, te = log[:, 0], log[:, 1], log[:, 2]
    nshadow = log[:, 5]
    prim, shad = (tp - t0).astype(np.float64), (te - tp).astype(np.float64)
    span = (te.max() - t0.min()) / 100.0
    has = nshadow > 0
    res = {"config": name, "frames": F, "waves": int(len(log)), "launch_us": round(span, 1),
           "wave_us_total": round((prim.sum() + shad.sum()) / 100.0, 1),
           "primary_frac": round(prim.sum() / (prim.sum() + shad.sum()), 4),
           "shadow_frac": round(shad.sum() / (prim.sum() + shad.sum()), 4),
           "waves_with_shadow_rays": int(has.sum()),
           "mean_wave_us": {"no_shadow": round(prim[~has].mean() / 100.0 + shad[~has].mean() / 100.0, 2),
                            "with_shadow_primary": round(prim[has].mean() / 100.0, 2),
                            "with_shadow_shadow": round(shad[has].mean() / 100.0, 2)},
           "mean_shadow_rays_per_wave": round(float(nshadow[has].mean()), 1)}
    print(json.dumps(res, indent=1))
    sc.close()


if __name__ == "__main__":
    main()
