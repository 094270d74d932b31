#!/usr/bin/env python3
"""How coherent are the fused kernel's fetches?  Loads a CERES_DIAG_UNIFORM=1 build
(make -C ceres-raytracer_amd/csrc variant VARIANT=diag DEFS=-DCERES_DIAG_UNIFORM=1), renders
bench.py's 8-frame orbit batch of a config and prints, per loop (primary BVH2 steps, primary
triangle tests, shadow BVH4 steps, shadow triangle tests): wave-steps, the fraction in which
every active lane fetches the same record, mean distinct records and mean active lanes per step.

usage: python tools/diag_uniform.py [config] [frames]
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)
from ab import load_build  # noqa: E402
import bench  # noqa: E402


def main():
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    lib = os.environ.get("DIAG_LIB", os.path.join(REPO, "ceres-raytracer_amd", "variants", "libceres_hip_diag.so"))
    mod = load_build(lib, "diag")
    L = mod.lib()
    L.ceres_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    cfg = mod.configs.CONFIGS[name]
    meta = bench.load_golden(name)
    mesh, bvh, cam = mod.prepare(cfg)
    sc = mod.Scene(mesh, bvh)
    W, H = cfg["W"], cfg["H"]
    b12, s3 = bench.step_views(mod, cfg, meta, cam, F, F)
    out = torch.empty(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    buf = (ctypes.c_uint64 * 34)()
    L.ceres_diag_read(buf)
    sc.render_batch_device(b12, s3, W, H, mode=mod.cfg_mode(cfg), d_rgb8=out.data_ptr())
    torch.cuda.synchronize()
    L.ceres_diag_read(buf)
    d = np.frombuffer(buf, np.uint64).astype(np.float64)
    res = {"config": name, "frames": F}
    for i, k in enumerate(("primary_steps", "primary_tris", "shadow_steps", "shadow_tris")):
        s, u, dist, act = d[4 * i: 4 * i + 4]
        nq, nqu, allq = d[16 + 4 * i: 16 + 4 * i + 3]
        res[k] = {"wave_steps": int(s), "uniform_frac": round(u / max(s, 1), 4),
                  "distinct_per_step": round(dist / max(s, 1), 2), "active_per_step": round(act / max(s, 1), 2),
                  "quad_uniform_frac": round(nqu / max(nq, 1), 4), "all_quads_uniform_frac": round(allq / max(s, 1), 4)}
    s0 = max(d[0], 1)
    res["primary_steps"]["distinct_lines_per_step"] = round(d[32] / s0, 2)
    res["primary_steps"]["distinct_lines_sibling_layout"] = round(d[33] / s0, 2)
    print(json.dumps(res, indent=1))
    sc.close()


if __name__ == "__main__":
    main()
