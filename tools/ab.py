#!/usr/bin/env python3
"""A/B kernel builds in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/ab.py [config] [rounds] [lib.so[@qbvh][#tag] ...]
Each argument is a build of libceres_hip.so (default: the in-tree one), e.g. one made with
`make -C ceres-raytracer_amd/csrc variant VARIANT=x DEFS=-DFOO`.  AB_ARITH=fma|exact (default fma,
bench.py's default): the reference CMake build's arithmetic or the contraction-free one.  Every build is loaded as its
own module instance (own ctypes handle, own HIP code object) and renders the config
alternately; prints device ms per frame (HIP events), median and min, and PPM parity.
"""
import hashlib
import importlib.util
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "ceres-raytracer_amd")
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_golden  # noqa: E402


def load_build(path, tag):
    spec = importlib.util.spec_from_file_location(f"ceres_ab_{tag}", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.LIB_PATH = os.path.abspath(path)
    mod.lib()
    return mod


def main():
    # kernel A/B: a host-buffer render is ONE launch (ceres_render_f32 splits frames of >= 32 MB into
    # row bands whose copies overlap later bands; their device time would include the bands' tails)
    os.environ.setdefault("CERES_HOST_BANDS", "1")
    import torch  # noqa: F401  (one HIP runtime for every build)
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    libs = sys.argv[3:] or [os.path.join(PKG_DIR, "libceres_hip.so")]
    meta, _, _ = load_golden(name)
    # "lib.so@qbvh": the same build rendering with CERES_MODE_QBVH4 (parity then means the budget);
    # "lib.so#2": a second instance of the same build (own scene copy: an A/A check of how much the
    # scene's placement in memory moves the timings)
    builds = {os.path.basename(p): load_build(p.split("#")[0].split("@")[0], i) for i, p in enumerate(libs)}
    qflag = {k: (m.MODE_QBVH4 if "@qbvh" in k else 0) for k, m in builds.items()}
    first = next(iter(builds.values()))
    cfg = first.configs.CONFIGS[name]
    build = "ref" if os.environ.get("AB_ARITH", "fma") == "fma" else "exact"
    arith = 1 if build == "ref" else 0
    mesh, bvh, cam = first.prepare(cfg, arith=arith)
    bb = meta["ref_basis"] if build == "ref" else meta["basis"]
    bits = [int(h, 16) for h in bb["dir"] + bb["u"] + bb["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    mode0 = first.cfg_mode(cfg, arith)
    scenes = {k: m.Scene(mesh, bvh) for k, m in builds.items()}
    ok = {}
    for k, sc in scenes.items():
        _, rgb, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode0 | qflag[k], want_pixels=False)
        ok[k] = hashlib.sha256(builds[k].ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"][build]
    want_px = os.environ.get("AB_FLOAT", "1") == "1"
    res = {k: [] for k in scenes}
    n_streams = int(os.environ.get("AB_STREAMS", "0"))
    if n_streams:
        # throughput regime (bench.py --streams S): AB_FRAMES frames round-robin over S streams
        # per round, wall ms per frame
        import time
        import torch
        W, H = cfg["W"], cfg["H"]
        per = int(os.environ.get("AB_FRAMES", "64"))
        strs = [torch.cuda.Stream() for _ in range(n_streams)]
        px = [torch.empty(3 * W * H, dtype=torch.float32, device="cuda") for _ in range(n_streams)]
        rgb = [torch.empty(3 * W * H, dtype=torch.uint8, device="cuda") for _ in range(n_streams)]
        b12 = basis[None, :].astype(np.float32)
        s3 = np.asarray(cfg["sun"], np.float32)[None, :]
        nb = int(os.environ.get("AB_BATCH", "1"))      # frames per launch (bench.py's --frames-per-gpu)
        if nb > 1:
            # bench.py's step views (pkg.bench_views); AB_VIEW0=1: nb copies of frame 0 (the C5 orbit
            # turns away from the heightfield for half of its views)
            b12, s3, _ = first.bench_views(cam, cfg["sun"], W, H, nb, basis0=basis)
            if os.environ.get("AB_VIEW0") == "1":
                b12, s3 = np.repeat(b12[:1], nb, 0), np.repeat(s3[:1], nb, 0)
            px = [torch.empty(nb * 3 * W * H, dtype=torch.float32, device="cuda") for _ in range(n_streams)]
            rgb = [torch.empty(nb * 3 * W * H, dtype=torch.uint8, device="cuda") for _ in range(n_streams)]
        for _ in range(rounds):
            for k, sc in scenes.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for f in range(per):
                    i = f % n_streams
                    sc.render_batch_device(b12, s3, W, H, mode=mode0 | qflag[k], d_pixels=px[i].data_ptr() if want_px else 0,
                                           d_rgb8=rgb[i].data_ptr(), stream=strs[i].cuda_stream)
                torch.cuda.synchronize()
                res[k].append((time.perf_counter() - t0) * 1e3 / (per * nb))
    for _ in range(0 if n_streams else rounds):
        for k, sc in scenes.items():
            _, _, st = sc.render(basis, cfg["sun"], cfg["W"], cfg["H"], mode=mode0 | qflag[k], want_pixels=want_px,
                                 want_rgb8=True)
            res[k].append(st["ms"])
    out = {k: {"median_ms": round(float(np.median(r)), 4), "min_ms": round(float(np.min(r)), 4),
               "mrays_s_median": round(meta[build]["rays"] / (np.median(r) * 1e3), 1), "parity": ok[k]}
           for k, r in res.items()}
    print(json.dumps({"config": name, "arith": build, "rounds": rounds, "streams": n_streams, "results": out}))


if __name__ == "__main__":
    main()
