#!/usr/bin/env python3
"""Time the GPU binned-SAH BVH build (ceres_bvh_build_device) against the host build
(ceres_bvh_build, the reference algorithm on the host's cores) on a config's mesh, and check the
GPU result against the fixture's canonical BVH hash.  Prints one JSON line.

  python tools/bvh_bench.py [--config proc_c5] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="proc_c5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host-reps", type=int, default=1)
    args = ap.parse_args()
    import torch
    from conftest import import_package, load_golden
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[args.config]
    mesh = pkg.proc_mesh(cfg["proc"]) if cfg.get("proc") else pkg.load_obj(pkg.configs.obj_path(cfg))
    if cfg.get("rotate"):
        pkg.rotate_triangles(mesh, cfg["rotate"][0], cfg["rotate"][1])
    n = len(mesh)
    dev = torch.device("cuda", 0)
    d_tri = torch.from_numpy(mesh.tri.reshape(-1)).to(dev)
    d_nodes = torch.empty((2 * n - 1) * 8, dtype=torch.int32, device=dev)
    d_prim = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    times = []
    m = 0
    for k in range(args.reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        m = pkg.build_bvh_device(d_tri.data_ptr(), n, d_nodes.data_ptr(), d_prim.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        if k:
            times.append((time.perf_counter() - t0) * 1e3)
    nodes = d_nodes[: m * 8].cpu().numpy().view(np.uint32).reshape(-1, 8)
    prim = d_prim.cpu().numpy().view(np.uint32).astype(np.uint64)
    import oracle
    sha = oracle.canonical_bvh_sha(nodes, prim)
    meta, _, _ = load_golden(args.config)
    host = []
    for _ in range(args.host_reps):
        t0 = time.perf_counter()
        pkg.build_bvh(mesh)
        host.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"config": args.config, "n_tri": n, "n_nodes": m,
                      "gpu_build_ms_median": round(float(np.median(times)), 3), "gpu_build_ms": [round(t, 3) for t in times],
                      "host_build_ms_median": round(float(np.median(host)), 3),
                      "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or os.cpu_count()),
                      "canonical_matches_reference": sha == meta.get("bvh_canonical_sha256")}), flush=True)


if __name__ == "__main__":
    main()
