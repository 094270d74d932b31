#!/usr/bin/env python3
"""CPU simulation of wave-wide packet traversal (tools/probes/packet_sim.cpp) on a bench config.

usage: python tools/packet_sim.py [config] [views]   (default dragon_1080, 2 of the 16 bench views)
Dumps the config's triangles, reference BVH and bench views to /tmp, builds the simulator with g++
and prints per-tile step counts of the per-lane loops and of a masked packet (primary and shadow).
"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    views = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    pkg = bench.import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta = bench.load_golden(name)
    mesh, bvh, cam = pkg.prepare(cfg)
    F = 16
    b12, s3, _ = pkg.bench_views(cam, cfg["sun"], cfg["W"], cfg["H"], F, basis0=bench.pinned_basis(meta, cfg, cam))
    base = f"/tmp/packet_sim_{name}"
    mesh.tri.astype(np.float32).tofile(base + ".tri")
    bvh.nodes.astype(np.uint32).tofile(base + ".nodes")
    bvh.prim.astype(np.uint64).tofile(base + ".prim")
    np.concatenate([b12.reshape(-1), s3.reshape(-1)]).astype(np.float32).tofile(base + ".views")
    exe = "/tmp/packet_sim"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(REPO, "tools", "probes", "packet_sim.cpp"), "-o", exe],
                   check=True)
    subprocess.run([exe, base, str(cfg["W"]), str(cfg["H"]), str(F), str(views)], check=True)


if __name__ == "__main__":
    main()
