#!/usr/bin/env python3
"""Print ceres_scene_info + ceres_scene_shadow_stacks of configs' scenes (reference CMake build's
arithmetic): BVH depth, primary / shadow stack bounds, device bytes.
usage: python tools/scene_info.py [config ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    pkg = bench.import_package()
    for name in sys.argv[1:] or ["dragon_1080"]:
        mesh, bvh, _ = pkg.prepare(pkg.configs.CONFIGS[name], arith=pkg.ARITH_FMA)
        scene = pkg.Scene(mesh, bvh)
        print(name, scene.info(), flush=True)
        scene.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
