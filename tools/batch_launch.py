#!/usr/bin/env python3
"""The launch bench.py's roofline blocks time, alone, for rocprofv3 (--kernel-trace --stats, or
one --pmc counter group per run): `n` launches back to back on ONE stream of

  frames = 1:  one whole frame of the config's own view (bench.py `roofline_solo`), or
  frames = F:  one ceres_render_batch_device launch of F frames, whole: F copies of the config's
               view (views = config, bench.py's default step and `roofline` launch) or the first F
               orbit views of the step (views = orbit, pkg.bench_views),

in the chosen arithmetic (fma = the reference CMake build's, exact = -ffp-contract=off), with the
float + RGB8 framebuffers bench.py writes.  Prints the mean launch duration from HIP events.

usage: python tools/batch_launch.py [config] [fma|exact] [frames] [n] [config|orbit]
BL_BUFFERS=float|rgb8 writes only that framebuffer (the write-amplification split), default both.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    arith_s = sys.argv[2] if len(sys.argv) > 2 else "fma"
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    views = sys.argv[5] if len(sys.argv) > 5 else "config"
    pkg = bench.import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta = bench.load_golden(name)
    build = "ref" if arith_s == "fma" else "exact"
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    scene = pkg.Scene(mesh, bvh)
    mode = pkg.cfg_mode(cfg, arith)
    b12, s3, _ = pkg.bench_views(cam, cfg["sun"], W, H, max(frames, 1),
                                 basis0=bench.pinned_basis(meta, cfg, cam, build))
    if views == "config" or cfg.get("bench_view0"):
        b12, s3 = np.repeat(b12[:1], len(b12), 0), np.repeat(s3[:1], len(s3), 0)
    rgb = torch.empty(frames * 3 * W * H, dtype=torch.uint8, device="cuda")
    px = torch.empty(frames * 3 * W * H, dtype=torch.float32, device="cuda")
    bufs = os.environ.get("BL_BUFFERS", "both")
    d_px = px.data_ptr() if bufs in ("both", "float") else 0
    d_rgb = rgb.data_ptr() if bufs in ("both", "rgb8") else 0
    st = torch.cuda.current_stream()
    whole = pkg.Tiling(H, 0, 1)

    def launch():
        if frames == 1:
            scene.render_device(b12[0], s3[0], W, H, mode=mode, tiling=whole, d_pixels=d_px,
                                d_rgb8=d_rgb, stream=st.cuda_stream)
        else:
            scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=whole, d_pixels=d_px,
                                      d_rgb8=d_rgb, stream=st.cuda_stream)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        launch()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{name} {arith_s} frames={frames} views={views} buffers={bufs} launches={n} mean_launch_ms={ms:.5f}", flush=True)
    scene.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
