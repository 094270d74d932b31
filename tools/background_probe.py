#!/usr/bin/env python3
"""What a background tile costs in the batch regime: one 16-frame ceres_render_batch_device
launch (whole frames, one stream, HIP events around n launches) of

  orbit       the bench step's 16 orbit views (bench.py's roofline launch),
  away        the same views with the view direction negated: every primary ray leaves the
              scene's root box behind it, so every tile is a background tile (stores only),
  away_rgb8   `away` without the float framebuffer (RGB8 stores only),
  orbit_rgb8  `orbit` without the float framebuffer.

away ÷ orbit bounds the share of a batch that background tiles take; away_rgb8 against away is
the float framebuffer's store cost.  usage: python tools/background_probe.py [config] [n]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    pkg = bench.import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta = bench.load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg, arith=pkg.ARITH_FMA)
    scene = pkg.Scene(mesh, bvh)
    mode = pkg.cfg_mode(cfg, pkg.ARITH_FMA)
    b12, s3, _ = pkg.bench_views(cam, cfg["sun"], W, H, 16, basis0=bench.pinned_basis(meta, cfg, cam, "ref"))
    away = b12.copy()
    away[:, 3:6] *= -1.0
    rgb = torch.empty(16 * 3 * W * H, dtype=torch.uint8, device="cuda")
    px = torch.empty(16 * 3 * W * H, dtype=torch.float32, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    whole = pkg.Tiling(H, 0, 1)
    out = {}
    for tag, views, floats in (("orbit", b12, True), ("away", away, True), ("away_rgb8", away, False),
                               ("orbit_rgb8", b12, False)):
        def launch(counters=0):
            scene.render_batch_device(views, s3, W, H, mode=mode, tiling=whole, d_pixels=px.data_ptr() if floats else 0,
                                      d_rgb8=rgb.data_ptr(), d_counters=counters, stream=st.cuda_stream)
        cnt.zero_()
        launch(cnt.data_ptr())
        torch.cuda.synchronize()
        hits = int(cnt[1].item())
        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            launch()
        e1.record(st)
        torch.cuda.synchronize()
        out[tag] = e0.elapsed_time(e1) / n
        print(f"{name} {tag:10s} hits={hits:9d} mean_launch_ms={out[tag]:.5f}", flush=True)
    print(f"{name} away/orbit={out['away'] / out['orbit']:.3f} "
          f"float_store_ms={out['away'] - out['away_rgb8']:.5f}", flush=True)
    scene.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
