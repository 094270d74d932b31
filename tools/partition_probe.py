#!/usr/bin/env python3
"""Batching gain or penalty of a view set: one ceres_render_batch_device launch of F frames vs
the same frames as F/4 launches of 4 (HIP events on the launch stream, serialised), for sets of
distinct orbit views and of near-copies of four views.  Found: near-copies of the same views in
one launch run slower (DESIGN.md "Multi-GPU"), so bench.step_views uses distinct views.
    python tools/partition_probe.py [config] [unused] [reps] > out.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import import_package, load_golden, step_views
    pkg = import_package()
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    cfg = pkg.configs.CONFIGS[name]
    meta = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    mode = pkg.cfg_mode(cfg)
    stream = torch.cuda.current_stream(dev)
    px = torch.empty(4 * N * 3 * W * H, dtype=torch.float32, device=dev)
    rgb = torch.empty(4 * N * 3 * W * H, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)

    def timed(b12, s3, til):
        counters.zero_()
        scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(), d_rgb8=rgb.data_ptr(),
                                  d_counters=counters.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        rays = int(counters[0].item())
        for _ in range(3):
            scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                      d_rgb8=rgb.data_ptr(), stream=stream.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                      d_rgb8=rgb.data_ptr(), stream=stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps, rays

    axis, step_deg = pkg.configs.BENCH_ORBIT

    def views_at(angles):
        b = np.zeros((len(angles), 12), np.float32)
        s3 = np.zeros((len(angles), 3), np.float32)
        for q, a in enumerate(angles):
            bb, ss = pkg.orbit_cameras(cam, cfg["sun"], W, H, 2, axis=axis, step_deg=float(a), rotate_first=False)
            b[q], s3[q] = bb[1], ss[1]
        return b, s3

    out = {"config": name, "reps": reps, "sets": []}
    # one launch of F frames vs the same frames as F/4 launches of 4: the batching gain (< 1) or
    # penalty (> 1) of a view set
    sets = {"4x45": [45 * q for q in range(4)],
            "8x45 (0..315)": [45 * q for q in range(8)],
            "8x22.5 (0..157.5)": [22.5 * q for q in range(8)],
            "8 = 4x45 twice, +0.5": [45 * (q % 4) + 0.5 * (q // 4) for q in range(8)],
            "8 = 4x45 twice, +5": [45 * (q % 4) + 5 * (q // 4) for q in range(8)],
            "8 = 4x45 twice, +11.25": [45 * (q % 4) + 11.25 * (q // 4) for q in range(8)],
            "16x11.25 (0..168.75)": [11.25 * q for q in range(16)],
            "32x5.625 (0..174.4)": [5.625 * q for q in range(32)],
            "32x11.25 (0..348.75)": [11.25 * q for q in range(32)],
            "32 = 4x45 x8, +0.5": [45 * (q % 4) + 0.5 * (q // 4) for q in range(32)]}
    for label, angles in sets.items():
        b, s3 = views_at(angles)
        ms, rays = timed(b, s3, pkg.Tiling(H, 0, 1))
        parts = [timed(b[q:q + 4].copy(), s3[q:q + 4].copy(), pkg.Tiling(H, 0, 1))[0] for q in range(0, len(angles), 4)]
        out["sets"].append({"views": label, "frames": len(angles), "ms": round(ms, 5), "rays": rays,
                            "ms_as_4frame_launches": round(sum(parts), 5), "ratio": round(ms / sum(parts), 4)})
        print(json.dumps(out["sets"][-1]), file=sys.stderr, flush=True)
    scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
