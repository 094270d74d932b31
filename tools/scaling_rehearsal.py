#!/usr/bin/env python3
"""Weak-scaling rehearsal on ONE MI355X: the per-rank work of bench.py at N = 1, 2, 4, 8 GPUs.

At N GPUs a bench step is F = N orbit frames, each frame's rows dealt in blocks of 8 over the
N ranks; rank r renders its rows of all F frames with one ceres_render_batch_device launch,
and rank 0 un-interleaves the gathered buffers with ceres_assemble_rgb8.  This tool runs,
on the one GPU it has, exactly the launch every rank would run (Tiling(8, r, N)) and the
rank-0 assembly, timed with HIP events on the launch stream.  The slowest rank's launch is
the predicted device time of a step; the RCCL gather is NOT modelled (one GPU has no xGMI
peer) -- it is pipelined behind the next step's render in bench.py (distributed.BatchGather).

    python tools/scaling_rehearsal.py [config] [reps] > gpurun_out/scaling_rehearsal.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import import_package, load_golden, pinned_basis
    pkg = import_package()
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    cfg = pkg.configs.CONFIGS[name]
    meta = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    mode = pkg.cfg_mode(cfg)
    axis, step_deg = pkg.configs.BENCH_ORBIT
    stream = torch.cuda.current_stream(dev)
    out = {"config": name, "W": W, "H": H, "reps": reps, "device": torch.cuda.get_device_name(0), "by_n": {}}
    base = None
    for N in (1, 2, 4, 8):
        F = N
        b12, s3 = pkg.orbit_cameras(cam, cfg["sun"], W, H, F, axis=axis, step_deg=step_deg, rotate_first=False)
        b12[0] = pinned_basis(meta, cfg, cam)
        s3[0] = np.asarray(cfg["sun"], np.float32)
        row_block = 8 if N > 1 else H
        per_rank = []
        rays = 0
        maxrows = max(pkg.local_rows(H, pkg.Tiling(row_block, r, N)) for r in range(N))
        px = torch.empty(F * 3 * W * maxrows, dtype=torch.float32, device=dev)
        rgb = torch.empty(F * 3 * W * maxrows, dtype=torch.uint8, device=dev)
        counters = torch.zeros(8, dtype=torch.int64, device=dev)
        for r in range(N):
            til = pkg.Tiling(row_block, r, N)
            counters.zero_()
            scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                      d_rgb8=rgb.data_ptr(), d_counters=counters.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            rays += int(counters[0].item())
            for _ in range(5):
                scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                          d_rgb8=rgb.data_ptr(), stream=stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                          d_rgb8=rgb.data_ptr(), stream=stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            per_rank.append(e0.elapsed_time(e1) / reps)
        asm_ms = 0.0
        if N > 1:
            recv = torch.zeros((N, F * maxrows, 3 * W), dtype=torch.uint8, device=dev)
            full = torch.empty((F, H, 3 * W), dtype=torch.uint8, device=dev)
            for _ in range(5):
                pkg.assemble_rgb8(recv.data_ptr(), recv[0].numel(), full.data_ptr(), F, W, H, row_block, N,
                                  stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                pkg.assemble_rgb8(recv.data_ptr(), recv[0].numel(), full.data_ptr(), F, W, H, row_block, N,
                                  stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            asm_ms = e0.elapsed_time(e1) / reps
        step_ms = max(per_rank)
        mrays = rays / (step_ms * 1e3)
        if base is None:
            base = mrays
        out["by_n"][N] = {"frames_per_step": F, "rays_per_step": rays, "rank_ms": [round(x, 5) for x in per_rank],
                          "slowest_rank_ms": round(step_ms, 5), "mean_rank_ms": round(float(np.mean(per_rank)), 5),
                          "assemble_ms_rank0": round(asm_ms, 5),
                          "gather_bytes_to_rank0": (N - 1) * F * maxrows * 3 * W,
                          "predicted_mrays_s_no_gather": round(mrays, 1),
                          "predicted_weak_efficiency": round(mrays / (N * base), 3)}
        print(json.dumps({"N": N, **out["by_n"][N]}), file=sys.stderr, flush=True)
    scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
