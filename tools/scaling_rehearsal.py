#!/usr/bin/env python3
"""Weak-scaling rehearsal on ONE MI355X: the per-rank work of bench.py at N = 1, 2, 4, 8 GPUs.

At N GPUs a bench step is F = k*N orbit frames (k = frames per GPU, bench.py's default 8), each frame's rows dealt in blocks of 8 over the
N ranks; rank r renders its rows of all F frames with one ceres_render_batch_device launch,
and rank 0 un-interleaves the gathered buffers with ceres_assemble_rgb8.  This tool runs,
on the one GPU it has, exactly the launch every rank would run (Tiling(8, r, N)) and the
rank-0 assembly, timed with HIP events on the launch stream.  The slowest rank's launch is
the predicted device time of a step, serialised (tail-bound) and in the bench's regime
(launches rotated over 8 streams, wall time per launch); the RCCL collective is NOT modelled (one GPU has no xGMI
peer) -- it is pipelined behind the next step's render in bench.py (distributed.BatchGather).

    python tools/scaling_rehearsal.py [config] [reps] [frames per GPU] [row block] > gpurun_out/scaling_rehearsal.json
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import import_package, load_golden, step_views
    pkg = import_package()
    if os.environ.get("CERES_LIB"):                               # A/B: another build of the library
        pkg.LIB_PATH = os.path.abspath(os.environ["CERES_LIB"])
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rb = int(sys.argv[4]) if len(sys.argv) > 4 else 8            # bench.py --row-block
    cfg = pkg.configs.CONFIGS[name]
    meta = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    mode = pkg.cfg_mode(cfg)
    stream = torch.cuda.current_stream(dev)
    S = 8
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    out = {"config": name, "W": W, "H": H, "reps": reps, "frames_per_gpu": k, "device": torch.cuda.get_device_name(0), "by_n": {}}
    base = None
    for N in (1, 2, 4, 8):
        F = k * N
        b12, s3 = step_views(pkg, cfg, meta, cam, F, k)      # the same arc at every N, as bench.py
        row_block = rb if N > 1 else H
        per_rank = []
        rank_rays = []
        rays = 0
        maxrows = max(pkg.local_rows(H, pkg.Tiling(row_block, r, N)) for r in range(N))
        px = torch.empty(F * 3 * W * maxrows, dtype=torch.float32, device=dev)
        rgb = torch.empty(F * 3 * W * maxrows, dtype=torch.uint8, device=dev)
        # the bench's regime: steps rotated over S streams, each with its own framebuffers
        spx = [torch.empty(F * 3 * W * maxrows, dtype=torch.float32, device=dev) for _ in range(S)]
        srgb = [torch.empty(F * 3 * W * maxrows, dtype=torch.uint8, device=dev) for _ in range(S)]
        piped = []
        counters = torch.zeros(8, dtype=torch.int64, device=dev)
        for r in range(N):
            til = pkg.Tiling(row_block, r, N)
            counters.zero_()
            scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(),
                                      d_rgb8=rgb.data_ptr(), d_counters=counters.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            rank_rays.append(int(counters[0].item()))
            rays += rank_rays[-1]
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
            for it in range(2):                          # warm, then timed
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for q in range(reps * S // 2):
                    scene.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=spx[q % S].data_ptr(),
                                              d_rgb8=srgb[q % S].data_ptr(), stream=streams[q % S].cuda_stream)
                torch.cuda.synchronize(dev)
            piped.append((time.perf_counter() - t0) * 1e3 / (reps * S // 2))
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
        pipe_ms = max(piped)
        mrays_p = rays / (pipe_ms * 1e3)
        if base is None:
            base, base_p = mrays, mrays_p
        del spx, srgb
        out["by_n"][N] = {"frames_per_step": F, "rays_per_step": rays, "rank_rays": rank_rays, "row_block": row_block, "rank_ms": [round(x, 5) for x in per_rank],
                          "slowest_rank_ms": round(step_ms, 5), "mean_rank_ms": round(float(np.mean(per_rank)), 5),
                          "assemble_ms_rank0": round(asm_ms, 5),
                          "gather_bytes_to_rank0": (N - 1) * F * maxrows * 3 * W,
                          "predicted_mrays_s_no_gather": round(mrays, 1),
                          "predicted_weak_efficiency": round(mrays / (N * base), 3),
                          "pipelined_rank_ms": [round(x, 5) for x in piped], "pipelined_streams": S,
                          "predicted_mrays_s_pipelined": round(mrays_p, 1),
                          "predicted_weak_efficiency_pipelined": round(mrays_p / (N * base_p), 3)}
        print(json.dumps({"N": N, **out["by_n"][N]}), file=sys.stderr, flush=True)
    scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
