#!/usr/bin/env python3
"""Weak-scaling rehearsal on ONE MI355X: the per-rank work of bench.py at N = 1, 2, 4, 8 GPUs.

At N GPUs a bench step is F = k*N orbit frames (k = frames per GPU, bench.py's default 16), each frame's rows dealt in blocks of 8 over the
N ranks; rank r renders its rows of all F frames with one ceres_render_batch_device launch,
and rank 0 un-interleaves the gathered buffers with ceres_assemble_rgb8.  This tool runs,
on the one GPU it has, exactly the launch every rank would run (Tiling(8, r, N)) and the
rank-0 assembly, timed with HIP events on the launch stream.  The slowest rank's launch is
the predicted device time of a step, serialised (tail-bound) and in the bench's regime
(launches rotated over 8 streams, wall time per launch).  One GPU has no xGMI peer, so the RCCL
all-to-all itself cannot run; its on-device cost is EMULATED in a third regime: after each
pipelined launch, a copy of the rank's receive volume (bench.py's FrameExchange: (N-1)/N of its k
frames' RGB8 rows, the bytes RCCL's copy kernels move into this GPU's HBM, read from the render's
output) plus the un-interleave of its k frames (ceres_assemble_rgb8_packed) run on a separate
"collective" stream, as in bench.py -- so the predicted efficiency pays the exchange's HBM
traffic and CU time.  The link time is budgeted separately: 1/N of the rank's k frames from each
peer over its own xGMI link at XGMI_GBS per link and direction (default 76.8 GB/s: 153.6 GB/s
bidirectional).

Round 4 adds the collective-free partition bench.py uses by default (--collect frames): rank q
renders its k frames of the step (batch frames q*k .. q*k+k-1 of exchange_order = orbit frames q,
q+N, ...) whole, one launch per step, pipelined over the 8 streams -- nothing to exchange, so its
predicted efficiency is the slowest rank's render against N = 1.  Arithmetic: CERES_ARITH=fma
(default, bench.py's) or exact.

    python tools/scaling_rehearsal.py [config] [reps] [frames per GPU] [row block] > gpurun_out/scaling_rehearsal.json
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
XGMI_GBS = float(os.environ.get("XGMI_GBS", "76.8"))     # per link and direction
XSKIP = os.environ.get("XSKIP", "")


def main():
    import torch
    from bench import import_package, load_golden, step_views
    pkg = import_package()
    if os.environ.get("CERES_LIB"):                               # A/B: another build of the library
        pkg.LIB_PATH = os.path.abspath(os.environ["CERES_LIB"])
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    rb = int(sys.argv[4]) if len(sys.argv) > 4 else 16           # bench.py --row-block (round 6: 16)
    cfg = pkg.configs.CONFIGS[name]
    meta = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    build = "ref" if os.environ.get("CERES_ARITH", "fma") == "fma" else "exact"
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    scene = pkg.Scene(mesh, bvh, device=0)
    mode = pkg.cfg_mode(cfg, arith)
    stream = torch.cuda.current_stream(dev)
    S = 8
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    out = {"config": name, "W": W, "H": H, "reps": reps, "frames_per_gpu": k, "arith": build,
           "device": torch.cuda.get_device_name(0), "by_n": {}}
    base = None
    import ceres_raytracer_amd.distributed as D
    for N in (1, 2, 4, 8):
        F = k * N
        b12, s3 = step_views(pkg, cfg, meta, cam, F, k, build=build)      # the same arc at every N, as bench.py
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
        piped_x = []
        # exchange emulation: per step, the receive volume of one rank ((N-1)/N of k frames) copied on a
        # collective stream out of the render's output, then the assembly of its k frames
        recv_bytes = (N - 1) * k * H * 3 * W // N
        # XPRIO=1: the collective stream at high priority (measured: C3 at N = 8 0.759 -> 0.711, the
        # exchange's copies then displace more of the render; default off)
        coll = torch.cuda.Stream(device=dev, priority=-1 if os.environ.get("XPRIO", "0") == "1" else 0)
        xrecv = [torch.empty(max(recv_bytes, 1), dtype=torch.uint8, device=dev) for _ in range(2)]
        xfull = torch.empty((k, H, 3 * W), dtype=torch.uint8, device=dev)
        xpack = torch.zeros((k * H, 3 * W), dtype=torch.uint8, device=dev)
        copied = [None] * S
        counters = [torch.zeros(8, dtype=torch.int64, device=dev) for _ in range((F + 63) // 64)]

        def launch(til, d_px, d_rgb, st, with_counters=False):
            # as bench.py: one ceres_render_batch_device launch per (at most) 64 frames of the step
            fb = 3 * W * max(pkg.local_rows(H, til), 1)
            for c, f0 in enumerate(range(0, F, 64)):
                f1 = min(F, f0 + 64)
                scene.render_batch_device(b12[f0:f1], s3[f0:f1], W, H, mode=mode, tiling=til, d_pixels=d_px + 4 * fb * f0,
                                          d_rgb8=d_rgb + fb * f0,
                                          d_counters=counters[c].data_ptr() if with_counters else 0, stream=st)

        for r in range(N):
            til = pkg.Tiling(row_block, r, N)
            launch(til, px.data_ptr(), rgb.data_ptr(), stream.cuda_stream, with_counters=True)
            torch.cuda.synchronize(dev)
            rank_rays.append(sum(int(c[0].item()) for c in counters))
            rays += rank_rays[-1]
            for _ in range(5):
                launch(til, px.data_ptr(), rgb.data_ptr(), stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                launch(til, px.data_ptr(), rgb.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            per_rank.append(e0.elapsed_time(e1) / reps)
            for it in range(2):                          # warm, then timed
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for q in range(reps * S // 2):
                    launch(til, spx[q % S].data_ptr(), srgb[q % S].data_ptr(), streams[q % S].cuda_stream)
                torch.cuda.synchronize(dev)
            piped.append((time.perf_counter() - t0) * 1e3 / (reps * S // 2))
            if N > 1:
                for it in range(2):                      # warm, then timed
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for q in range(reps * S // 2):
                        st = streams[q % S]
                        if copied[q % S] is not None:
                            st.wait_event(copied[q % S])  # the slot's rows were read by the exchange
                        launch(til, spx[q % S].data_ptr(), srgb[q % S].data_ptr(), st.cuda_stream)
                        done = torch.cuda.Event()
                        done.record(st)
                        coll.wait_event(done)
                        with torch.cuda.stream(coll):
                            if XSKIP != "copy":             # diagnosis: XSKIP=copy|asm drops one part
                                xrecv[q % 2].copy_(srgb[q % S][:recv_bytes])
                            if XSKIP != "asm":
                                pkg.assemble_rgb8_packed(xpack.data_ptr(), xfull.data_ptr(), k, W, H, row_block, N,
                                                         coll.cuda_stream)
                            ev = torch.cuda.Event()
                            ev.record(coll)
                        copied[q % S] = ev
                    torch.cuda.synchronize(dev)
                piped_x.append((time.perf_counter() - t0) * 1e3 / (reps * S // 2))
        # --collect frames: rank q's k frames whole (exchange_order batch frames q*k ..), pipelined
        order = D.exchange_order(F, N)
        ob12, os3 = b12[order], s3[order]
        whole = pkg.Tiling(H, 0, 1)
        fpx = [torch.empty(k * 3 * W * H, dtype=torch.float32, device=dev) for _ in range(S)]
        frgb = [torch.empty(k * 3 * W * H, dtype=torch.uint8, device=dev) for _ in range(S)]
        piped_f = []
        for r in range(N):
            rb12, rs3 = ob12[r * k:(r + 1) * k], os3[r * k:(r + 1) * k]
            for it in range(2):                          # warm, then timed
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for q in range(reps * S // 2):
                    for f0 in range(0, k, 64):
                        f1 = min(k, f0 + 64)
                        scene.render_batch_device(rb12[f0:f1], rs3[f0:f1], W, H, mode=mode, tiling=whole,
                                                  d_pixels=fpx[q % S].data_ptr() + 4 * 3 * W * H * f0,
                                                  d_rgb8=frgb[q % S].data_ptr() + 3 * W * H * f0,
                                                  stream=streams[q % S].cuda_stream)
                torch.cuda.synchronize(dev)
            piped_f.append((time.perf_counter() - t0) * 1e3 / (reps * S // 2))
        del fpx, frgb
        # --collect bands: rank r renders band (r + f) mod N of every frame f (ceres_tiling.bands: one
        # launch per <= 64 frames, the band rotating from frame to frame inside the kernel) and the
        # exchange lands every received band in place in its owner's frame (RCCL point-to-point into
        # the PPM body slice; distributed.FrameBands): no un-interleave.  Emulated like the exchange
        # above: the receive volume copied on the collective stream after each step, no assembly.
        # (Round 6 first tried one launch per band, N per step: 0.807 render-only, 0.73 with the
        # exchange for C3 at N = 8 -- the small launches' tails.)
        piped_b, piped_bx = [], []
        if N > 1:
            bh = D.band_height(H, N)
            bb = [torch.empty(F * 3 * W * bh, dtype=torch.uint8, device=dev) for _ in range(S)]
            bp = [torch.empty(F * 3 * W * bh, dtype=torch.float32, device=dev) for _ in range(S)]
            xband = torch.empty(max(recv_bytes, 1), dtype=torch.uint8, device=dev)
            bcopied = [None] * S
            fbb = 3 * W * bh
            for r in range(N):
                def band_step(q, st):
                    for f0 in range(0, F, 64):
                        f1 = min(F, f0 + 64)
                        scene.render_batch_device(b12[f0:f1], s3[f0:f1], W, H, mode=mode,
                                                  tiling=pkg.Tiling(bh, (r + f0) % N, N, 1),
                                                  d_pixels=bp[q % S].data_ptr() + 4 * fbb * f0,
                                                  d_rgb8=bb[q % S].data_ptr() + fbb * f0, stream=st.cuda_stream)

                for exch, sink in ((False, piped_b), (True, piped_bx)):
                    for it in range(2):                  # warm, then timed
                        torch.cuda.synchronize(dev)
                        t0 = time.perf_counter()
                        for q in range(reps * S // 2):
                            st = streams[q % S]
                            if exch and bcopied[q % S] is not None:
                                st.wait_event(bcopied[q % S])
                            band_step(q, st)
                            if exch:
                                done = torch.cuda.Event()
                                done.record(st)
                                coll.wait_event(done)
                                with torch.cuda.stream(coll):
                                    xband.copy_(bb[q % S][:recv_bytes])
                                    ev = torch.cuda.Event()
                                    ev.record(coll)
                                bcopied[q % S] = ev
                        torch.cuda.synchronize(dev)
                    sink.append((time.perf_counter() - t0) * 1e3 / (reps * S // 2))
            del bb, bp, xband
        pipe_f_ms = max(piped_f)
        mrays_f = rays / (pipe_f_ms * 1e3)
        if N == 1:
            base_f = mrays_f
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
        pipe_x_ms = max(piped_x) if piped_x else pipe_ms
        mrays_x = rays / (pipe_x_ms * 1e3)
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
                          "predicted_weak_efficiency_pipelined": round(mrays_p / (N * base_p), 3),
                          "exchange_recv_bytes_per_rank_step": recv_bytes,
                          "xgmi_link_ms_per_step": round(k * H * 3 * W / N / (XGMI_GBS * 1e6), 4),
                          "pipelined_with_exchange_rank_ms": [round(x, 5) for x in piped_x],
                          "predicted_mrays_s_pipelined_with_exchange": round(mrays_x, 1),
                          "predicted_weak_efficiency_pipelined_with_exchange": round(mrays_x / (N * base_p), 3),
                          "frames_partition_rank_ms": [round(x, 5) for x in piped_f],
                          "predicted_mrays_s_frames_partition": round(mrays_f, 1),
                          "predicted_weak_efficiency_frames_partition": round(mrays_f / (N * base_f), 3)}
        if piped_b:
            out["by_n"][N].update({
                "bands_rank_ms": [round(x, 5) for x in piped_b],
                "predicted_weak_efficiency_bands": round(rays / (max(piped_b) * 1e3) / (N * base_p), 3),
                "bands_with_exchange_rank_ms": [round(x, 5) for x in piped_bx],
                "predicted_weak_efficiency_bands_with_exchange": round(rays / (max(piped_bx) * 1e3) / (N * base_p), 3)})
        print(json.dumps({"N": N, **out["by_n"][N]}), file=sys.stderr, flush=True)
    scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
