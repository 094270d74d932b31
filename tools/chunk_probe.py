#!/usr/bin/env python3
"""Probe: does splitting one C3 frame into C interleaved row chunks on C HIP streams (each
chunk a primary+shadow launch pair, overlapping the other chunks' tails) beat one launch pair?
Uses C independent scenes (own shard counters / job queues) and the ceres_tiling row split."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    import torch
    pkg = import_package()
    name = "dragon_1080"
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    sun = np.asarray(cfg["sun"], np.float32)
    scenes = [pkg.Scene(mesh, bvh) for _ in range(8)]
    rgb = torch.empty(3 * W * H, dtype=torch.uint8, device="cuda")
    px = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(7)]
    res = {}
    for rb in (16, 8):
        for C in (1, 2, 3, 4, 6, 8):
            for nstreams in sorted({1, C}):
                tilings = [pkg.Tiling(rb if C > 1 else H, c, C) for c in range(C)]
                offs = [0]
                for t in tilings:
                    offs.append(offs[-1] + pkg.local_rows(H, t))

                def frame():
                    main = streams[0]
                    ev = torch.cuda.Event()
                    ev.record(main)
                    for c in range(C):
                        s = streams[c % nstreams]
                        if s is not main:
                            s.wait_event(ev)
                        scenes[c].render_device(basis, sun, W, H, tiling=tilings[c],
                                                d_pixels=px.data_ptr() + 12 * W * offs[c],
                                                d_rgb8=rgb.data_ptr() + 3 * W * offs[c], stream=s.cuda_stream)
                    for c in range(1, min(C, nstreams)):
                        e2 = torch.cuda.Event()
                        e2.record(streams[c])
                        main.wait_event(e2)
                for _ in range(10):
                    frame()
                torch.cuda.synchronize()
                ts = []
                for rep in range(5):
                    t0 = time.perf_counter()
                    for _ in range(50):
                        frame()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) / 50 * 1e3)
                res[f"rb{rb}_C{C}_s{nstreams}"] = round(min(ts), 4)
                print(f"row_block {rb} chunks {C} streams {nstreams}: {min(ts):.4f} ms/frame (median {np.median(ts):.4f})",
                      flush=True)


if __name__ == "__main__":
    main()
