#!/usr/bin/env python3
"""Probe: successive frames on S HIP streams (round-robin), so frame k+1's kernel fills the tail of
frame k.  A single C3 frame is tail-bound (DESIGN.md "Where the time goes"): half of its
duration runs with a few long wavefronts resident.  Prints ms per frame for S = 1..4 and
checks every stream's last frame against the reference PPM hash.

    python tools/stream_overlap.py [config] [frames] [S list, e.g. 2,4]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from bench import import_package, load_golden, pinned_basis
    pkg = import_package()
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    cfg = pkg.configs.CONFIGS[name]
    meta = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    dev = torch.device("cuda", 0)
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    b12 = pinned_basis(meta, cfg, cam)[None, :]
    s3 = np.asarray(cfg["sun"], np.float32)[None, :]
    out = {"config": name, "frames": frames, "by_streams": {}}
    for S in [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3,4").split(",")]:
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
        px = [torch.empty(3 * W * H, dtype=torch.float32, device=dev) for _ in range(S)]
        rgb = [torch.empty(3 * W * H, dtype=torch.uint8, device=dev) for _ in range(S)]

        def run(n):
            for k in range(n):
                s = k % S
                scene.render_batch_device(b12, s3, W, H, d_pixels=px[s].data_ptr(), d_rgb8=rgb[s].data_ptr(),
                                          stream=streams[s].cuda_stream)
        run(4 * S)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(frames)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / frames
        ok = all(hashlib.sha256(pkg.ppm(W, H, r.cpu().numpy())).hexdigest() == meta["ppm_sha256"]["exact"] for r in rgb)
        out["by_streams"][S] = {"ms_per_frame": round(ms, 5), "mrays_s": round(meta["exact"]["rays"] / (ms * 1e3), 1),
                                "parity": ok}
        print(json.dumps({"S": S, **out["by_streams"][S]}), file=sys.stderr, flush=True)
    scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
