#!/usr/bin/env python3
"""Time the GPU OBJ loader (ceres_obj_parse_device) against the host loader (ceres_obj_load,
the reference's single-threaded std::istream-style parse) on the C5 heightfield written as OBJ
text (tools/probes/proc_obj), and check both against ceres_proc_mesh bit for bit.
Prints one JSON line.   python tools/obj_bench.py [--n 2237] [--reps 3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2237)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from conftest import import_package
    pkg = import_package()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "c5.obj")
        subprocess.run([os.path.join(REPO, "tools", "probes", "proc_obj"), str(args.n), path], check=True)
        text = open(path, "rb").read()
        ref = pkg.proc_mesh(args.n)
        t0 = time.perf_counter()
        host = pkg.load_obj(path)
        host_ms = (time.perf_counter() - t0) * 1e3
        dev = torch.device("cuda", 0)
        d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        times = []
        n = 0
        for k in range(args.reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            d_tri, d_norm, n = pkg.parse_obj_device(d_text.data_ptr(), len(text), stream)
            torch.cuda.synchronize(dev)
            if k:
                times.append((time.perf_counter() - t0) * 1e3)
            pkg.device_free(d_tri)
            pkg.device_free(d_norm)
        gpu_mesh = pkg.load_obj_gpu(path)
        ok = lambda a, b: np.array_equal(a.tri.view(np.uint32), b.tri.view(np.uint32)) and \
            np.array_equal(a.norm.view(np.uint32), b.norm.view(np.uint32))
        print(json.dumps({"n_tri": n, "text_bytes": len(text), "gpu_parse_ms_median": round(float(np.median(times)), 3),
                          "gpu_parse_ms": [round(t, 3) for t in times], "host_parse_ms": round(host_ms, 1),
                          "gpu_equals_proc_mesh": ok(gpu_mesh, ref), "host_equals_proc_mesh": ok(host, ref)}), flush=True)


if __name__ == "__main__":
    main()
