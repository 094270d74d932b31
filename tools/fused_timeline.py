#!/usr/bin/env python3
"""Diagnostic: per-wavefront timeline of the fused frame kernel (stats scene, s_memrealtime at
100 MHz): when each 8x8 tile's wave starts and ends, how long its primary phase (closest-hit,
the longest lane chain) and its work-stealing shadow phase take, and what the slowest waves
are made of.  usage: python tools/fused_timeline.py [config]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_package, load_golden  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon_1080"
    pkg = import_package()
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, _ = pkg.prepare(cfg)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    sc = pkg.Scene(mesh, bvh, stats=True)
    for _ in range(3):
        _, _, st = sc.render(basis, cfg["sun"], W, H, want_pixels=False)
    log = sc.wave_log(1 << 20).astype(np.int64)
    sc.close()
    log = log[log[:, 2] > 0]
    t0 = log[:, 0].min()
    us = lambda a: a / 100.0  # noqa: E731  (100-MHz ticks -> us)
    start, mid, end = us(log[:, 0] - t0), us(log[:, 1] - t0), us(log[:, 2] - t0)
    prim, shad, life = mid - start, end - mid, end - start
    chain, iters, hits, ppairs, spairs = log[:, 3], log[:, 4], log[:, 5], log[:, 6], log[:, 7]
    q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 99, 100)]  # noqa: E731
    out = {"config": name, "waves": int(log.shape[0]), "span_us": round(float(end.max()), 2),
           "stats_render_ms": round(st["ms"], 4),
           "start_us_pct": q(start), "end_us_pct": q(end), "life_us_pct": q(life),
           "primary_us_pct": q(prim), "shadow_us_pct": q(shad),
           "max_chain_pct": q(chain), "shadow_iters_pct": q(iters),
           "us_per_primary_step_pct": q(prim[chain > 0] / chain[chain > 0]),
           "us_per_shadow_iter_pct": q(shad[iters > 0] / iters[iters > 0]),
           "waves_ending_after_half_span": int((end > 0.5 * end.max()).sum()),
           "waves_with_shadow": int((hits > 0).sum()),
           # lane efficiency: node-pair visits / (64 x the wave's loop trips) per phase, and how
           # the summed wave-time splits between the phases
           "primary_lane_eff": round(float(ppairs.sum() / max(1, 64 * chain.sum())), 3),
           "shadow_lane_eff": round(float(spairs.sum() / max(1, 64 * iters.sum())), 3),
           "wave_us_primary_sum": round(float(prim.sum()), 1), "wave_us_shadow_sum": round(float(shad.sum()), 1),
           "wave_us_primary_sum_chain_gt1": round(float(prim[chain > 1].sum()), 1),
           "primary_steps_sum": int(chain.sum()), "shadow_iters_sum": int(iters.sum())}
    # waves resident over time (10 samples across the span) and the peak
    ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    out["resident_waves_peak"] = int(conc.max())
    out["resident_waves_at"] = {f"{f:.1f}": int(conc[np.searchsorted(ev[:, 0], f * end.max(), side="right") - 1])
                                for f in np.linspace(0.05, 0.95, 10)}
    out["mean_resident_waves"] = round(float(life.sum() / end.max()), 1)
    top = np.argsort(-end)[:12]
    out["last_to_finish"] = [{"start": round(float(start[i]), 1), "primary": round(float(prim[i]), 1),
                              "shadow": round(float(shad[i]), 1), "chain": int(chain[i]), "shadow_iters": int(iters[i]),
                              "hits": int(hits[i]), "primary_pairs": int(ppairs[i]), "shadow_pairs": int(spairs[i])}
                             for i in top]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
