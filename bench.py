#!/usr/bin/env python3
"""bench.py -- Mrays/s of the CERES hot path on MI355X (BASELINE.json metric).

Workload (default): C3 = dragon.obj 1920x1080, primary + shadow rays, static.cpp camera
(static.cpp:38-47,72-73) -- the configuration BASELINE.json's metric is quoted on.

A step renders F frames (F = --frames, default = 16 per GPU): views of the anim.cpp:76-88 orbit
of the C3 camera + sun about z, frame f rotated once by f x 360 / F degrees (frame 0 = C3
exactly).  At N = 1 a step is sixteen C3-size frames 22.5 degrees apart; at N GPUs it is 16N
distinct frames over the same turn, 22.5/N degrees apart (pkg.bench_views) -- WEAK scaling,
sixteen frames' work per GPU from the same orbit at every N (one batch launch per 64 frames).
Every one of those views has its reference PPM sha256 and rays/hits in
tests/golden/orbit/<config>.json (made by the reference's own render(), make_golden.py --orbit),
and every frame the validation step assembles is checked against it.
At N > 1 (--collect, default auto):
  frames    the frames are the units: rank q renders orbit frames q, q + N, q + 2N, ... (16 of the
            16N) whole, with one ceres_render_batch_device launch, into its own HBM -- no
            collective, nothing on the xGMI links (frames are independent: render.hpp:104-153);
  exchange  every frame's rows are interleaved over the ranks in blocks of --row-block rows; each
            rank renders its rows of all F frames, then ONE RCCL all-to-all per step gathers each
            frame to its owner rank (rank q owns the same 16 frames as above) and
            ceres_assemble_rgb8_packed un-interleaves them -- the tiled framebuffer of BASELINE's
            C4 ("framebuffer tiled across 8x MI355X with RCCL gather");
  gather    rows interleaved, all F frames to rank 0.
  auto = exchange for configs defined as a tiled framebuffer (configs.py "tiled": C4) except at
  N = 2, where the exchange would put 16 frames' worth of rows on one xGMI link per step and
  outlast the render (DESIGN.md "Multi-GPU"); frames otherwise.
RGB8 + float framebuffers in HBM.  Steps rotate over --streams HIP streams (own buffers each):
the collective/assembly of step k and the tail of its render overlap later steps; the timed
region ends when every step's frames are assembled.
Scene upload, OBJ load and BVH build are outside the timed region, as in the reference
(static.cpp:129-133).  value = (primary + shadow rays of all F frames) x steps / wall time
(max over ranks).  One process per GPU (torch.distributed, backend nccl = RCCL).

Arithmetic (--arith): "fma" (default) = the reference as its own CMake build compiles it
(CMakeLists.txt:11-13, g++ -O3 -mavx2 -mfma: GCC contracts a*b+c into FMA; the scene, camera,
orbit and kernels use CERES_ARITH_FMA / CERES_MODE_FMA) -- the same build the CPU baseline times
(oracle/_ref/ref_render) -- so every frame is checked against THAT build's PPM; "exact" = the
contraction-free reference (-ffp-contract=off), checked against its PPMs.

Also reported (rank 0):
  roofline      the dominant kernel AS THE STEP RUNS IT: one ceres_render_batch_device launch of 16
                of the step's orbit views (whole frames), launched back to back on ONE stream
                between two HIP events (mean launch duration = per-kernel evidence, comparable
                with a single-stream rocprofv3 trace).  achieved = the launch's ALGORITHMIC bytes
                (pinned reference statistics per view, tests/golden/orbit/<cfg>.json, SURVEY.md
                §8(d): 64 B per node-pair visit + 56 B per triangle test) / that duration.  `bound`
                is chosen from the measured counters (profiles/pmc_summary.json, rocprofv3 --pmc of
                the same launch): "hbm" when the DRAM bytes are at least half the algorithmic
                bytes, else "l2" (served on-die; priced against the ~34.5 TB/s aggregate L2);
                `limiter` names what the counters say stalls the kernel; `hbm_frac_algorithmic`
                keeps SURVEY §8(d)'s algorithmic-bytes-vs-8-TB/s figure.
  roofline_step the timed regime itself: algorithmic bytes of every frame of a step (all ranks)
                / ms_per_step, per GPU, priced against the L2 and against HBM (steps overlap on
                --streams streams, so this is a throughput, not a launch duration).
  roofline_solo one whole frame of frame 0's view per launch (the latency regime), as `roofline`.
  c3_only       the same timed loop with all F frames = the C3 view itself (the orbit mix is
                lighter: fewer shadow rays per frame), value + shadow-ray fractions of both.
  cpu_baseline  the REFERENCE hot path (oracle/_ref/ref_render, reference CMake flags) timed
                on this host's cores on a bounded sample of the same workload (N = 1 only);
                falls back to the oracle restatement if the reference binary is absent.
  parity        sha256 of frame 0's PPM vs the reference fixture, rays/hits vs the fixture, and
                every assembled frame of the step vs the reference orbit fixtures.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "ceres-raytracer_amd")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md §L2: aggregate over the 8 XCD L2s, ~34.5 TB/s


def import_package():
    import importlib.util
    if "ceres_raytracer_amd" in sys.modules:
        return sys.modules["ceres_raytracer_amd"]
    spec = importlib.util.spec_from_file_location("ceres_raytracer_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ceres_raytracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_golden(name):
    p = os.path.join(REPO, "tests", "golden", name + ".json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def pinned_basis(meta, cfg, cam, build="exact"):
    """C3 camera basis from the fixture's hex bits (never trust a host libm for parity); build =
    "ref" (the reference CMake build's basis, FMA arithmetic) or "exact"."""
    if meta is None:
        return cam.basis(cfg["W"], cfg["H"])
    b = meta["ref_basis"] if build == "ref" else meta["basis"]
    bits = [int(h, 16) for h in b["dir"] + b["u"] + b["v"]]
    return np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])


def view_entry(e, build):
    """A view of an orbit fixture in one build: the contraction-free entry or its "ref" part."""
    if e is None:
        return None
    return e.get("ref") if build == "ref" else e


def algorithmic_bytes(stats):
    """64 B per node-pair visit + 56 B per triangle test (48-B Triangle + 8-B
    primitive index), from the reference's own Statistics (single_ray_traverser.hpp:132-135)."""
    return 64 * (stats["primary_pairs"] + stats.get("shadow_pairs", 0)) + \
        56 * (stats["primary_tests"] + stats.get("shadow_tests", 0))


def step_views(pkg, cfg, meta, cam, F, V=None, build="exact"):
    """Cameras (basis12 [F,12], sun3 [F,3]) of one bench step of F frames (pkg.bench_views: frame f
    rotated once by f x 360 / F degrees about z, frame 0 = C3 with the fixture's basis bits).
    `V` is accepted for older tools and ignored."""
    b12, s3, _ = pkg.bench_views(cam, cfg["sun"], cfg["W"], cfg["H"], F, basis0=pinned_basis(meta, cfg, cam, build))
    return b12, s3


def load_orbit_fixture(name):
    """tests/golden/orbit/<name>.json: reference sha256 / rays / hits per orbit view, keyed by the
    float32 step's hex bits (tests/golden/make_golden.py --orbit), or None."""
    p = os.path.join(REPO, "tests", "golden", "orbit", name + ".json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)["by_step_bits"]


def step_key(step):
    return "%08x" % int(np.asarray(step, np.float32).view(np.uint32))


def cpu_baseline(cfg_name, cfg, rays_per_frame, budget_s=3.0, build="ref"):
    """Reference CPU path on this host, bounded sample of the same workload (rank 0, N = 1)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import configs
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    # the reference binary of the same arithmetic as the GPU run (the CMake-flag build by default)
    ref = os.path.join(REPO, "oracle", "_ref", "ref_render" if build == "ref" else "ref_render_exact")
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    if os.access(ref, os.X_OK):
        try:
            args = [ref] + configs.cli_args(cfg)
            probe = json.loads(subprocess.run(args + ["--reps", "2"], capture_output=True, text=True, check=True,
                                              env=env, timeout=300).stdout.strip().splitlines()[-1])
            reps = int(max(3, min(200, budget_s * 1e3 / max(probe["render_ms_best"], 1e-3))))
            out = json.loads(subprocess.run(args + ["--reps", str(reps)], capture_output=True, text=True, check=True,
                                            env=env, timeout=600).stdout.strip().splitlines()[-1])
            ms = out["render_ms_median"]
            return {"value": round(out["rays"] / (ms * 1e3), 3), "unit": "Mrays/s", "cores": threads,
                    "kind": "reference",
                    "sample": f"{cfg_name}: {reps} full frames of reference render() (render.hpp:87, "
                              f"-O3 -mavx2 -mfma -fopenmp{'' if build == 'ref' else ' -ffp-contract=off'}), "
                              f"median {ms:.2f} ms/frame, {out['rays']} rays/frame",
                    "cpu_model": _cpu_model()}
        except Exception as e:  # noqa: BLE001 -- fall through to the port
            sys.stderr.write(f"reference CPU baseline failed ({e}); timing the oracle port\n")
    import oracle
    sc = oracle.prepare(cfg, contract=build == "ref")
    oracle.render(sc, cfg, want_pixels=True, want_ppm=False, threads=threads)
    times = []
    t_end = time.time() + budget_s
    while time.time() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        oracle.render(sc, cfg, want_pixels=True, want_ppm=False, threads=threads)
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {"value": round(rays_per_frame / (ms * 1e3), 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{cfg_name}: {len(times)} full frames of oracle/liboracle.so, median {ms:.2f} ms/frame",
            "cpu_model": _cpu_model()}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_entry(cfg_name, kernel):
    """rocprofv3 --pmc summary of `kernel`'s solo launch for a config (profiles/pmc_summary.json,
    tools/pmc_summary.py), or None."""
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get(cfg_name, {}).get(kernel)
    except Exception:  # noqa: BLE001
        return None


def roofline_block(name, nbytes, ms, pmc, scene_bytes):
    """The roofline object for the dominant kernel (one launch = one frame).

    achieved = ALGORITHMIC bytes per launch / the launch's mean duration.  The
    bound is picked from the measured counters: DRAM bytes (FETCH_SIZE x2 + WRITE_SIZE, the gfx950
    correction) per launch >= half the algorithmic bytes -> "hbm" (8 TB/s); otherwise the bytes
    are served on-die and the ceiling they are priced against is the aggregate L2 (~34.5 TB/s,
    MI355X_MICROARCH.md §L2) -- an upper bound on L2 use, since L1 / scalar-cache hits count
    too.  `limiter` reads the counters: wave cycles parked on s_waitcnt, TA busy, and whether the
    L2 fabric reads exceed the scene (the scene streams from MALL/DRAM) or not."""
    achieved = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    traffic = None if pmc is None else pmc.get("hbm_bytes_per_launch")
    dram_gbs = traffic / (ms * 1e-3) / 1e9 if traffic and ms > 0 else None
    bound = "hbm" if traffic and traffic >= 0.5 * nbytes else "l2"
    peak = HBM_PEAK_GBS if bound == "hbm" else L2_PEAK_GBS
    out = {"bound": bound, "kernel": name, "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
           "frac": round(achieved / peak, 4), "traffic": traffic,
           "algorithmic_bytes_per_launch": nbytes, "mean_launch_ms": round(ms, 5),
           "hbm_frac_algorithmic": round(achieved / HBM_PEAK_GBS, 4),
           "dram_gbs": None if dram_gbs is None else round(dram_gbs, 1),
           "dram_frac": None if dram_gbs is None else round(dram_gbs / HBM_PEAK_GBS, 4),
           "scene_device_bytes": scene_bytes}
    if pmc is None:
        out["limiter"] = "unmeasured (no rocprofv3 --pmc summary for this config)"
        return out
    wait = pmc.get("waitcnt_parked_frac")
    ta = pmc.get("ta_busy_frac")
    rd = pmc.get("hbm_read_bytes_per_launch")
    out.update({k: pmc.get(k) for k in ("waitcnt_parked_frac", "issue_stall_frac", "ta_busy_frac", "td_busy_frac",
                                        "l2_hit_rate", "valu_lane_utilisation", "hbm_read_bytes_per_launch",
                                        "hbm_write_bytes_per_launch") if pmc.get(k) is not None})
    out["pmc_source"] = "profiles/pmc_summary.json (rocprofv3 --pmc, solo launches of this config)"
    hit = pmc.get("l2_hit_rate")
    if bound == "hbm" and dram_gbs and dram_gbs >= 0.5 * HBM_PEAK_GBS:
        lim = "HBM bandwidth"
    else:
        # the counters say latency or issue, not bandwidth (dram_frac, frac << 1); where the L2 misses
        # are served follows from the scene's size against the 8 x 4 MiB L2s and the 256-MiB MALL
        where = ("DRAM (scene larger than the 256-MiB Infinity Cache)" if scene_bytes and scene_bytes > 256 << 20
                 else "MALL (scene larger than the L2s)" if scene_bytes and scene_bytes > 32 << 20
                 else "MALL (scene L2-resident; misses are each XCD's first touches)")
        kind = "dependent-load latency" if wait is not None and wait >= 0.45 else \
            "vector-memory issue + dependent-load latency" if ta is not None and ta >= 0.5 else \
            "dependent-load latency and issue"
        lim = f"{kind}: waves parked on s_waitcnt {wait:.2f} of cycles" if wait is not None else kind
        if ta is not None:
            lim += f", TA busy {ta:.2f}"
        if hit is not None:
            lim += f"; L2 hit {hit:.2f}, misses to {where}"
        if rd:
            lim += f", fabric reads {rd / 1e6:.0f} MB/launch"
    out["limiter"] = lim
    return out


def roofline_step_block(nbytes, ms_step, world):
    """The timed regime priced at the roofline: the algorithmic bytes of every frame of a step (all
    ranks) / ms_per_step, per GPU, against the aggregate L2 (~34.5 TB/s) and against HBM (8 TB/s).
    Steps overlap on several streams, so this is a sustained throughput, not a launch duration."""
    if not nbytes or ms_step <= 0:
        return None
    job = nbytes / (ms_step * 1e-3) / 1e9
    per_gpu = job / world
    return {"algorithmic_bytes_per_step": int(nbytes), "ms_per_step": round(ms_step, 5), "unit": "GB/s",
            "achieved_job": round(job, 1), "achieved_per_gpu": round(per_gpu, 1),
            "frac_l2": round(per_gpu / L2_PEAK_GBS, 4), "frac_hbm": round(per_gpu / HBM_PEAK_GBS, 4),
            "source": "per-view reference Statistics, tests/golden/orbit/<config>.json (64 B/node pair + 56 B/test)"}


def choose_collect(requested, cfg, world, frames):
    """The N > 1 partition of a step (DESIGN.md "Multi-GPU"): "auto" = "exchange" (rows dealt over
    the ranks, one RCCL all-to-all) for a config defined as ONE framebuffer tiled over the GPUs
    (configs.py "tiled": C4, C5) except at N = 2, where one xGMI link would carry every split frame's
    rows; "frames" (each rank renders its frames whole, no collective) otherwise.  Partitions that
    deal whole frames need F to be a multiple of N, else every frame goes to rank 0 ("gather")."""
    collect = requested
    if collect == "auto":
        collect = "exchange" if cfg.get("tiled") and world != 2 else "frames"
    if collect in ("frames", "exchange") and frames % world:
        collect = "gather"
    return collect


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="dragon_1080")
    ap.add_argument("--frames", type=int, default=0,
                    help="orbit frames per step (default: --frames-per-gpu x number of GPUs)")
    ap.add_argument("--frames-per-gpu", type=int, default=16,
                    help="frames of work per GPU per step when --frames is not given (weak scaling)")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-view0-only", action="store_true",
                    help="skip the second timed loop with every frame = frame 0's view (C3 itself)")
    ap.add_argument("--no-float", action="store_true", help="skip the float framebuffer (RGB8 only)")
    ap.add_argument("--collect", choices=("auto", "frames", "exchange", "gather"), default="auto",
                    help="N > 1: frames = unsplit frames, each rank renders its F/N frames whole (no collective); "
                         "exchange = every frame's rows dealt over the ranks, each frame gathered to one owner rank "
                         "in one all-to-all; gather = rows dealt, all frames to rank 0; auto = exchange for "
                         "configs defined as a tiled framebuffer (C4) except at N = 2, where one link would carry "
                         "it (DESIGN.md \"Multi-GPU\"), else frames")
    ap.add_argument("--prime-s", type=float, default=0.3,
                    help="untimed setup: seconds of steps before the W warmup steps (GPU clock ramp)")
    ap.add_argument("--streams", type=int, default=8,
                    help="HIP streams the steps rotate over (step k on stream k %% S, its own buffers): step k+1 "
                         "fills the tail of step k")
    ap.add_argument("--arith", choices=("fma", "exact"), default="fma",
                    help="fma: the reference's CMake build (GCC FMA contraction); exact: -ffp-contract=off")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    pkg = import_package()
    import ceres_raytracer_amd.distributed as D
    cfg = pkg.configs.CONFIGS[args.config]
    meta = load_golden(args.config)
    orbit_fx = load_orbit_fixture(args.config)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.stderr.write("bench.py --gpus N>1 must be launched with torch.distributed.run (one rank per GPU)\n")
            return 2
    # CERES_BENCH_SHARE_GPU=1 (rehearsal on a box with fewer GPUs than ranks): rank -> device
    # local_rank mod device count
    dev_id = local_rank % torch.cuda.device_count() if os.environ.get("CERES_BENCH_SHARE_GPU") else local_rank
    torch.cuda.set_device(dev_id)
    dev = torch.device("cuda", dev_id)
    local_rank = dev_id
    if world > 1:
        backend = os.environ.get("CERES_BENCH_BACKEND", "nccl")      # gloo: shared-GPU rehearsal only
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    W, H = cfg["W"], cfg["H"]
    F = args.frames or args.frames_per_gpu * world
    build = "ref" if args.arith == "fma" else "exact"          # the fixtures' key for this arithmetic
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    scene = pkg.Scene(mesh, bvh, device=local_rank)
    # F views of the orbit, frame f rotated once by f x 360 / F degrees (frame 0 = C3, fixture bits)
    b12, s3, steps_deg = pkg.bench_views(cam, cfg["sun"], W, H, F, basis0=pinned_basis(meta, cfg, cam, build))
    view0_step = bool(cfg.get("bench_view0"))
    if view0_step:
        # C5: the orbit about z through the origin leaves the [0,1]^2 heightfield for views 40..96 of
        # 128 (no triangle in view), which would flatter the step; its step is F copies of the
        # config's own view instead (each checked against the reference's PPM of that view)
        b12, s3, steps_deg = np.repeat(b12[:1], F, 0), np.repeat(s3[:1], F, 0), np.repeat(steps_deg[:1], F)
    collect = choose_collect(args.collect, cfg, world, F)
    owner = world > 1 and collect == "frames"              # unsplit frames: no collective
    exchange = world > 1 and collect in ("exchange", "frames")
    if exchange:
        # batch order for the all-to-all: rank q owns batch frames q*k .. q*k+k-1, which are orbit
        # frames q, q + N, q + 2N, ... (batch frame 0 = orbit frame 0 = C3)
        order = D.exchange_order(F, world)
        b12, s3, steps_deg = b12[order], s3[order], steps_deg[order]
    mode = pkg.cfg_mode(cfg, arith)
    full_mode = (mode & 0xf) == pkg.MODE_FULL
    row_block = args.row_block if world > 1 and not owner else H
    tiling = pkg.Tiling(row_block, rank, world) if not owner else pkg.Tiling(H, 0, 1)
    S = max(1, args.streams)
    job_steps = steps_deg                        # the whole job's views, in batch order
    Fl = F                                       # frames this rank's launches render
    if owner:        # rank q renders batch frames q*k .. q*k+k-1 whole
        gather = D.FrameOwner(W, H, rank, world, frames=F, device=dev, slots=max(2, S))
        mine_f = gather.owned_frames()
        Fl = len(mine_f)
        b12_all, s3_all = b12, s3
        b12, s3, steps_deg = b12[mine_f], s3[mine_f], steps_deg[mine_f]
    elif exchange:   # each frame to one owner rank: a rank's ingress is (N-1)/N of its k frames per step
        gather = D.FrameExchange(W, H, row_block, rank, world, frames=F, device=dev, slots=max(2, S))
    else:            # every frame -> rank 0
        gather = D.BatchGather(W, H, row_block, rank, world, frames=F, device=dev, slots=max(2, S))
    rows = gather.local_rows
    d_px = [None if args.no_float else torch.empty(Fl * 3 * W * max(rows, 1), dtype=torch.float32, device=dev)
            for _ in range(S)]
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    # steps rotate over S streams, each with its own framebuffers / gather slot: a step's frames
    # are complete when its stream is, and step k+1's kernel fills the tail of step k (a single
    # frame ends with a few long wavefronts resident, DESIGN.md "Where the time goes")
    streams = [stream] if S == 1 else [torch.cuda.Stream(device=dev) for _ in range(S)]
    slots = max(2, S)
    pending = [False] * slots

    MAXF = 64                                    # frames per ceres_render_batch_device launch (kMaxFrames)
    chunk_counters = [torch.zeros(8, dtype=torch.int64, device=dev) for _ in range((Fl + MAXF - 1) // MAXF)]
    views = {"b12": b12, "s3": s3, "steps": steps_deg,       # what this rank renders every step
             "job": job_steps}                               # ... and the whole step's views (batch order)

    def render(slot, st, with_counters=False):
        # one launch per (at most) 64 frames of the step; frame f's rows at f * 3 * W * rows
        px = d_px[slot % S]
        fb = 3 * W * max(rows, 1)
        vb, vs = views["b12"], views["s3"]
        for c, f0 in enumerate(range(0, Fl, MAXF)):
            f1 = min(Fl, f0 + MAXF)
            scene.render_batch_device(vb[f0:f1], vs[f0:f1], W, H, mode=mode, tiling=tiling,
                                      d_pixels=0 if px is None else px.data_ptr() + 4 * fb * f0,
                                      d_rgb8=gather.local_ptr(slot) + fb * f0,
                                      d_counters=chunk_counters[c].data_ptr() if with_counters else 0,
                                      stream=st.cuda_stream)
        if with_counters:
            with torch.cuda.stream(st):
                cs = torch.stack(chunk_counters)
                counters.copy_(torch.cat([cs[:, :6].sum(0), cs[:, 6:7].max(0).values, cs[:, 7:].sum(0)]))

    def step(k):
        slot = k % slots
        st = streams[k % S]
        with torch.cuda.stream(st):
            if pending[slot]:                  # the previous use of this slot (step k - slots)
                gather.finish(slot)
                pending[slot] = False
            render(slot, st)
            gather.start(slot)
            pending[slot] = True
            if S == 1:                         # one stream: complete the previous step's gather now
                prev = (k - 1) % slots
                if pending[prev] and prev != slot:
                    gather.finish(prev)
                    pending[prev] = False

    def drain():
        for k_ in range(slots):
            if pending[k_]:
                with torch.cuda.stream(streams[k_ % S]):
                    gather.finish(k_)
                pending[k_] = False
        gather.wait_assembled()

    def validate():
        """Untimed: one counted step of the current views.  Returns (rays, hits, checks) where checks
        compares every frame this rank assembled with the REFERENCE's PPM of the same view
        (tests/golden/orbit/<config>.json; sha256 of "P6 W H 255\n" + body, static.cpp:135-147)
        and the step's rays / hits with the reference's per-view counts (render.hpp:155)."""
        render(0, stream, with_counters=True)
        gather.start(0)
        full = gather.finish(0)
        gather.wait_assembled()
        torch.cuda.synchronize(dev)
        c = counters.clone()
        if world > 1:
            dist.all_reduce(c)
        c = c.cpu().numpy()
        if c[6]:
            # ceres_finalize's error word: a traversal stack overflowed (single_ray_traverser.hpp:29
            # asserts instead), so some frame of the batch is wrong -- never time a wrong render
            raise SystemExit(f"bench.py: traversal stack overflow in the validation batch (error word {int(c[6]):#x})")
        mine = (list(zip(gather.owned_frames(), full)) if exchange
                else ([(f, full[f]) for f in range(F)] if rank == 0 else []))
        head = b"P6 %d %d 255\n" % (W, H)
        n = [0, 0, 0]                                            # [checked, matched, unpinned]
        for f, body in mine:
            e = None if orbit_fx is None else view_entry(orbit_fx.get(step_key(views["job"][f])), build)
            if e is None:
                n[2] += 1
                continue
            n[0] += 1
            n[1] += int(hashlib.sha256(head + body.cpu().numpy().tobytes()).hexdigest() == e["sha256"])
        stat = torch.tensor(n, dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(stat)
        stat = stat.cpu().numpy()
        keys = [None if orbit_fx is None else view_entry(orbit_fx.get(step_key(x)), build) for x in views["job"]]
        ref_rays = sum(e["rays"] for e in keys) if all(keys) else None
        ref_hits = sum(e["hits"] for e in keys) if all(keys) else None
        checks = {"frames": F, "frames_checked": int(stat[0]), "frames_unpinned": int(stat[2]),
                  "all_frames_match_reference": bool(stat[2] == 0 and stat[1] == stat[0] == F),
                  "step_rays_match_reference": None if ref_rays is None else int(c[0]) == ref_rays,
                  "step_hits_match_reference": None if ref_hits is None else int(c[1]) == ref_hits}
        return int(c[0]), int(c[1]), checks

    def timed(prime):
        """W warmup steps (after >= --prime-s of untimed steps when `prime`), then exactly K steps
        between barrier + device synchronise; returns the max-over-ranks wall time."""
        if prime:
            # untimed setup before the W warmup steps: steps over every stream and collective slot
            # for at least --prime-s seconds, so no stream's first launch lands in the timed region
            # when W < S and the GPU has left its idle clock state (measured: K = 20 after W = 5
            # from a cold start ran 6 % below the same K after W = 200; after this priming they agree)
            t_prime = time.perf_counter()
            for k in range(slots):
                step(k)
            drain()
            torch.cuda.synchronize(dev)
            per_step = max((time.perf_counter() - t_prime) / slots, 1e-5)
            # the same number of steps on every rank (each step is a collective)
            more = torch.tensor([min(20000, max(0, int(args.prime_s / per_step) - slots))], dtype=torch.int64,
                                device=dev)
            if world > 1:
                dist.all_reduce(more, op=dist.ReduceOp.MAX)
            for k in range(int(more.item())):
                step(slots + k)
            drain()
            torch.cuda.synchronize(dev)
        for k in range(args.warmup):
            step(k)
        drain()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(k)
        drain()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        return float(elapsed.item())

    def step_bytes(steps):
        """Algorithmic bytes of one step's frames (whole job), from every view's pinned reference
        statistics, or None when a view is unpinned."""
        if orbit_fx is None:
            return None
        es = [view_entry(orbit_fx.get(step_key(x)), build) for x in steps]
        if not all(e is not None and "stats" in e for e in es):
            return None
        return int(sum(algorithmic_bytes(e["stats"]) for e in es))

    # validation step of the orbit views (not timed): exact counts + every frame vs the reference
    rays_step, hits_step, orbit_checks = validate()
    parity = None
    if rank == 0 and meta is not None:
        parity = {}
        # frame 0's ray / hit counts (render.hpp:155) from a counted whole-frame render
        c0 = torch.zeros(8, dtype=torch.int64, device=dev)
        rgb0 = torch.empty(3 * W * H, dtype=torch.uint8, device=dev)
        scene.render_device(b12[0], s3[0], W, H, mode=mode, tiling=pkg.Tiling(H, 0, 1), d_rgb8=rgb0.data_ptr(),
                            d_counters=c0.data_ptr(), stream=sh)
        torch.cuda.synchronize(dev)
        c0 = c0.cpu().numpy()
        body = b"P6 %d %d 255\n" % (W, H) + rgb0.view(H, 3 * W).cpu().numpy().tobytes()
        parity.update(reference_build="reference CMake flags (-O3 -mavx2 -mfma, GCC FMA contraction)" if build == "ref"
                      else "reference with -ffp-contract=off",
                      frame0_ppm_sha256_matches_reference=hashlib.sha256(body).hexdigest() == meta["ppm_sha256"][build],
                      rays_match=int(c0[0]) == meta[build]["rays"], hits_match=int(c0[1]) == meta[build]["hits"])
    if parity is not None:
        parity.update(orbit_checks)

    T = timed(prime=True)
    value = rays_step * args.steps / T / 1e6
    bytes_step = step_bytes(views["job"])
    primary_step = F * W * H
    view0 = None
    if not args.no_view0_only and not view0_step:
        # the same loop with every frame = frame 0's view (C3 itself for dragon_1080): the orbit mix
        # has fewer shadow rays per frame than C3, so report both
        v0b, v0s, v0d = (b12_all[:1], s3_all[:1], job_steps[:1]) if owner else (b12[:1], s3[:1], steps_deg[:1])
        views.update(b12=np.repeat(v0b, Fl, 0), s3=np.repeat(v0s, Fl, 0), steps=np.repeat(v0d, Fl),
                     job=np.repeat(v0d, F))
        rays0, hits0, checks0 = validate()
        T0 = timed(prime=False)
        b0 = step_bytes(views["job"])
        view0 = {"value": round(rays0 * args.steps / T0 / 1e6, 3), "unit": "Mrays/s",
                 "roofline_step": roofline_step_block(b0, T0 / args.steps * 1e3, world),
                 "ms_per_step": round(T0 / args.steps * 1e3, 5), "rays_per_step": rays0, "hits_per_step": hits0,
                 "shadow_ray_frac": round((rays0 - primary_step) / rays0, 4) if full_mode else 0.0,
                 "parity": checks0}

    roofline = roofline_solo = None
    cpu = None
    if rank == 0 and not args.no_roofline and meta is not None:
        # the step's kernel: one 16-frame launch of the step's first 16 orbit views (whole frames),
        # n_b launches back to back on ONE stream between two HIP events -- no other stream's work
        # overlaps, so the mean is a per-launch duration (and agrees with a single-stream trace)
        nb_f = min(16, F)
        vb12, vs3, vsteps = b12[np.argsort(steps_deg)][:nb_f], s3[np.argsort(steps_deg)][:nb_f], \
            np.sort(steps_deg)[:nb_f]
        bat_rgb = torch.empty(nb_f * 3 * W * H, dtype=torch.uint8, device=dev)
        bat_px = None if args.no_float else torch.empty(nb_f * 3 * W * H, dtype=torch.float32, device=dev)
        whole = pkg.Tiling(H, 0, 1)

        def batch_launch():
            scene.render_batch_device(vb12, vs3, W, H, mode=mode, tiling=whole,
                                      d_pixels=0 if bat_px is None else bat_px.data_ptr(), d_rgb8=bat_rgb.data_ptr(),
                                      stream=sh)
        for _ in range(3):
            batch_launch()
        n_b = max(10, min(args.steps, 100))
        evb0, evb1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        evb0.record(stream)
        for _ in range(n_b):
            batch_launch()
        evb1.record(stream)
        torch.cuda.synchronize(dev)
        batch_ms = evb0.elapsed_time(evb1) / n_b
        bb = step_bytes(vsteps)
        kname = "ceres_fused" if full_mode else "ceres_primary"
        if bb is not None:
            roofline = roofline_block(kname, bb, batch_ms,
                                      pmc_entry(args.config, f"{kname}_batch{nb_f}_{args.arith}"),
                                      scene.info()["device_bytes"])
            roofline.update(launch=f"ceres_render_batch_device, {nb_f} orbit views (steps {vsteps[0]:g}..{vsteps[-1]:g} "
                                   f"deg), whole {W}x{H} frames, {n_b} launches back to back on one stream",
                            frames_per_launch=nb_f)
        # dominant kernel, timed live with HIP events on the launch stream (one full frame, this GPU)
        solo = pkg.Tiling(H, 0, 1)
        solo_rgb = torch.empty(3 * W * H, dtype=torch.uint8, device=dev)
        solo_px = torch.empty(3 * W * H, dtype=torch.float32, device=dev)
        n_t = max(10, min(args.steps, 200))
        for _ in range(3):                            # the solo frame's tile order, warm
            scene.render_device(b12[0], s3[0], W, H, mode=mode, tiling=solo, d_pixels=solo_px.data_ptr(),
                                d_rgb8=solo_rgb.data_ptr(), stream=sh)
        # n_t back-to-back launches between two HIP events on their stream: mean launch duration
        # (per-launch event pairs would add each launch's dispatch latency, ~13 us here)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(n_t):
            scene.render_device(b12[0], s3[0], W, H, mode=mode, tiling=solo, d_pixels=solo_px.data_ptr(),
                                d_rgb8=solo_rgb.data_ptr(), stream=sh)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        mean_ms = ev0.elapsed_time(ev1) / n_t
        ex = meta[build]
        b_p = 64 * ex["primary_pairs"] + 56 * ex["primary_tests"]
        b_s = 64 * ex["shadow_pairs"] + 56 * ex["shadow_tests"]
        # one kernel per frame: ceres_fused (primary + shadow + shading) or ceres_primary (primary only)
        name, nbytes = ("ceres_fused", b_p + b_s) if full_mode else ("ceres_primary", b_p)
        pmc = pmc_entry(args.config, f"{name}_solo_{args.arith}") or \
            (pmc_entry(args.config, name) if args.arith == "exact" else None)
        roofline_solo = roofline_block(name, nbytes, mean_ms, pmc, scene.info()["device_bytes"])
        if roofline is None:
            roofline = roofline_solo
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, cfg, rays_step if F == 1 else meta[build]["rays"], build=build)

    if rank == 0:
        line = {
            "metric": "Mrays/sec (primary+shadow) on dragon.obj 1920x1080; 1/2/4/8-GPU scaling"
            if args.config == "dragon_1080" else f"Mrays/sec ({args.config})",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(T / args.steps * 1e3, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "arith": args.arith,
            "data": ("real mesh from the reference repo (data/%s)" % cfg["obj"] if cfg["obj"] else
                     "procedural %dx%d-vertex heightfield generated in-process (SURVEY.md §8(d) C5 definition)"
                     % (cfg["proc"], cfg["proc"]))
                    + ("; every frame = the config camera" if view0_step else
                       "; frame 0 = the config camera, frames 1.. = the anim.cpp-style orbit about z"),
            "config": {"workload": f"{args.config}: {cfg['obj'] or 'proc'} {W}x{H} "
                                   f"{'primary+shadow' if full_mode else 'primary only'}, "
                                   + (f"{F} copies of the config view per step" if view0_step
                                      else f"{F} orbit frame(s) per step"),
                       "W": W, "H": H, "frames_per_step": F, "rays_per_step": rays_step, "hits_per_step": hits_step,
                       "shadow_ray_frac": round((rays_step - primary_step) / rays_step, 4)
                       if full_mode else 0.0,
                       "row_block": row_block,
                       "parallelism": (f"unsplit frames x{world}: rank q renders orbit frames q, q+{world}, ... whole, "
                                       "no collective" if owner else
                                       f"row-interleaved frames x{world}"
                                       + ((" + one RCCL all-to-all per step: frame f gathered to rank f (pipelined)"
                                           if exchange else " + one RCCL gather per step to rank 0 (pipelined)")
                                          if world > 1 else "")),
                       "collect": collect if world > 1 else None,
                       "float_framebuffer": d_px[0] is not None, "streams": S},
            # the step's one collective against the xGMI budget (DESIGN.md "Multi-GPU"): bytes one rank
            # receives per step, 1/N of them from each peer over that peer's direct link (one link per
            # peer in a fully connected 8-GPU node) at 76.8 GB/s per link and direction
            "collective": None if world == 1 or owner else {
                "kind": "all_to_all" if exchange else "gather",
                "recv_bytes_per_rank_step": (world - 1) * (F // world if exchange else F) * H * 3 * W // world,
                "xgmi_link_ms_est": round((F // world if exchange else F) * H * 3 * W / world / 76.8e6, 4),
                "ms_per_step": round(T / args.steps * 1e3, 5)},
            "roofline": roofline, "roofline_step": roofline_step_block(bytes_step, T / args.steps * 1e3, world),
            "roofline_solo": roofline_solo, "cpu_baseline": cpu, "parity": parity,
        }
        if view0 is not None:
            line["c3_only_value" if args.config == "dragon_1080" else "view0_only_value"] = view0["value"]
            line["view0_only"] = view0
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
