#!/usr/bin/env python3
"""bench.py -- Mrays/s of the CERES hot path on MI355X (BASELINE.json metric).

Workload (default): C3 = dragon.obj 1920x1080, primary + shadow rays, static.cpp camera
(static.cpp:38-47,72-73) -- the configuration BASELINE.json's metric is quoted on.

A step renders F frames (F = --frames, default = 16 per GPU).  --views config (default): every
frame is the config's own view -- for dragon_1080 the C3 camera + sun with the fixture's pinned
basis bits, so `value` is C3 itself.  --views orbit: frame f is the anim.cpp:76-88 orbit of that
camera + sun about z, rotated once by f x 360 / F degrees (pkg.bench_views); reported beside the
headline as `orbit_value` (a lighter mix on dragon: fewer shadow rays per frame).  WEAK scaling:
sixteen frames' work per GPU at every N (one batch launch per 64 frames).  Every view has its
reference PPM sha256 and rays/hits in tests/golden/orbit/<config>.json (made by the reference's
own render(), make_golden.py --orbit), and every frame the validation step assembles is checked
against it.
At N > 1 (--collect, default auto):
  exchange  the framebuffer partition BASELINE.json's north star names: every frame's rows are
            interleaved over the ranks in blocks of --row-block rows; each rank renders its rows of
            all F frames, then ONE RCCL all-to-all per step gathers each frame to its owner rank
            (rank q owns 16 frames) and ceres_assemble_rgb8_packed un-interleaves them;
  frames    rank q renders frames q, q + N, q + 2N, ... (16 of the 16N) whole, with one
            ceres_render_batch_device launch, into its own HBM -- no collective (frames are
            independent: render.hpp:104-153);
  gather    rows interleaved, all F frames to rank 0.
  auto = frames (the step's frames are independent units: no data-path collective), except for
  the configs BASELINE.json defines as one framebuffer tiled across the GPUs (C4, C5) at N >= 4:
  exchange (at N = 2 the single xGMI link would carry 16 split frames' rows per step and outlast
  the render, DESIGN.md "Multi-GPU").  The other partition of the same step is timed too and
  reported as `partition_alt`; the line carries the world size and backend RCCL ran with.
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
                of the step's views (whole frames; 16 copies of C3 by default), launched back to back on ONE stream
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
  orbit         the same timed loop over the orbit views (`orbit_value`), value + shadow-ray fraction.
  partition_alt N > 1: the same step under the other partition (frames <-> bands).
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
N_CU = 256                     # MI355X_MICROARCH.md chip table
CLOCK_GHZ = 2.4                # max clock (chip table); the issue ceilings below use it, so they are upper bounds
VALU_PER_CU_CYCLE = 2.0        # 4 SIMD-32 per CU, a wave64 VALU instruction every 2 cycles per SIMD (MI355X_MICROARCH.md:54)
SALU_PER_CU_CYCLE = 1.0        # one scalar unit per CU shared by its 4 SIMDs
L2_REQ_BYTES = 128             # one TCC request = at most one 128-B L2 line (an upper bound on its bytes)


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
    hc = host_cpus()
    # every core this process may use: the affinity mask, capped by the cgroup quota and by
    # OMP_NUM_THREADS (the GPU lease's CPU share: 16 on the one-GPU box) when those are set
    threads = hc["affinity_cpus"] or os.cpu_count()
    if hc["cgroup_cpu_quota"]:
        threads = min(threads, max(1, int(hc["cgroup_cpu_quota"])))
    if hc["omp_num_threads"]:
        threads = min(threads, int(hc["omp_num_threads"]))
    note = (f"{threads} threads = the CPUs this process may use (affinity {hc['affinity_cpus']}, cgroup quota "
            f"{hc['cgroup_cpu_quota']}, OMP_NUM_THREADS {hc['omp_num_threads']}); the node exposes "
            f"{hc['node_cpus']} CPUs, the rest belong to the other GPUs' leases")
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
                    "cpu_model": _cpu_model(), "host": hc, "cores_note": note}
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
            "cpu_model": _cpu_model(), "host": hc, "cores_note": note}


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


def l1_peak():
    """The vector-L1 (TCP) ceiling in cache accesses per CU-cycle, calibrated on this chip with
    tools/probes/l1_peak.hip under rocprofv3 --pmc (profiles/r06/l1_probe/l1_peak.json: the most
    TCP_TOTAL_CACHE_ACCESSES per CU-cycle any of its load shapes sustained), or None."""
    p = os.path.join(REPO, "profiles", "r06", "l1_probe", "l1_peak.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get("tcp_accesses_per_cu_cycle_peak")


def measured_ceilings(pmc, ms, launches=1.0):
    """Every ceiling the kernel's own counters price (round 6): the counts of
    `launches` launches (rocprofv3 --pmc of that launch, per dispatch) over `ms` of wall time.
      valu_issue   SQ_INSTS_VALU / (256 CUs x 2 wave-instructions per CU-cycle x 2.4 GHz)
      salu_issue   SQ_INSTS_SALU / (256 x 1 x 2.4 GHz)
      vmem_ta      TA busy cycles / TA cycles (measured in the profiled run itself)
      vmem_td      TD busy cycles / TD cycles
      l1           TCP_TOTAL_CACHE_ACCESSES / (256 x the probe's accesses per CU-cycle x 2.4 GHz)
      l2           TCC_REQ x 128 B / 34.5 TB/s (128 B per request: an upper bound on its bytes)
      hbm          DRAM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction) / 8 TB/s
    Returns {name: {achieved, peak, unit, frac}} (only the ceilings the summary has counters for)."""
    if not pmc or ms <= 0:
        return {}
    c = pmc.get("counters_mean_per_dispatch", {})
    sec = ms * 1e-3
    cyc = N_CU * CLOCK_GHZ * 1e9 * sec                      # CU-cycles in the window at max clock
    out = {}

    def put(k, achieved, peak, unit, note):
        out[k] = {"achieved": round(achieved, 3), "peak": round(peak, 3), "unit": unit,
                  "frac": round(achieved / peak, 4) if peak else None, "what": note}
    if c.get("SQ_INSTS_VALU"):
        put("valu_issue", launches * c["SQ_INSTS_VALU"] / sec / 1e9, N_CU * VALU_PER_CU_CYCLE * CLOCK_GHZ,
            "G wave-instr/s", "VALU wave-instructions vs 2 per CU-cycle at 2.4 GHz")
    if c.get("SQ_INSTS_SALU"):
        put("salu_issue", launches * c["SQ_INSTS_SALU"] / sec / 1e9, N_CU * SALU_PER_CU_CYCLE * CLOCK_GHZ,
            "G wave-instr/s", "SALU wave-instructions vs 1 per CU-cycle at 2.4 GHz")
    if pmc.get("ta_busy_frac") is not None:
        put("vmem_ta", pmc["ta_busy_frac"], 1.0, "busy fraction", "texture addresser (vector-memory issue) busy cycles")
    if pmc.get("td_busy_frac") is not None:
        put("vmem_td", pmc["td_busy_frac"], 1.0, "busy fraction", "texture data (vector-memory return) busy cycles")
    peak_l1 = l1_peak()
    if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") and peak_l1:
        put("l1", launches * c["TCP_TOTAL_CACHE_ACCESSES_sum"] / sec / 1e9, N_CU * peak_l1 * CLOCK_GHZ,
            "G accesses/s", "vector-L1 (TCP) cache accesses vs the l1_peak probe's rate per CU-cycle")
    if c.get("TCC_REQ_sum"):
        put("l2", launches * c["TCC_REQ_sum"] * L2_REQ_BYTES / sec / 1e9, L2_PEAK_GBS, "GB/s",
            "L2 (TCC) requests x 128 B vs the aggregate L2 bandwidth")
    if pmc.get("hbm_bytes_per_launch"):
        put("hbm", launches * pmc["hbm_bytes_per_launch"] / sec / 1e9, HBM_PEAK_GBS, "GB/s",
            "DRAM bytes (FETCH_SIZE x 2 + WRITE_SIZE) vs 8 TB/s")
    del cyc
    return out


def traffic_levels(pmc, launches=1.0):
    """The measured traffic per level of the memory hierarchy, per launch: vector-L1 accesses,
    L1 -> L2 read requests, L2 requests, DRAM bytes (rocprofv3 --pmc of the same launch)."""
    if not pmc:
        return None
    c = pmc.get("counters_mean_per_dispatch", {})
    g = lambda k: None if c.get(k) is None else int(round(launches * c[k]))   # noqa: E731
    return {"tcp_accesses": g("TCP_TOTAL_CACHE_ACCESSES_sum"), "tcp_to_tcc_reads": g("TCP_TCC_READ_REQ_sum"),
            "tcc_requests": g("TCC_REQ_sum"), "tcc_hit_rate": pmc.get("l2_hit_rate"),
            "l1_hit_rate": None if not c.get("TCP_TOTAL_CACHE_ACCESSES_sum") or c.get("TCP_TCC_READ_REQ_sum") is None
            else round(1 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"], 4),
            "dram_read_bytes": None if pmc.get("hbm_read_bytes_per_launch") is None
            else int(launches * pmc["hbm_read_bytes_per_launch"]),
            "dram_write_bytes": None if pmc.get("hbm_write_bytes_per_launch") is None
            else int(launches * pmc["hbm_write_bytes_per_launch"]),
            "valu_instructions": g("SQ_INSTS_VALU"), "salu_instructions": g("SQ_INSTS_SALU"),
            "vmem_read_instructions": g("SQ_INSTS_VMEM_RD"), "smem_instructions": g("SQ_INSTS_SMEM")}


def roofline_block(name, nbytes, ms, pmc, scene_bytes, counted=None, launches=1.0):
    """The roofline object of the dominant kernel (round 6: priced against the kernel's own
    measured ceilings).

    `bound` is the NEAREST measured ceiling -- the one with the largest achieved / peak among
    measured_ceilings(): VALU and SALU issue, the vector-memory path (TA / TD busy), the vector
    L1, the L2 and HBM -- so `frac` <= 1 by construction.  The reference's algorithmic bytes
    (64 B per node-pair visit + 56 B per triangle test, Statistics of
    single_ray_traverser.hpp:132-135) stay as the side block `algorithmic`; `build_bytes` is what
    the build's own fetch sites moved (the counting build, bench.counted_bytes); `traffic_levels`
    the measured bytes / requests per level.  Without counters: the bound is "unmeasured"."""
    achieved_alg = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    traffic = None if pmc is None else pmc.get("hbm_bytes_per_launch")
    ceil = measured_ceilings(pmc, ms, launches)
    out = {"kernel": name, "mean_launch_ms": round(ms, 5), "traffic": traffic, "scene_device_bytes": scene_bytes,
           "algorithmic_bytes_per_launch": nbytes,
           "algorithmic": {"bytes_per_launch": nbytes, "achieved_gbs": round(achieved_alg, 1),
                           "frac_l2": round(achieved_alg / L2_PEAK_GBS, 4),
                           "frac_hbm": round(achieved_alg / HBM_PEAK_GBS, 4),
                           "source": "reference Statistics per view (64 B / node pair + 56 B / triangle test); "
                                     "not what this build fetches (see build_bytes), not a ceiling"},
           "hbm_frac_algorithmic": round(achieved_alg / HBM_PEAK_GBS, 4)}
    if counted:
        cb = dict(counted)
        cb["achieved_gbs"] = round(cb["total"] / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
        out["build_bytes"] = cb
    if not ceil:
        out.update({"bound": "unmeasured", "achieved": round(achieved_alg, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                    "frac": None, "limiter": "unmeasured (no rocprofv3 --pmc summary for this launch)"})
        return out
    bname, b = max(ceil.items(), key=lambda kv: kv[1]["frac"] or 0.0)
    out.update({"bound": bname, "achieved": b["achieved"], "peak": b["peak"], "unit": b["unit"], "frac": b["frac"],
                "ceilings": ceil, "traffic_levels": traffic_levels(pmc, launches)})
    out.update({k: pmc.get(k) for k in ("waitcnt_parked_frac", "issue_stall_frac", "active_inst_frac",
                                        "l2_hit_rate", "valu_lane_utilisation") if pmc.get(k) is not None})
    out["pmc_source"] = "profiles/pmc_summary.json (rocprofv3 --pmc of this launch, per dispatch)"
    out["limiter"] = limiter_text(ceil, pmc, scene_bytes)
    return out


def limiter_text(ceil, pmc, scene_bytes):
    """What the counters say bounds the launch, in numbers: each ceiling's fraction, nearest first,
    then where the waves' cycles went."""
    parts = [f"{k} {v['frac']:.2f}" for k, v in sorted(ceil.items(), key=lambda kv: -(kv[1]["frac"] or 0))]
    wait, stall, act = pmc.get("waitcnt_parked_frac"), pmc.get("issue_stall_frac"), pmc.get("active_inst_frac")
    txt = "ceilings (frac of peak): " + ", ".join(parts)
    if wait is not None:
        txt += (f"; wave-cycles: parked on s_waitcnt {wait:.2f}, issue-stalled {stall:.2f}, issuing {act:.2f}"
                if stall is not None and act is not None else f"; waves parked on s_waitcnt {wait:.2f}")
    top = max(v["frac"] or 0 for v in ceil.values())
    if top < 0.7:
        where = ("DRAM (scene larger than the 256-MiB Infinity Cache)" if scene_bytes and scene_bytes > 256 << 20
                 else "MALL (scene larger than the L2s)" if scene_bytes and scene_bytes > 32 << 20
                 else "L1 / L2 (scene L2-resident)")
        txt += (f" -- no unit saturated: latency-bound (dependent record fetches served from {where}) "
                "at the issue rate the resident waves sustain")
    return txt


def legacy_roofline_block(name, nbytes, ms, pmc, scene_bytes):
    """Rounds 3-5's roofline object (kept so their committed bench lines still recompute,
    tests/test_bench_roofline.py): algorithmic bytes priced against the L2 or HBM by a DRAM-bytes
    rule -- a model bound, replaced in round 6 by roofline_block's measured ceilings.

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


def step_trace_entry(cfg_name, arith):
    """rocprofv3 kernel trace of bench.py's own timed loop for a config (tools/step_trace.py,
    profiles/r06/step_trace_<config>_<arith>.json), or None."""
    p = os.path.join(REPO, "profiles", "r06", f"step_trace_{cfg_name}_{arith}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def roofline_step_block(nbytes, ms_step, world, pmc=None, launches_per_step=None, trace=None, scene_bytes=None):
    """The timed regime (K steps over --streams streams) priced at its ceilings, per GPU.

    Round 6: with the counters of the step's launch (`pmc`, per dispatch)
    the step's own counts are launches_per_step x those, over ms_per_step: the same measured
    ceilings as `roofline` (bound = the nearest, frac <= 1).  `trace` is the rocprofv3 kernel
    trace of this very loop (tools/step_trace.py): the GPU's busy time per step and the summed
    launch durations per step beside ms_per_step.  The algorithmic bytes per step stay as a side
    field."""
    if not nbytes or ms_step <= 0:
        return None
    job = nbytes / (ms_step * 1e-3) / 1e9
    per_gpu = job / world
    out = {"algorithmic_bytes_per_step": int(nbytes), "ms_per_step": round(ms_step, 5),
           "algorithmic": {"achieved_job_gbs": round(job, 1), "achieved_per_gpu_gbs": round(per_gpu, 1),
                           "frac_l2": round(per_gpu / L2_PEAK_GBS, 4), "frac_hbm": round(per_gpu / HBM_PEAK_GBS, 4),
                           "source": "per-view reference Statistics, tests/golden/orbit/<config>.json "
                                     "(64 B/node pair + 56 B/test); not a ceiling"}}
    ceil = measured_ceilings(pmc, ms_step, launches_per_step) if pmc and launches_per_step else {}
    if ceil:
        bname, b = max(ceil.items(), key=lambda kv: kv[1]["frac"] or 0.0)
        out.update({"bound": bname, "achieved": b["achieved"], "peak": b["peak"], "unit": b["unit"],
                    "frac": b["frac"], "launches_per_step": launches_per_step, "ceilings": ceil,
                    "limiter": limiter_text(ceil, pmc, scene_bytes)})
    else:
        out.update({"bound": "unmeasured", "frac": None})
    if trace:
        out["trace"] = {k: trace.get(k) for k in ("span_ms_per_step", "busy_ms_per_step", "kernel_ms_per_step",
                                                  "mean_launch_ms", "overlap", "bench_ms_per_step", "steps",
                                                  "streams")}
        out["trace"]["source"] = "rocprofv3 --kernel-trace of bench.py's timed loop (tools/step_trace.py, profiles/r06/)"
    return out


def legacy_roofline_step_block(nbytes, ms_step, world):
    """Rounds 4-5's step block (kept so their committed lines recompute): the algorithmic bytes of a
    step / ms_per_step, per GPU, against the L2 and HBM -- a model, not a measured ceiling."""
    if not nbytes or ms_step <= 0:
        return None
    job = nbytes / (ms_step * 1e-3) / 1e9
    per_gpu = job / world
    return {"algorithmic_bytes_per_step": int(nbytes), "ms_per_step": round(ms_step, 5), "unit": "GB/s",
            "achieved_job": round(job, 1), "achieved_per_gpu": round(per_gpu, 1),
            "frac_l2": round(per_gpu / L2_PEAK_GBS, 4), "frac_hbm": round(per_gpu / HBM_PEAK_GBS, 4)}


def counted_bytes(count_pkg, mesh, bvh, device, b12, s3, W, H, mode, tiling, with_float):
    """The build's own bytes for one launch (round 6): the same launch through
    the counting build (libceres_hip_count.so: the same kernels with a tally at every fetch site,
    `make count`), {kind: bytes}, vector kinds per lane, scalar kinds per wavefront, + totals."""
    import torch
    sc = count_pkg.Scene(mesh, bvh, device=device)
    F = len(b12)
    rgb = torch.empty(F * 3 * W * H, dtype=torch.uint8, device=f"cuda:{device}")
    px = torch.empty(F * 3 * W * H, dtype=torch.float32, device=f"cuda:{device}") if with_float else None
    count_pkg.fetch_counters(device, reset=True)
    til = count_pkg.Tiling(tiling.row_block, tiling.rank, tiling.world)      # the count module's own ctypes type
    err = torch.zeros(8, dtype=torch.int64, device=f"cuda:{device}")
    sc.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=0 if px is None else px.data_ptr(),
                           d_rgb8=rgb.data_ptr(), d_counters=err.data_ptr(), stream=0)
    c = count_pkg.fetch_counters(device, reset=True)
    sc.close()
    # this build also carries the production walk's stack guard (CERES_STACK_GUARD): its error word
    c["guard_error_word"] = int(err[6].item())
    vec = sum(v for k, v in c.items() if k.endswith("_vector"))
    scal = sum(v for k, v in c.items() if k.endswith("_scalar"))
    c.update({"vector_total": vec, "scalar_total": scal, "total": vec + scal,
              "note": "counting build: vector kinds x active lanes, scalar kinds once per wavefront; "
                      "stores included (store_vector)"})
    return c


def load_count_package():
    """The counting build as its own module instance (its own ctypes handle and code object), or
    None when it was not built."""
    import importlib.util
    path = os.path.join(PKG_DIR, "variants", "libceres_hip_count.so")
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location("ceres_count_build", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.LIB_PATH = path
    mod.lib()
    return mod


def host_cpus():
    """What the host exposes and what this process may use: the node's CPUs, the affinity mask,
    the cgroup CPU quota (cpu.max), OMP_NUM_THREADS."""
    info = {"node_cpus": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    return info


def choose_collect(requested, cfg, world, frames):
    """The N > 1 partition of a step (DESIGN.md "Multi-GPU").  "auto": the step's frames are the
    units -- each rank renders its 16 frames whole with no data-path collective ("frames"; render.hpp
    :104-153 touches one frame, pixels are independent) -- except for the configs BASELINE.json
    defines as ONE framebuffer tiled across the GPUs (configs.py "tiled": C4, C5) at N >= 4, whose
    frames are cut into contiguous bands -- rank r renders band (r + f) mod N of frame f -- and each
    band is sent point to point into its owner rank's frame ("bands", the north star's framebuffer
    partition; round 6: no un-interleave, one-GPU rehearsal at N = 8 with the exchange's traffic
    emulated C3 0.822 / C4 0.797 / C5 0.933 against 0.754 / 0.737 / 0.882 for "exchange", the round-5 row-interleaved
    blocks + all-to-all + assembly, which stays selectable).  At N = 2 those take "frames" too: the
    single xGMI link would carry 16 split frames' rows per step and outlast the render (C4 1.23x).
    The other partition is timed in the same run and reported beside it (alt_collect).  Partitions
    that deal whole frames need F to be a multiple of N, else every frame goes to rank 0 ("gather")."""
    collect = requested
    if collect == "auto":
        collect = "bands" if cfg.get("tiled") and world >= 4 else "frames"
    if collect in ("frames", "exchange", "bands") and frames % world:
        collect = "gather"
    return collect


def alt_collect(collect):
    """The other partition bench.py reports beside the headline one at N > 1 (`partition_alt`)."""
    return "frames" if collect in ("exchange", "bands", "gather") else "bands"


def result_line(*, config_name, cfg, world, backend, collect, views_kind, F, steps, warmup, T, rays_step,
                hits_step, full_mode, row_block, streams, float_fb, arith, roofline, roofline_step, roofline_solo,
                cpu, parity, alt=None, orbit=None):
    """bench.py's one JSON line (rank 0).  `T` = max-over-ranks wall seconds of the `steps` timed
    steps; value = the whole job's rays per second."""
    W, H = cfg["W"], cfg["H"]
    primary_step = F * W * H
    value = rays_step * steps / T / 1e6
    untiled = world > 1 and collect == "frames"
    line = {
        "metric": "Mrays/sec (primary+shadow) on dragon.obj 1920x1080; 1/2/4/8-GPU scaling"
        if config_name == "dragon_1080" else f"Mrays/sec ({config_name})",
        "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(T / steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "arith": arith,
        "world_size": world, "backend": backend,
        "data": ("real mesh from the reference repo (data/%s)" % cfg["obj"] if cfg["obj"] else
                 "procedural %dx%d-vertex heightfield generated in-process (SURVEY.md §8(d) C5 definition)"
                 % (cfg["proc"], cfg["proc"]))
                + ("; every frame = the config camera (static.cpp:39-47 for C3)" if views_kind == "config" else
                   "; frame 0 = the config camera, frames 1.. = the anim.cpp-style orbit about z"),
        "config": {"workload": f"{config_name}: {cfg['obj'] or 'proc'} {W}x{H} "
                               f"{'primary+shadow' if full_mode else 'primary only'}, "
                               + (f"{F} copies of the config view per step" if views_kind == "config"
                                  else f"{F} orbit frame(s) per step"),
                   "views": views_kind,
                   "W": W, "H": H, "frames_per_step": F, "rays_per_step": rays_step, "hits_per_step": hits_step,
                   "shadow_ray_frac": round((rays_step - primary_step) / rays_step, 4) if full_mode else 0.0,
                   "row_block": row_block if world > 1 and not untiled else H,
                   "parallelism": (f"untiled: unsplit frames x{world}, rank q renders frames q, q+{world}, ... "
                                   "whole, no collective" if untiled else
                                   (f"framebuffer cut into {world} contiguous bands of {row_block} rows, rank r renders "
                                    f"band (r + f) mod {world} of frame f; RCCL point-to-point sends each band into its "
                                    "owner rank's frame in place (pipelined, no assembly)" if collect == "bands" else
                                    f"framebuffer rows interleaved over {world} GPU(s) in blocks of {row_block} rows"
                                    + ((" + one RCCL all-to-all per step: frame f gathered to its owner rank "
                                        "(pipelined)" if collect == "exchange" else
                                        " + one RCCL gather per step to rank 0 (pipelined)")
                                       if world > 1 else ""))
                                   if world > 1 else "one GPU, whole frames"),
                   "collect": collect if world > 1 else None,
                   "float_framebuffer": float_fb, "streams": streams},
        # the step's one collective against the xGMI budget (DESIGN.md "Multi-GPU"): bytes one rank
        # receives per step, 1/N of them from each peer over that peer's direct link (one link per
        # peer in a fully connected 8-GPU node) at 76.8 GB/s per link and direction
        "collective": None if world == 1 or untiled else {
            "kind": {"exchange": "all_to_all", "bands": "p2p_bands"}.get(collect, "gather"),
            "recv_bytes_per_rank_step": (world - 1) * (F // world if collect in ("exchange", "bands") else F) * H * 3 * W
            // world,
            "xgmi_link_ms_est": round((F // world if collect in ("exchange", "bands") else F) * H * 3 * W / world / 76.8e6,
                                      4),
            "ms_per_step": round(T / steps * 1e3, 5)},
        "roofline": roofline, "roofline_step": roofline_step,
        "roofline_solo": roofline_solo, "cpu_baseline": cpu, "parity": parity,
    }
    if alt is not None:
        line["partition_alt"] = alt
    if orbit is not None:
        line["orbit_value"] = orbit["value"]
        line["orbit"] = orbit
    return line


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="dragon_1080")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per step (default: --frames-per-gpu x number of GPUs)")
    ap.add_argument("--frames-per-gpu", type=int, default=16,
                    help="frames of work per GPU per step when --frames is not given (weak scaling)")
    ap.add_argument("--views", choices=("config", "orbit"), default="config",
                    help="config: every frame of the step is the config's own view (C3 = static.cpp's camera, "
                         "the headline); orbit: frame f = the anim.cpp orbit view f x 360/F degrees about z")
    ap.add_argument("--row-block", type=int, default=16,
                    help="rows per block of the row-interleaved partitions (round 6: 16, was 8 -- the one-GPU "
                         "rehearsal at N = 8 predicts 0.919 render-only weak efficiency for C3 against 0.875 with "
                         "8-row blocks, C4 0.920 against 0.897; profiles/r06/rehearsal)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-count", action="store_true",
                    help="skip the counting build's pass (roofline.build_bytes: the build's own fetched bytes)")
    ap.add_argument("--no-orbit", action="store_true",
                    help="skip the second timed loop over the orbit views (`orbit_value`)")
    ap.add_argument("--no-alt", action="store_true",
                    help="N > 1: skip the timed loop of the other partition (`partition_alt`)")
    ap.add_argument("--no-float", action="store_true", help="skip the float framebuffer (RGB8 only)")
    ap.add_argument("--collect", choices=("auto", "frames", "exchange", "bands", "gather"), default="auto",
                    help="N > 1: bands = every frame cut into N contiguous bands, rank r renders band (r + f) mod N "
                         "of frame f, each band sent point to point into its owner rank's frame (no un-interleave); "
                         "exchange = rows dealt in blocks, each frame gathered to one owner rank in one RCCL "
                         "all-to-all + un-interleave; frames = each rank renders its F/N frames whole (no "
                         "collective); gather = rows dealt, all frames to rank 0; auto = frames, except bands "
                         "for the tiled C4/C5 at N >= 4 (choose_collect; DESIGN.md \"Multi-GPU\")")
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
    backend = None
    if world > 1:
        backend = os.environ.get("CERES_BENCH_BACKEND", "nccl")      # gloo: shared-GPU rehearsal only
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        world = dist.get_world_size()

    W, H = cfg["W"], cfg["H"]
    F = args.frames or args.frames_per_gpu * world
    build = "ref" if args.arith == "fma" else "exact"          # the fixtures' key for this arithmetic
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    scene = pkg.Scene(mesh, bvh, device=local_rank)
    # the orbit: frame f rotated once by f x 360 / F degrees (frame 0 = the config view, fixture bits)
    ob12, os3, osteps = pkg.bench_views(cam, cfg["sun"], W, H, F, basis0=pinned_basis(meta, cfg, cam, build))
    # C5's z orbit leaves the [0,1]^2 heightfield for views 40..96 of 128 (no triangle in view), so
    # its orbit is never a bench step; every config's headline step is F copies of its own view
    views_kind = "config" if cfg.get("bench_view0") else args.views

    def view_set(kind):
        if kind == "config":
            return np.repeat(ob12[:1], F, 0), np.repeat(os3[:1], F, 0), np.repeat(osteps[:1], F)
        return ob12, os3, osteps

    mode = pkg.cfg_mode(cfg, arith)
    full_mode = (mode & 0xf) == pkg.MODE_FULL
    S = max(1, args.streams)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    # steps rotate over S streams, each with its own framebuffers / collective slot: a step's frames
    # are complete when its stream is, and step k+1's kernel fills the tail of step k (a single
    # frame ends with a few long wavefronts resident, DESIGN.md "Where the time goes")
    streams = [stream] if S == 1 else [torch.cuda.Stream(device=dev) for _ in range(S)]
    slots = max(2, S)
    MAXF = 64                                    # frames per ceres_render_batch_device launch (kMaxFrames)

    class Run:
        """One partition of the step over the ranks (`collect`) and one set of views, with its
        framebuffers and collective slots: validate() and timed() as the bench contract says."""

        def __init__(self, collect, kind):
            self.collect, self.kind = collect, kind
            b12, s3, steps_deg = view_set(kind)
            self.owner = world > 1 and collect == "frames"              # unsplit frames: no collective
            self.exchange = world > 1 and collect in ("exchange", "frames", "bands")
            if self.exchange:
                # batch order for the all-to-all: rank q owns batch frames q*k .. q*k+k-1, which are
                # orbit frames q, q + N, q + 2N, ... (batch frame 0 = orbit frame 0 = the config view)
                order = D.exchange_order(F, world)
                b12, s3, steps_deg = b12[order], s3[order], steps_deg[order]
            self.row_block = args.row_block if world > 1 and not self.owner else H
            self.tiling = pkg.Tiling(self.row_block, rank, world) if not self.owner else pkg.Tiling(H, 0, 1)
            self.job = steps_deg                     # the whole job's views, in batch order
            self.Fl = F                              # frames this rank's launches render
            if self.owner:
                self.gather = D.FrameOwner(W, H, rank, world, frames=F, device=dev, slots=slots)
                mine = self.gather.owned_frames()
                self.Fl = len(mine)
                b12, s3 = b12[mine], s3[mine]
            elif collect == "bands":   # contiguous bands rotated per frame, received in place (no assembly)
                self.gather = D.FrameBands(W, H, rank, world, frames=F, device=dev, slots=slots)
                self.row_block = self.gather.band
                self.tiling = pkg.Tiling(*self.gather.tiling_args())
            elif self.exchange:   # each frame to one owner rank: a rank's ingress is (N-1)/N of its k frames
                self.gather = D.FrameExchange(W, H, self.row_block, rank, world, frames=F, device=dev, slots=slots)
            else:                 # every frame -> rank 0
                self.gather = D.BatchGather(W, H, self.row_block, rank, world, frames=F, device=dev, slots=slots)
            self.b12, self.s3 = b12, s3
            self.rows = self.gather.local_rows
            self.d_px = [None if args.no_float else
                         torch.empty(self.Fl * 3 * W * max(self.rows, 1), dtype=torch.float32, device=dev)
                         for _ in range(S)]
            self.pending = [False] * slots
            self.chunk_counters = [torch.zeros(8, dtype=torch.int64, device=dev)
                                   for _ in range((self.Fl + MAXF - 1) // MAXF)]
            self.counters = torch.zeros(8, dtype=torch.int64, device=dev)

        def call_tiling(self, f0):
            """The tiling of a call whose frame 0 is batch frame f0 (bands rotate with the frame)."""
            t = self.tiling
            return pkg.Tiling(t.row_block, (t.rank + f0) % t.world, t.world, 1) if t.bands else t

        def render(self, slot, st, with_counters=False):
            # one launch per (at most) 64 frames of the step; frame f's rows at f * 3 * W * rows
            px = self.d_px[slot % S]
            fb = 3 * W * max(self.rows, 1)
            for c, f0 in enumerate(range(0, self.Fl, MAXF)):
                f1 = min(self.Fl, f0 + MAXF)
                scene.render_batch_device(self.b12[f0:f1], self.s3[f0:f1], W, H, mode=mode, tiling=self.call_tiling(f0),
                                          d_pixels=0 if px is None else px.data_ptr() + 4 * fb * f0,
                                          d_rgb8=self.gather.local_ptr(slot) + fb * f0,
                                          d_counters=self.chunk_counters[c].data_ptr() if with_counters else 0,
                                          stream=st.cuda_stream)
            if with_counters:
                with torch.cuda.stream(st):
                    cs = torch.stack(self.chunk_counters)
                    self.counters.copy_(torch.cat([cs[:, :6].sum(0), cs[:, 6:7].max(0).values, cs[:, 7:].sum(0)]))

        def step(self, k):
            slot = k % slots
            st = streams[k % S]
            with torch.cuda.stream(st):
                if self.pending[slot]:             # the previous use of this slot (step k - slots)
                    self.gather.finish(slot)
                    self.pending[slot] = False
                self.render(slot, st)
                self.gather.start(slot)
                self.pending[slot] = True
                if S == 1:                         # one stream: complete the previous step's gather now
                    prev = (k - 1) % slots
                    if self.pending[prev] and prev != slot:
                        self.gather.finish(prev)
                        self.pending[prev] = False

        def drain(self):
            for k_ in range(slots):
                if self.pending[k_]:
                    with torch.cuda.stream(streams[k_ % S]):
                        self.gather.finish(k_)
                    self.pending[k_] = False
            self.gather.wait_assembled()

        def validate(self):
            """Untimed: one counted step.  Returns (rays, hits, checks) where checks compares every
            frame this rank assembled with the REFERENCE's PPM of the same view
            (tests/golden/orbit/<config>.json; sha256 of "P6 W H 255\\n" + body, static.cpp:135-147)
            and the step's rays / hits with the reference's per-view counts (render.hpp:155)."""
            self.render(0, stream, with_counters=True)
            self.gather.start(0)
            full = self.gather.finish(0)
            self.gather.wait_assembled()
            torch.cuda.synchronize(dev)
            c = self.counters.clone()
            if world > 1:
                dist.all_reduce(c)
            c = c.cpu().numpy()
            if c[6]:
                # ceres_finalize's error word: a traversal stack overflowed (single_ray_traverser.hpp:29
                # asserts instead), so some frame of the batch is wrong -- never time a wrong render
                raise SystemExit(f"bench.py: traversal stack overflow in the validation batch (error word {int(c[6]):#x})")
            # The production kernels' BVH2 walk has no per-step stack check (the bound is exact by
            # construction); the stats kernels -- the same walk in the same order, with clamps and
            # the overflow flag -- trace this rank's views of the step once more, and the timed
            # loop runs only if they report no overflow.
            sc_stats = pkg.Scene(mesh, bvh, device=local_rank, stats=True)
            cs = torch.zeros(8, dtype=torch.int64, device=dev)
            # (band launches have no stats kernels: there the pass deals the same frames' rows in row
            # blocks -- over the ranks it still traces every ray of the step)
            st_til = pkg.Tiling(args.row_block, rank, world) if self.tiling.bands else None
            st_rows = pkg.local_rows(H, st_til) if st_til is not None else self.rows
            for f0 in range(0, self.Fl, MAXF):
                f1 = min(self.Fl, f0 + MAXF)
                tmp = torch.empty((f1 - f0) * 3 * W * max(st_rows, 1), dtype=torch.uint8, device=dev)
                sc_stats.render_batch_device(self.b12[f0:f1], self.s3[f0:f1], W, H, mode=mode,
                                             tiling=st_til if st_til is not None else self.call_tiling(f0),
                                             d_rgb8=tmp.data_ptr(), d_counters=cs.data_ptr(), stream=stream.cuda_stream)
                torch.cuda.synchronize(dev)
                if int(cs[6].item()):
                    raise SystemExit("bench.py: the stats kernels report a traversal stack overflow for the step's views")
            sc_stats.close()
            self.stack_checked = True
            mine = (list(zip(self.gather.owned_frames(), full)) if self.exchange
                    else ([(f, full[f]) for f in range(F)] if rank == 0 else []))
            head = b"P6 %d %d 255\n" % (W, H)
            n = [0, 0, 0]                                            # [checked, matched, unpinned]
            for f, body in mine:
                e = None if orbit_fx is None else view_entry(orbit_fx.get(step_key(self.job[f])), build)
                if e is None:
                    n[2] += 1
                    continue
                n[0] += 1
                n[1] += int(hashlib.sha256(head + body.cpu().numpy().tobytes()).hexdigest() == e["sha256"])
            stat = torch.tensor(n, dtype=torch.int64, device=dev)
            if world > 1:
                dist.all_reduce(stat)
            stat = stat.cpu().numpy()
            keys = [None if orbit_fx is None else view_entry(orbit_fx.get(step_key(x)), build) for x in self.job]
            ref_rays = sum(e["rays"] for e in keys) if all(keys) else None
            ref_hits = sum(e["hits"] for e in keys) if all(keys) else None
            checks = {"frames": F, "frames_checked": int(stat[0]), "frames_unpinned": int(stat[2]),
                      "stack_bound_checked": "production error word (BVH4 walks) + a stats-kernel pass of the "
                                             "step's views (BVH2 clamps + overflow flag): no overflow",
                      "all_frames_match_reference": bool(stat[2] == 0 and stat[1] == stat[0] == F),
                      "step_rays_match_reference": None if ref_rays is None else int(c[0]) == ref_rays,
                      "step_hits_match_reference": None if ref_hits is None else int(c[1]) == ref_hits}
            return int(c[0]), int(c[1]), checks

        def timed(self, prime):
            """W warmup steps (after >= --prime-s of untimed steps when `prime`), then exactly K steps
            between barrier + device synchronise; returns the max-over-ranks wall time."""
            if prime:
                # untimed setup before the W warmup steps: steps over every stream and collective slot
                # for at least --prime-s seconds, so no stream's first launch lands in the timed region
                # when W < S and the GPU has left its idle clock state (measured: K = 20 after W = 5
                # from a cold start ran 6 % below the same K after W = 200; after this priming they agree)
                t_prime = time.perf_counter()
                for k in range(slots):
                    self.step(k)
                self.drain()
                torch.cuda.synchronize(dev)
                per_step = max((time.perf_counter() - t_prime) / slots, 1e-5)
                # the same number of steps on every rank (each step is a collective)
                more = torch.tensor([min(20000, max(0, int(args.prime_s / per_step) - slots))], dtype=torch.int64,
                                    device=dev)
                if world > 1:
                    dist.all_reduce(more, op=dist.ReduceOp.MAX)
                for k in range(int(more.item())):
                    self.step(slots + k)
                self.drain()
                torch.cuda.synchronize(dev)
            for k in range(args.warmup):
                self.step(k)
            self.drain()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(args.steps):
                self.step(k)
            self.drain()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            if world > 1:
                dist.barrier()
            elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
            return float(elapsed.item())

        def close(self):
            self.d_px = self.gather = None

    def step_bytes(steps):
        """Algorithmic bytes of one step's frames (whole job), from every view's pinned reference
        statistics, or None when a view is unpinned."""
        if orbit_fx is None:
            return None
        es = [view_entry(orbit_fx.get(step_key(x)), build) for x in steps]
        if not all(e is not None and "stats" in e for e in es):
            return None
        return int(sum(algorithmic_bytes(e["stats"]) for e in es))

    primary_step = F * W * H

    def loop_block(run, rays, hits, checks, T):
        return {"value": round(rays * args.steps / T / 1e6, 3), "unit": "Mrays/s",
                "ms_per_step": round(T / args.steps * 1e3, 5), "rays_per_step": rays, "hits_per_step": hits,
                "shadow_ray_frac": round((rays - primary_step) / rays, 4) if full_mode else 0.0,
                "roofline_step": roofline_step_block(step_bytes(run.job), T / args.steps * 1e3, world),
                "parity": checks}

    collect = choose_collect(args.collect, cfg, world, F)
    main_run = Run(collect, views_kind)
    # validation step (not timed): exact counts + every frame vs the reference
    rays_step, hits_step, step_checks = main_run.validate()
    parity = None
    if rank == 0 and meta is not None:
        # frame 0's ray / hit counts (render.hpp:155) from a counted whole-frame render of the config view
        c0 = torch.zeros(8, dtype=torch.int64, device=dev)
        rgb0 = torch.empty(3 * W * H, dtype=torch.uint8, device=dev)
        scene.render_device(ob12[0], os3[0], W, H, mode=mode, tiling=pkg.Tiling(H, 0, 1), d_rgb8=rgb0.data_ptr(),
                            d_counters=c0.data_ptr(), stream=sh)
        torch.cuda.synchronize(dev)
        c0 = c0.cpu().numpy()
        body = b"P6 %d %d 255\n" % (W, H) + rgb0.view(H, 3 * W).cpu().numpy().tobytes()
        parity = {"reference_build": "reference CMake flags (-O3 -mavx2 -mfma, GCC FMA contraction)" if build == "ref"
                  else "reference with -ffp-contract=off",
                  "frame0_ppm_sha256_matches_reference": hashlib.sha256(body).hexdigest() == meta["ppm_sha256"][build],
                  "rays_match": int(c0[0]) == meta[build]["rays"], "hits_match": int(c0[1]) == meta[build]["hits"]}
        parity.update(step_checks)

    T = main_run.timed(prime=True)
    bytes_step = step_bytes(main_run.job)
    main_run.close()
    del main_run
    torch.cuda.empty_cache()

    alt = None
    if world > 1 and not args.no_alt:
        # the other partition of the same step, same views (frames <-> exchange)
        acol = choose_collect(alt_collect(collect), cfg, world, F)
        if acol != collect:
            run = Run(acol, views_kind)
            r_, h_, ch_ = run.validate()
            Ta = run.timed(prime=True)
            alt = dict(collect=acol, **loop_block(run, r_, h_, ch_, Ta))
            run.close()
            del run
            torch.cuda.empty_cache()

    orbit = None
    if views_kind == "config" and not args.no_orbit and not cfg.get("bench_view0"):
        # the same loop over the anim.cpp orbit views (frame f turned f x 360/F degrees about z): lighter
        # than the config view on dragon (fewer shadow rays per frame), reported beside it
        run = Run(collect, "orbit")
        r_, h_, ch_ = run.validate()
        To = run.timed(prime=False)
        orbit = loop_block(run, r_, h_, ch_, To)
        run.close()
        del run
        torch.cuda.empty_cache()

    roofline = roofline_solo = None
    cpu = None
    if rank == 0 and not args.no_roofline and meta is not None:
        # the step's kernel: one 16-frame launch of the step's views (whole frames; views_kind
        # "config": 16 copies of the config view), n_b launches back to back on ONE stream between two
        # HIP events -- no other stream's work overlaps, so the mean is a per-launch duration (and
        # agrees with a single-stream trace of tools/batch_launch.py)
        nb_f = min(16, F)
        vb12, vs3, vsteps = view_set(views_kind)
        order = np.argsort(vsteps, kind="stable")[:nb_f]
        vb12, vs3, vsteps = vb12[order], vs3[order], vsteps[order]
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
            pmc_views = "" if views_kind == "config" else "_orbit"
            batch_pmc = pmc_entry(args.config, f"{kname}_batch{nb_f}{pmc_views}_{args.arith}")
            counted = None
            if not args.no_count:
                cp = load_count_package()
                if cp is not None:
                    counted = counted_bytes(cp, mesh, bvh, local_rank, vb12, vs3, W, H, mode, whole, bat_px is not None)
            roofline = roofline_block(kname, bb, batch_ms, batch_pmc, scene.info()["device_bytes"], counted=counted)
            what = (f"{nb_f} copies of the config view" if views_kind == "config" else
                    f"{nb_f} orbit views (steps {vsteps[0]:g}..{vsteps[-1]:g} deg)")
            roofline.update(launch=f"ceres_render_batch_device, {what}, whole {W}x{H} frames, {n_b} launches "
                                   f"back to back on one stream", frames_per_launch=nb_f, views=views_kind)
        del bat_rgb, bat_px
        # one full frame per launch (the render() call's regime), timed live with HIP events on the
        # launch stream
        solo = pkg.Tiling(H, 0, 1)
        solo_rgb = torch.empty(3 * W * H, dtype=torch.uint8, device=dev)
        solo_px = torch.empty(3 * W * H, dtype=torch.float32, device=dev)
        n_t = max(10, min(args.steps, 200))
        for _ in range(3):                            # the solo frame's tile order, warm
            scene.render_device(ob12[0], os3[0], W, H, mode=mode, tiling=solo, d_pixels=solo_px.data_ptr(),
                                d_rgb8=solo_rgb.data_ptr(), stream=sh)
        # n_t back-to-back launches between two HIP events on their stream: mean launch duration
        # (per-launch event pairs would add each launch's dispatch latency, ~13 us here)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(n_t):
            scene.render_device(ob12[0], os3[0], W, H, mode=mode, tiling=solo, d_pixels=solo_px.data_ptr(),
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
    # the step's counts: its render launches (one per <= 56 frames per rank; rank 0's) x the counters of
    # the 16-frame launch `roofline` prices (the step IS such launches: 16 copies of the config view)
    step_pmc = None
    launches_step = None
    if world == 1 and F % 16 == 0:
        kstep = "ceres_fused" if full_mode else "ceres_primary"
        step_pmc = pmc_entry(args.config, f"{kstep}_batch16{'' if views_kind == 'config' else '_orbit'}_{args.arith}")
        launches_step = F // 16
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, cfg, meta[build]["rays"] if meta else rays_step // F, build=build)

    if rank == 0:
        line = result_line(config_name=args.config, cfg=cfg, world=world, backend=backend, collect=collect,
                           views_kind=views_kind, F=F, steps=args.steps, warmup=args.warmup, T=T,
                           rays_step=rays_step, hits_step=hits_step, full_mode=full_mode, row_block=args.row_block,
                           streams=S, float_fb=not args.no_float, arith=args.arith, roofline=roofline,
                           roofline_step=roofline_step_block(bytes_step, T / args.steps * 1e3, world, step_pmc,
                                                             launches_step, step_trace_entry(args.config, args.arith),
                                                             scene_bytes=scene.info()["device_bytes"]),
                           roofline_solo=roofline_solo, cpu=cpu, parity=parity, alt=alt, orbit=orbit)
        line["native"] = pkg.native_provenance()
        print(json.dumps(line), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
