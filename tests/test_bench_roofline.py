"""bench.py's roofline object (CPU): the bound is chosen from the measured counters, never
hard-coded, and no field named as the bound exceeds its peak.

Checked two ways: synthetic counter summaries through `bench.roofline_block`, and every committed
bench line (`profiles/r03_end/sweep/bench_*.log`, `profiles/r0[45]/**/bench_*.log`) recomputed from its
own algorithmic bytes, mean launch time and `profiles/pmc_summary.json` entry (round 5: the
session's own `pmc_summary_*.json` beside the log when it has the entry); round-4 lines also
carry `roofline_step` (the timed regime), whose bytes are recomputed from the per-view reference
statistics of tests/golden/orbit/<cfg>.json."""
import glob
import importlib.util
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("ceres_bench", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bound_follows_counters(bench):
    nbytes, ms = 1_362_909_224, 0.1647
    l2 = bench.roofline_block("ceres_fused", nbytes, ms, {"hbm_bytes_per_launch": 52e6,
                                                         "waitcnt_parked_frac": 0.36, "ta_busy_frac": 0.10,
                                                         "l2_hit_rate": 0.67}, 3_764_016)
    assert l2["bound"] == "l2" and l2["peak"] == bench.L2_PEAK_GBS
    assert 0 < l2["frac"] <= 1 and l2["hbm_frac_algorithmic"] > 1     # bytes served on-die
    assert "L2-resident" in l2["limiter"]
    hbm = bench.roofline_block("k", 1e9, 0.2, {"hbm_bytes_per_launch": 0.9e9,
                                               "waitcnt_parked_frac": 0.2, "ta_busy_frac": 0.6}, 1 << 30)
    assert hbm["bound"] == "hbm" and hbm["peak"] == bench.HBM_PEAK_GBS
    assert hbm["limiter"] == "HBM bandwidth"                            # 4.5 TB/s of DRAM traffic
    dram_lat = bench.roofline_block("k", 2e9, 3.0, {"hbm_bytes_per_launch": 1.5e9,
                                                    "waitcnt_parked_frac": 0.55, "l2_hit_rate": 0.75},
                                   1_260_000_000)
    assert dram_lat["bound"] == "hbm" and dram_lat["frac"] < 0.1
    assert dram_lat["limiter"].startswith("dependent-load latency") and "DRAM" in dram_lat["limiter"]
    none = bench.roofline_block("k", 1e9, 1.0, None, 1 << 20)
    assert none["traffic"] is None and none["limiter"].startswith("unmeasured")


def _bench_lines():
    out = []
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "r03_end", "sweep", "bench_*.log")) +
                    glob.glob(os.path.join(REPO, "profiles", "r04", "**", "bench_*.log"), recursive=True) +
                    glob.glob(os.path.join(REPO, "profiles", "r05", "**", "bench_*.log"), recursive=True)):
        with open(p) as f:
            lines = [ln for ln in f if ln.startswith("{") and '"roofline"' in ln]
        if lines:
            out.append((os.path.relpath(p, os.path.join(REPO, "profiles")), json.loads(lines[-1])))
    return out


def _pmc_key(line, rf, which):
    """The pmc_summary.json kernel key a line's roofline block was priced with."""
    if "arith" not in line:                               # round-3 lines: the solo launch, no suffix
        return rf["kernel"]
    if which == "roofline" and "frames_per_launch" in rf:
        # round 5: the batch launch is 16 copies of the config view ("views": "config"); orbit
        # batches carry an "_orbit" key (round-4 lines: orbit batches without the suffix)
        orbit = "_orbit" if rf.get("views") == "orbit" else ""
        return f"{rf['kernel']}_batch{rf['frames_per_launch']}{orbit}_{line['arith']}"
    return f"{rf['kernel']}_solo_{line['arith']}"


def _session_pmc(name, cfg, key):
    """The counters a round-5 session priced its bench line with: that session's own summary
    (`pmc_summary_*.json` beside the bench log, merged into profiles/pmc_summary.json on the box
    before the bench ran), which a later session's merge may have replaced globally."""
    for p in glob.glob(os.path.join(REPO, "profiles", os.path.dirname(name), "pmc_summary_*.json")):
        with open(p) as f:
            e = json.load(f).get(cfg, {}).get(key)
        if e is not None:
            return e
    return None


@pytest.mark.parametrize("name,line", _bench_lines())
def test_committed_sweep_roofline_recomputes(bench, name, line):
    cfg = line["config"]["workload"].split(":")[0]
    for which in ("roofline", "roofline_solo"):
        rf = line.get(which)
        if rf is None:
            continue
        key = _pmc_key(line, rf, which)
        pmc = _session_pmc(name, cfg, key) or bench.pmc_entry(cfg, key)   # None: the line must say "unmeasured"
        if which == "roofline_solo" and line.get("arith") == "exact" and rf["traffic"] is not None and \
                (pmc or {}).get("hbm_bytes_per_launch") != rf["traffic"]:
            pmc = bench.pmc_entry(cfg, rf["kernel"])          # bench.py's fallback for the exact solo launch
        again = bench.roofline_block(rf["kernel"], rf["algorithmic_bytes_per_launch"], rf["mean_launch_ms"],
                                     pmc, rf["scene_device_bytes"])
        if rf["traffic"] is None and pmc is not None:
            # the counters were collected after this line (same build, same launch): the line
            # recomputes to the priced block; only its bound may then differ
            assert rf["limiter"].startswith("unmeasured"), (name, which)
        else:
            for k in ("bound", "peak", "traffic", "limiter"):
                assert again[k] == rf[k], (name, which, k)
        assert abs(again["achieved"] - rf["achieved"]) <= 1e-3 * rf["achieved"] + 0.2
        assert again["frac"] <= 1.0, (name, which, again["frac"])
    assert line["parity"]["all_frames_match_reference"] is True
    if line.get("roofline") and "arith" in line and line.get("world_size", 1) == 1:
        _check_trace_agreement(name, line)


def _check_trace_agreement(name, line):
    """Round 5: a bench line kept next to a single-stream rocprofv3 trace of the
    same launch (`<dir>/trace_batch_<cfg>_<arith>_kernel_stats.csv`, tools/batch_launch.py under
    rocprofv3 --kernel-trace --stats, same session) must agree with it on the mean launch duration
    within 3 %."""
    import csv
    rf = line["roofline"]
    cfg = line["config"]["workload"].split(":")[0]
    # the trace kept in the same directory as the bench line (one session, one build)
    for p in glob.glob(os.path.join(REPO, "profiles", os.path.dirname(name),
                                    f"trace_batch_{cfg}_{line['arith']}_kernel_stats.csv")):
        with open(p) as f:
            rows = [r for r in csv.DictReader(f) if rf["kernel"] + "<" in r["Name"]]
        assert rows, p
        avg_ms = float(rows[0]["AverageNs"]) / 1e6
        assert abs(avg_ms - rf["mean_launch_ms"]) <= 0.03 * avg_ms, (name, p, avg_ms, rf["mean_launch_ms"])


@pytest.mark.parametrize("name,line", [x for x in _bench_lines() if "roofline_step" in x[1]])
def test_committed_roofline_step_recomputes(bench, name, line):
    """roofline_step = the step's algorithmic bytes (every frame's pinned reference statistics, in the
    line's arithmetic) / ms_per_step, per GPU, against L2 and HBM."""
    rs = line["roofline_step"]
    cfg = line["config"]["workload"].split(":")[0]
    import numpy as np
    sys_path = os.path.join(REPO, "ceres-raytracer_amd")
    import sys
    if sys_path not in sys.path:
        sys.path.insert(0, sys_path)
    import configs
    fx = bench.load_orbit_fixture(cfg)
    build = "ref" if line["arith"] == "fma" else "exact"
    F = line["config"]["frames_per_step"]
    # round 5: "views": "config" = every frame is the config view (orbit step 0)
    views = line["config"].get("views", "orbit")
    steps = [configs.orbit_step(f, F) if views == "orbit" else 0.0 for f in range(F)]
    nbytes = sum(bench.algorithmic_bytes(bench.view_entry(fx[bench.step_key(np.float32(x))], build)["stats"])
                 for x in steps)
    assert nbytes == rs["algorithmic_bytes_per_step"]
    again = bench.roofline_step_block(nbytes, line["ms_per_step"], line["n_gpus"])
    for k in ("achieved_job", "achieved_per_gpu", "frac_l2", "frac_hbm"):
        assert abs(again[k] - rs[k]) <= 1e-3 * abs(rs[k]) + 1e-3, k
    # per-ray bytes may exceed the L2 rate (packets: one scalar-cache read per wavefront for ~60
    # rays; L1 hits); bench.py says so in the block
    assert again["frac_l2"] <= 1.0 or rs.get("above_l2_note"), (name, again["frac_l2"])


def test_headline_trace_pairing_is_kept():
    """The final build's headline launch has its bench line and single-stream trace side by side
    (the check above is not vacuous): at least one profiles/r05 directory holds both."""
    pairs = [p for p in glob.glob(os.path.join(REPO, "profiles", "r05", "**", "trace_batch_dragon_1080_fma_kernel_stats.csv"),
                                  recursive=True) if os.path.exists(os.path.join(os.path.dirname(p), "bench_dragon_1080.log"))]
    assert pairs
