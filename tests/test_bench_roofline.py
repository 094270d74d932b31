"""bench.py's roofline object (CPU): the bound is chosen from the measured counters, never
hard-coded, and no field named as the bound exceeds its peak.

Checked two ways: synthetic counter summaries through `bench.roofline_block`, and every bench
line of the committed end-of-round sweep (`profiles/r03_end/sweep/bench_*.log`) recomputed from
its own algorithmic bytes, mean launch time and `profiles/pmc_summary.json` entry."""
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
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "r03_end", "sweep", "bench_*.log"))):
        with open(p) as f:
            lines = [ln for ln in f if ln.startswith("{") and '"roofline"' in ln]
        if lines:
            out.append((os.path.basename(p), json.loads(lines[-1])))
    return out


@pytest.mark.parametrize("name,line", _bench_lines())
def test_committed_sweep_roofline_recomputes(bench, name, line):
    rf = line["roofline"]
    cfg = line["config"]["workload"].split(":")[0]
    pmc = bench.pmc_entry(cfg, rf["kernel"])          # None (C1): the line must say "unmeasured"
    again = bench.roofline_block(rf["kernel"], rf["algorithmic_bytes_per_launch"], rf["mean_launch_ms"],
                                 pmc, rf["scene_device_bytes"])
    for k in ("bound", "peak", "traffic", "limiter"):
        assert again[k] == rf[k], (name, k)
    assert abs(again["frac"] - rf["frac"]) <= 2e-4 * max(1.0, rf["frac"]) + 1e-4
    assert rf["frac"] <= 1.0, (name, rf["frac"])
    assert line["parity"]["all_frames_match_reference"] is True
