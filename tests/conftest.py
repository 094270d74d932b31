"""Shared test setup: the `gpu` marker, package import, oracle (checker) import, fixtures."""
import gzip
import importlib.util
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "ceres-raytracer_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, PKG_DIR)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def import_package():
    """Import ceres-raytracer_amd/ (hyphenated directory) as module `ceres_raytracer_amd`."""
    if "ceres_raytracer_amd" in sys.modules:
        return sys.modules["ceres_raytracer_amd"]
    spec = importlib.util.spec_from_file_location("ceres_raytracer_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ceres_raytracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def golden_names():
    return sorted(f[:-5] for f in os.listdir(GOLDEN) if f.endswith(".json"))


def load_golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    rec = dict(np.load(os.path.join(GOLDEN, name + ".records.npz")))
    ppm = {}
    for kind in ("exact", "ref"):
        p = os.path.join(GOLDEN, f"{name}.{kind}.ppm.gz")
        if os.path.exists(p):
            with open(p, "rb") as f:
                ppm[kind] = gzip.decompress(f.read())
    if "exact" in ppm and "ref" not in ppm:
        ppm["ref"] = ppm["exact"]
    return meta, rec, ppm


def load_ref_records(name):
    """<name>.ref.records.npz: the per-pixel records of the reference-flag build (make_golden.py)."""
    return dict(np.load(os.path.join(GOLDEN, name + ".ref.records.npz")))


def ref_scene_hashes(meta, contract):
    """(tri48, norm36, canonical BVH) sha256 of the fixture's exact or reference-flag build."""
    if contract:
        r = meta["ref_scene"]
        return r["tri48_sha256"], r["norm36_sha256"], r["bvh_canonical_sha256"]
    return meta["tri48_sha256"], meta["norm36_sha256"], meta["bvh_canonical_sha256"]


def load_orbit(name):
    """tests/golden/orbit/<name>.json (make_golden.py --orbit): the reference's PPM sha256 and
    rays / hits of every bench orbit view, keyed by the float32 step's hex bits."""
    with open(os.path.join(GOLDEN, "orbit", name + ".json")) as f:
        return json.load(f)


def hexbits(a):
    return ["0x%08x" % int(x) for x in np.asarray(a, np.float32).view(np.uint32)]


def ppm_budget_ok(a, b, W, H, frac=1e-5):
    """SURVEY.md §7 parity budget: every channel within +-1 LSB, except <= max(1, frac*W*H) pixels."""
    a = np.frombuffer(a, np.uint8).astype(np.int16)
    b = np.frombuffer(b, np.uint8).astype(np.int16)
    assert a.shape == b.shape
    d = np.abs(a - b)
    hdr = len(b"P6 %d %d 255\n" % (W, H))
    d = d[hdr:].reshape(-1, 3).max(axis=1)
    bad = int(np.count_nonzero(d > 1))
    return bad <= max(1, int(frac * W * H)), bad


@pytest.fixture(scope="session")
def pkg():
    return import_package()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle
