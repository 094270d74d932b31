"""Double precision (render<double>, anim.cpp -d): the product's host scene preparation in
double -- OBJ load with strtof coordinates widened to double and double normal sums
(obj_norms.hpp:57-118), rotate_triangles<double> (render.hpp:24-44), BinnedSahBuilder over
Bvh<double> (64-B nodes), the double camera basis (render.hpp:91-97) and the Transform<double>
orbit (anim.cpp:76-88) -- equals the reference's own double build bit for bit
(tests/golden/f64/, made by tests/golden/make_golden_f64.py from oracle/_ref/ref_render_f64)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

import configs

F64 = os.path.join(GOLDEN, "f64")
NAMES = sorted(f[:-5] for f in os.listdir(F64) if f.endswith(".json"))


def hex64(a):
    return ["0x%016x" % int(x) for x in np.asarray(a, np.float64).view(np.uint64)]


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("build", ["exact", "ref"])
def test_f64_scene_prep_matches_reference(pkg, name, build):
    """build "exact": the -ffp-contract=off double build; "ref": the reference's own CMake build
    (-O3 -mavx2 -mfma, GCC's FMA contraction; CERES_ARITH_FMA) -- round 5."""
    import make_golden_f64
    meta = json.load(open(os.path.join(F64, name + ".json")))
    cfg = configs.CONFIGS[name]
    arith = 1 if build == "ref" else 0
    want = meta["ref_scene"] if build == "ref" else meta
    basis, pose = (meta["ref_basis"], meta["ref_pose"]) if build == "ref" else (meta["basis"], meta["pose"])
    mesh, bvh, cam = pkg.prepare(cfg, f64=True, arith=arith)
    assert mesh.tri.dtype == np.float64 and len(mesh) == meta["n_tri"]
    assert hashlib.sha256(mesh.tri.tobytes()).hexdigest() == want["tri96_sha256"]
    assert hashlib.sha256(mesh.norm.tobytes()).hexdigest() == want["norm72_sha256"]
    assert make_golden_f64.canonical_bvh64_sha(bvh.nodes.tobytes(), bvh.prim.tobytes()) == want["bvh_canonical_sha256"]
    if build == "exact":
        assert bvh.nodes.shape[0] == meta["n_nodes"]
    b = cam.basis(cfg["W"], cfg["H"])
    assert hex64(b[:3]) == pose["eye"]
    assert hex64(b[3:]) == basis["dir"] + basis["u"] + basis["v"]
    assert hex64(pkg.pose_f64(cfg, arith)[1]) == pose["sun"]


def test_f64_builds_differ_in_the_scene():
    """The two double builds do prepare different scenes (FMA contraction of the normals and the
    rotation), so the "ref" cases above pin something the "exact" ones do not."""
    differ = [n for n in NAMES if json.load(open(os.path.join(F64, n + ".json")))["ref_scene"]["tri96_sha256"] !=
              json.load(open(os.path.join(F64, n + ".json")))["tri96_sha256"]]
    assert len(differ) >= 6, differ


def test_f64_fixtures_cover_the_paths():
    assert {"dragon_1080", "bunny_97x61_primary", "dragon_orbit3_333x217", "tri1", "degenerate"} <= set(NAMES)
