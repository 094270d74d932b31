"""Product host-side scene preparation (libceres_hip.so, C++) against the reference fixtures.

The OBJ loader, rotate_triangles, camera basis and binned-SAH builder of the product must
produce exactly the bits the reference produces (they feed the GPU kernels): checked here on
CPU without touching a GPU -- in both arithmetics: ARITH_EXACT against the contraction-free
reference build, ARITH_FMA against the reference's own CMake build (the "ref*" fixture keys).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_names, hexbits, load_golden, ref_scene_hashes

import configs

NAMES = [n for n in golden_names() if n != "proc_c5"]


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
@pytest.mark.parametrize("name", NAMES)
def test_product_scene_prep_matches_reference(pkg, name, arith):
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    tri, nor, canon = ref_scene_hashes(meta, arith)
    assert len(mesh) == meta["n_tri"]
    assert hashlib.sha256(mesh.tri.tobytes()).hexdigest() == tri
    assert hashlib.sha256(mesh.norm.tobytes()).hexdigest() == nor
    import make_golden
    assert make_golden.canonical_bvh_sha(bvh.nodes.tobytes(), bvh.prim.tobytes()) == canon
    assert bvh.nodes.shape[0] == meta["ref_n_nodes" if arith else "n_nodes"]
    b = cam.basis(cfg["W"], cfg["H"])
    pose, basis = (meta["ref_pose"], meta["ref_basis"]) if arith else (meta["pose"], meta["basis"])
    assert hexbits(b[:3]) == pose["eye"]
    assert hexbits(b[3:]) == basis["dir"] + basis["u"] + basis["v"]
    assert hexbits(pkg.pose(cfg, arith=arith)[1]) == pose["sun"]


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
@pytest.mark.parametrize("name", ["dragon_orbit3_333x217", "bunny_orbit7_160x120"])
def test_orbit_frames_match_reference_transform(pkg, oracle_mod, name, arith):
    """anim.cpp orbit (transform.hpp): the product's multi-frame orbit equals the reference pose
    pinned by the fixture at frame `count`, and the oracle's restatement at every frame."""
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    (axis, step, count) = cfg["orbit"]
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"], arith=arith)
    n = count + 4
    b, s3 = pkg.orbit_cameras(cam0, cfg["sun"], cfg["W"], cfg["H"], n, axis=axis, step_deg=step, rotate_first=False)
    pose, basis = (meta["ref_pose"], meta["ref_basis"]) if arith else (meta["pose"], meta["basis"])
    assert hexbits(b[count, :3]) == pose["eye"]
    assert hexbits(b[count, 3:]) == basis["dir"] + basis["u"] + basis["v"]
    assert hexbits(s3[count]) == pose["sun"]
    for k in range(n):
        e, d, s = oracle_mod.orbit(axis, step, k, cfg["eye"], cfg["dir"], cfg["sun"], contract=arith)
        assert hexbits(b[k, :3]) == hexbits(e) and hexbits(s3[k]) == hexbits(s)
        assert hexbits(b[k, 3:]) == hexbits(oracle_mod.camera_basis(e, d, cfg["up"], cfg["fov"], cfg["W"], cfg["H"],
                                                                    contract=arith))
    # rotate_first (anim.cpp's own order) is the same sequence shifted by one frame
    b1, s1 = pkg.orbit_cameras(cam0, cfg["sun"], cfg["W"], cfg["H"], n - 1, axis=axis, step_deg=step)
    np.testing.assert_array_equal(b1.view(np.uint32), b[1:].view(np.uint32))
    np.testing.assert_array_equal(s1.view(np.uint32), s3[1:].view(np.uint32))


def test_product_matches_oracle_on_c5_mesh(pkg, oracle_mod):
    """C5 procedural mesh generation + normals: product == oracle (== reference loader, pinned above)."""
    m = pkg.proc_mesh(301)
    t, n = oracle_mod.load_mesh(None, proc=301)
    np.testing.assert_array_equal(m.tri.view(np.uint32), t.view(np.uint32))
    np.testing.assert_array_equal(m.norm.view(np.uint32), n.view(np.uint32))
    b = pkg.build_bvh(m)
    nodes, prim = oracle_mod.build_bvh(t)
    import make_golden
    assert make_golden.canonical_bvh_sha(b.nodes.tobytes(), b.prim.tobytes()) == \
        make_golden.canonical_bvh_sha(nodes.tobytes(), prim.tobytes())


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
def test_product_c5_scene_matches_reference(pkg, oracle_mod, arith):
    """Full C5 (9,999,392 triangles): rotated triangles, normals and the binned-SAH BVH of the
    product's host path equal the reference's dump (tests/golden/proc_c5.json scene hashes)."""
    meta, _, _ = load_golden("proc_c5")
    mesh, bvh, _ = pkg.prepare(configs.CONFIGS["proc_c5"], arith=arith)
    tri, nor, canon = ref_scene_hashes(meta, arith)
    assert len(mesh) == meta["n_tri"] and bvh.nodes.shape[0] == meta["ref_n_nodes" if arith else "n_nodes"]
    assert hashlib.sha256(mesh.tri.tobytes()).hexdigest() == tri
    assert hashlib.sha256(mesh.norm.tobytes()).hexdigest() == nor
    assert oracle_mod.canonical_bvh_sha(bvh.nodes, bvh.prim) == canon


def test_oracle_canonical_hash_equals_python_definition(pkg, oracle_mod):
    import make_golden
    mesh, bvh, _ = pkg.prepare(configs.CONFIGS["dragon_1080"])
    assert oracle_mod.canonical_bvh_sha(bvh.nodes, bvh.prim) == \
        make_golden.canonical_bvh_sha(bvh.nodes.tobytes(), bvh.prim.tobytes())


def test_obj_edge_cases(pkg, tmp_path):
    # unreadable file -> empty scene, like obj_norms.hpp:123-126
    m = pkg.load_obj(str(tmp_path / "missing.obj"))
    assert len(m) == 0
    # bad index (obj_norms.hpp:90 assert) -> loud error
    p = tmp_path / "bad.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n")
    with pytest.raises(pkg.CeresError):
        pkg.load_obj(str(p))
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n")
    with pytest.raises(pkg.CeresError):
        pkg.load_obj(str(p))
    # empty scene cannot be built (static.cpp:77-80)
    with pytest.raises(pkg.CeresError):
        pkg.build_bvh(pkg.Mesh(np.zeros((0, 12), np.float32), np.zeros((0, 9), np.float32)))
    # comments, blank lines, CRLF, polygon fan, relative indices
    p.write_text("# c\r\n\r\nv 0 0 0\r\nv 1 0 0\r\nv 1 1 0\r\nv 0 1 0\r\nf 1 2 3 4\r\nf -4 -3 -2\r\n")
    m = pkg.load_obj(str(p))
    assert len(m) == 3


def test_obj_long_line_stops_reading(pkg, oracle_mod, tmp_path):
    """A line of >= 1024 chars makes istream::getline fail: the reference stops reading there."""
    p = tmp_path / "long.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n# " + "x" * 1100 + "\nf 1 3 2\n")
    m = pkg.load_obj(str(p))
    t, _ = oracle_mod.load_mesh(str(p))
    assert len(m) == 1 == t.shape[0]
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n# " + "x" * 1021 + "\nf 1 3 2\n")   # 1023 chars: fine
    assert len(pkg.load_obj(str(p))) == 2 == oracle_mod.load_mesh(str(p))[0].shape[0]


def test_golden_tiny_meshes_exist():
    for f in ("tri1.obj", "quad.obj", "degenerate.obj"):
        assert os.path.exists(os.path.join(GOLDEN, f))


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
@pytest.mark.parametrize("name", ["bunny_640", "dragon_1080", "bunny_1080", "bunny_1080_primary", "dragon_4096", "proc_c5"])
def test_bench_views_are_the_pinned_reference_poses(pkg, name, arith):
    """Every view bench.py can time at N = 1, 2, 4, 8 (pkg.bench_views, F = 16N) is pinned in
    tests/golden/orbit/<cfg>.json for both reference builds, with its traversal statistics, and
    the host's orbit pose (ceres_orbit_cameras, eye and sun) equals the reference Transform's bits
    for it in that build's arithmetic (anim.cpp:76-88, transform.hpp:67-112)."""
    from conftest import load_orbit
    fx = load_orbit(name)
    by = fx["by_step_bits"]
    assert len(by) == fx["views"] == pkg.configs.ORBIT_FIXTURE_VIEWS
    cfg = pkg.configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    build = "ref" if arith else "exact"
    view = (lambda e: e["ref"]) if arith else (lambda e: e)
    cam = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"], arith=arith)
    v0 = view([e for e in by.values() if e["k"] == 0][0])
    assert v0["sha256"] == meta["ppm_sha256"][build] and v0["rays"] == meta[build]["rays"]
    for k in ("primary_pairs", "primary_tests", "shadow_pairs", "shadow_tests"):
        assert v0["stats"][k] == meta[build][k]
    for n in (1, 2, 4, 8):
        F = 16 * n
        b12, s3, steps = pkg.bench_views(cam, cfg["sun"], cfg["W"], cfg["H"], F)
        for f in range(F):
            e0 = by["%08x" % int(np.asarray(steps[f], np.float32).view(np.uint32))]
            e = view(e0)
            assert e0["k"] == f * 128 // F
            assert e["stats"]["loop_vs_render_mismatch"] == 0 and e["stats"]["primary_pairs"] > 0
            if f:
                assert hexbits(b12[f, :3]) == e["eye"], (n, f)
                assert hexbits(s3[f]) == e["sun"], (n, f)
