"""GPU parity in the reference CMake build's arithmetic (CERES_MODE_FMA + CERES_ARITH_FMA).

The reference builds with g++ -O3 -mavx2 -mfma (CMakeLists.txt:11-13), where GCC contracts
a*b+c into FMA at the sites its optimiser picks; the image that build renders differs from the
contraction-free one (C5: thousands of bytes, many pixels beyond +-1 LSB).  The product's FMA
flavour puts an explicit fmaf at exactly those sites (oracle/contraction_sites.txt), in the
host scene preparation (ARITH_FMA) and in every kernel (MODE_FMA).  Bar: bit-identical to
_ref/ref_render -- PPM sha256 = the fixture's ppm_sha256.ref, rays/hits = meta["ref"], sampled
float pixels and hit records = <cfg>.ref.records.npz, on every fixture config including C5.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_names, load_golden, load_ref_records

import configs

pytestmark = pytest.mark.gpu

ALL = [n for n in golden_names() if n != "proc_c5"]
FMA = 1


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


_scenes = {}


def scene_for(pkg, name, stats=False):
    key = (name, stats)
    if key not in _scenes:
        mesh, bvh, cam = pkg.prepare(configs.CONFIGS[name], arith=FMA)
        _scenes[key] = (pkg.Scene(mesh, bvh, device=0, stats=stats), cam)
    return _scenes[key]


def _hexf(hx):
    return np.asarray([int(h, 16) for h in hx], np.uint32).view(np.float32)


def ref_basis(meta):
    """The reference-flag build's camera basis and pose, from the fixture's hex bits."""
    b = meta["ref_basis"]
    return np.concatenate([_hexf(meta["ref_pose"]["eye"]), _hexf(b["dir"] + b["u"] + b["v"])])


def ref_sun(meta):
    return _hexf(meta["ref_pose"]["sun"])


@pytest.mark.parametrize("name", ALL)
def test_fma_frame_matches_reference_build(gpu, name):
    pkg = gpu
    meta, _, ppm = load_golden(name)
    rec = load_ref_records(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, cam = scene_for(pkg, name)
    assert np.array_equal(cam.basis(W, H).view(np.uint32), ref_basis(meta).view(np.uint32))
    px, rgb, st = scene.render(ref_basis(meta), ref_sun(meta), W, H, mode=pkg.cfg_mode(cfg, FMA))
    assert (st["rays"], st["hits"]) == (meta["ref"]["rays"], meta["ref"]["hits"])
    body = pkg.ppm(W, H, rgb)
    assert hashlib.sha256(body).hexdigest() == meta["ppm_sha256"]["ref"]
    if "ref" in ppm:
        assert body == ppm["ref"]
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(px.reshape(-1, 3)[pix].view(np.uint32), rec["rgb"].view(np.uint32))


@pytest.mark.parametrize("name", ["bunny_640", "dragon_640", "proc_101", "bunny_97x61_primary", "tri1", "quad",
                                  "degenerate", "dragon_1080", "dragon_orbit3_333x217", "dupleaf",
                                  "dragon_333x217_robust"])
def test_fma_hit_records_match_reference_build(gpu, name):
    pkg = gpu
    meta, _, _ = load_golden(name)
    rec = load_ref_records(name)
    cfg = configs.CONFIGS[name]
    scene, _ = scene_for(pkg, name)
    prim, tuv, sh, _ = scene.records(ref_basis(meta), ref_sun(meta), cfg["W"], cfg["H"], mode=pkg.cfg_mode(cfg, FMA))
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(prim[pix], rec["prim"])
    np.testing.assert_array_equal(sh[pix], rec["shadow"])
    hit = rec["prim"] >= 0
    for k, key in enumerate(("t", "u", "v")):
        np.testing.assert_array_equal(tuv[pix][hit, k].view(np.uint32), rec[key][hit].view(np.uint32))


@pytest.mark.parametrize("name", ["dragon_640", "bunny_640", "proc_101"])
def test_fma_full_float_image_matches_oracle(gpu, oracle_mod, name):
    """Every float of the frame equals the oracle's contract=True restatement."""
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _ = scene_for(pkg, name)
    basis = ref_basis(meta)
    px, rgb, _ = scene.render(basis, ref_sun(meta), W, H, mode=pkg.cfg_mode(cfg, FMA))
    sc = oracle_mod.prepare(cfg, contract=True)
    r = oracle_mod.render(sc, cfg, basis=basis[3:], eye=basis[:3], sun=ref_sun(meta))
    np.testing.assert_array_equal(px.view(np.uint32), r["pixels"].view(np.uint32))
    np.testing.assert_array_equal(rgb, r["ppm"])


@pytest.mark.parametrize("name", ["dragon_640", "bunny_1080_primary", "dragon_333x217_robust"])
def test_fma_traversal_statistics_match_reference_build(gpu, name):
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    scene, _ = scene_for(pkg, name, stats=True)
    mode = pkg.cfg_mode(cfg, FMA)
    _, _, st = scene.render(ref_basis(meta), ref_sun(meta), cfg["W"], cfg["H"], mode=mode, want_pixels=False)
    ref = meta["ref"]
    if cfg["mode"] == "primary":
        assert (st["node_pairs"], st["tri_tests"]) == (ref["primary_pairs"], ref["primary_tests"])
    else:
        assert ref["primary_pairs"] <= st["node_pairs"] <= ref["primary_pairs"] + ref["shadow_pairs"]
        assert ref["primary_tests"] <= st["tri_tests"] <= ref["primary_tests"] + ref["shadow_tests"]


@pytest.mark.parametrize("name", ALL)
def test_fma_batch_kernel_frame_matches_reference_build(gpu, name):
    """The multi-frame kernel (shadow packets, octant loops) in the FMA flavour: 3 copies of the
    fixture view, each = the reference-flag build's PPM."""
    import torch
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _ = scene_for(pkg, name)
    b12 = np.repeat(ref_basis(meta)[None, :], 3, 0).astype(np.float32)
    s3 = np.repeat(ref_sun(meta)[None, :], 3, 0)
    rgb = torch.zeros((3, H, 3 * W), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    scene.render_batch_device(b12, s3, W, H, mode=pkg.cfg_mode(cfg, FMA), d_rgb8=rgb.data_ptr(),
                              d_counters=cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    assert (int(c[0]), int(c[1])) == (3 * meta["ref"]["rays"], 3 * meta["ref"]["hits"])
    assert int(c[6]) == 0
    head = b"P6 %d %d 255\n" % (W, H)
    for f in range(3):
        assert hashlib.sha256(head + rgb[f].cpu().numpy().tobytes()).hexdigest() == meta["ppm_sha256"]["ref"], f


def test_fma_c5_matches_reference_build(gpu):
    """C5 (10M triangles, 3840x2160) -- where the contraction-free image is furthest from the
    reference-flag build's -- in the FMA flavour: PPM, counts and sampled pixels of _ref/ref_render,
    as one whole-frame device launch and through the host-buffer call."""
    import torch
    pkg = gpu
    if not os.path.exists(os.path.join(GOLDEN, "proc_c5.ref.records.npz")):
        pytest.skip("C5 fixture not generated")
    meta, _, _ = load_golden("proc_c5")
    rec = load_ref_records("proc_c5")
    cfg = configs.CONFIGS["proc_c5"]
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, _ = pkg.prepare(cfg, arith=FMA)
    scene = pkg.Scene(mesh, bvh)
    del mesh, bvh
    try:
        mode = pkg.cfg_mode(cfg, FMA)
        px, rgb, st = scene.render(ref_basis(meta), ref_sun(meta), W, H, mode=mode)
        assert (st["rays"], st["hits"]) == (meta["ref"]["rays"], meta["ref"]["hits"])
        assert hashlib.sha256(pkg.ppm(W, H, rgb)).hexdigest() == meta["ppm_sha256"]["ref"]
        pix = rec["pixel"].astype(np.int64)
        np.testing.assert_array_equal(px.reshape(-1, 3)[pix].view(np.uint32), rec["rgb"].view(np.uint32))
        d = torch.empty(3 * W * H, dtype=torch.uint8, device="cuda")
        c = torch.zeros(8, dtype=torch.int64, device="cuda")
        scene.render_device(ref_basis(meta), ref_sun(meta), W, H, mode=mode, d_rgb8=d.data_ptr(),
                            d_counters=c.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert hashlib.sha256(pkg.ppm(W, H, d.cpu().numpy())).hexdigest() == meta["ppm_sha256"]["ref"]
    finally:
        scene.close()


def test_exact_and_fma_flavours_differ_where_the_builds_differ(gpu):
    """Control: on a config where the two reference builds disagree, the two product flavours
    disagree the same way (the FMA flag really selects different arithmetic)."""
    pkg = gpu
    name = "bunny_640"
    meta, _, ppm = load_golden(name)
    assert meta["ppm_sha256"]["ref"] != meta["ppm_sha256"]["exact"]
    cfg = configs.CONFIGS[name]
    scene, _ = scene_for(pkg, name)
    _, rgb_f, _ = scene.render(ref_basis(meta), ref_sun(meta), cfg["W"], cfg["H"], mode=pkg.cfg_mode(cfg, FMA),
                               want_pixels=False)
    _, rgb_e, _ = scene.render(ref_basis(meta), ref_sun(meta), cfg["W"], cfg["H"], mode=pkg.cfg_mode(cfg),
                               want_pixels=False)
    assert not np.array_equal(rgb_f, rgb_e)
    assert pkg.ppm(cfg["W"], cfg["H"], rgb_f) == ppm["ref"]
