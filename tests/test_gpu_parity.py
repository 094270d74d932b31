"""GPU parity: the gfx950 kernels (through the C ABI) against the reference fixtures and oracle.

Bar (BASELINE.json north star): the PPM equals the contraction-free reference
render byte for byte (and stays within +-1 LSB / 1e-5-pixel budget of the reference-flag
build); ray/hit counts equal the reference's; float pixels and hit records {prim, t, u, v,
shadow} are bit-identical to the oracle (the north star's "hit-t within 1e-5 rel" is met with
0 ulp); at full sizes the same holds by PPM sha256.  Also: row tilings (multi-GPU layout)
reassemble the single-GPU frame exactly, traversal statistics match the reference's counters,
and the drop-in render.hpp / ./render CLI produce the same bytes.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO, golden_names, hexbits, load_golden, load_ref_records, ppm_budget_ok

import configs

pytestmark = pytest.mark.gpu

ALL = [n for n in golden_names() if n != "proc_c5"]


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
        cfg = configs.CONFIGS[name]
        mesh, bvh, cam = pkg.prepare(cfg)
        _scenes[key] = (pkg.Scene(mesh, bvh, device=0, stats=stats), cam, mesh, bvh)
    return _scenes[key]


def _hexf(hx):
    return np.asarray([int(h, 16) for h in hx], np.uint32).view(np.float32)


def pinned_basis(meta, cfg):
    """Camera basis from the fixture's hex bits (never trust the box's libm)."""
    eye = _hexf(meta["pose"]["eye"]) if "pose" in meta else np.asarray(cfg["eye"], np.float32)
    return np.concatenate([eye, _hexf(meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"])])


def pinned_sun(meta, cfg):
    return _hexf(meta["pose"]["sun"]) if "pose" in meta else np.asarray(cfg["sun"], np.float32)


@pytest.mark.parametrize("name", ALL)
def test_frame_matches_reference(gpu, name):
    pkg = gpu
    meta, rec, ppm = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, cam, _, _ = scene_for(pkg, name)
    basis = pinned_basis(meta, cfg)
    if hexbits(cam.basis(W, H)) != hexbits(basis):
        import warnings
        warnings.warn("host libm camera basis differs from the fixture; rendering with the pinned basis")
    mode = pkg.cfg_mode(cfg)
    px, rgb, st = scene.render(basis, pinned_sun(meta, cfg), W, H, mode=mode)
    assert (st["rays"], st["hits"]) == (meta["exact"]["rays"], meta["exact"]["hits"])
    body = pkg.ppm(W, H, rgb)
    assert hashlib.sha256(body).hexdigest() == meta["ppm_sha256"]["exact"]
    if "ref" in ppm:
        ok, bad = ppm_budget_ok(body, ppm["ref"], W, H)
        assert ok, f"{bad} pixels beyond +-1 LSB vs the reference-flag build"
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(px.reshape(-1, 3)[pix].view(np.uint32), rec["rgb"].view(np.uint32))


@pytest.mark.parametrize("name", ["bunny_640", "dragon_640", "proc_101", "dragon_333x217", "bunny_97x61_primary",
                                  "tri1", "quad", "degenerate", "dragon_1080", "dragon_orbit3_333x217", "dupleaf"])
def test_hit_records_match_reference(gpu, name):
    """prim / t / u / v / shadow per pixel, bit-exact vs the reference records (all pixels when small)."""
    pkg = gpu
    meta, rec, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    mode = pkg.cfg_mode(cfg)
    prim, tuv, sh, st = scene.records(pinned_basis(meta, cfg), pinned_sun(meta, cfg), W, H, mode=mode)
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(prim[pix], rec["prim"])
    np.testing.assert_array_equal(sh[pix], rec["shadow"])
    hit = rec["prim"] >= 0
    for k, key in enumerate(("t", "u", "v")):
        np.testing.assert_array_equal(tuv[pix][hit, k].view(np.uint32), rec[key][hit].view(np.uint32))


@pytest.mark.parametrize("name", ["dragon_640", "bunny_640", "proc_101"])
def test_full_float_image_matches_oracle(gpu, oracle_mod, name):
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    basis = pinned_basis(meta, cfg)
    px, rgb, _ = scene.render(basis, cfg["sun"], W, H)
    sc = oracle_mod.prepare(cfg)
    r = oracle_mod.render(sc, cfg, basis=basis[3:])
    np.testing.assert_array_equal(px.view(np.uint32), r["pixels"].view(np.uint32))
    np.testing.assert_array_equal(rgb, r["ppm"])


@pytest.mark.parametrize("name", ["dragon_640", "bunny_1080_primary"])
def test_traversal_statistics_match_reference(gpu, name):
    """Device counters vs single_ray_traverser.hpp Statistics: primary rays exactly; shadow rays
    use any-hit, so they visit at most the reference's closest-hit counts."""
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    scene, _, _, _ = scene_for(pkg, name, stats=True)
    mode = pkg.cfg_mode(cfg)
    _, _, st = scene.render(pinned_basis(meta, cfg), cfg["sun"], cfg["W"], cfg["H"], mode=mode, want_pixels=False)
    ex = meta["exact"]
    if mode == pkg.MODE_PRIMARY:
        assert (st["node_pairs"], st["tri_tests"]) == (ex["primary_pairs"], ex["primary_tests"])
    else:
        assert ex["primary_pairs"] <= st["node_pairs"] <= ex["primary_pairs"] + ex["shadow_pairs"]
        assert ex["primary_tests"] <= st["tri_tests"] <= ex["primary_tests"] + ex["shadow_tests"]


@pytest.mark.parametrize("world,row_block", [(2, 16), (3, 5), (8, 16)])
def test_row_tiling_reassembles_frame(gpu, world, row_block):
    """The multi-GPU row partition rendered rank by rank on one device == the single-GPU frame."""
    import torch
    pkg = gpu
    import ceres_raytracer_amd.distributed as D
    name = "dragon_640"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    basis = pinned_basis(meta, cfg)
    src, maxrows = D.ppm_row_permutation(H, row_block, world)
    bufs = []
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    rays = hits = 0
    for r in range(world):
        t = pkg.Tiling(row_block, r, world)
        buf = torch.zeros((maxrows, 3 * W), dtype=torch.uint8, device="cuda")
        scene.render_device(basis, cfg["sun"], W, H, tiling=t, d_rgb8=buf.data_ptr(), d_counters=counters.data_ptr(),
                            stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        c = counters.cpu().numpy()
        rays += int(c[0]); hits += int(c[1])
        bufs.append(buf)
    full = torch.cat(bufs)[torch.as_tensor(src, device="cuda")].cpu().numpy()
    body = pkg.ppm(W, H, full)
    assert hashlib.sha256(body).hexdigest() == meta["ppm_sha256"]["exact"]
    assert (rays, hits) == (meta["exact"]["rays"], meta["exact"]["hits"])


def _oracle_frame(oracle_mod, sc, cfg, basis12, sun3):
    return oracle_mod.render(sc, cfg, basis=basis12[3:], eye=basis12[:3], sun=sun3, want_pixels=False)


@pytest.mark.parametrize("world,row_block,frames", [(1, 1080, 4), (3, 16, 3), (2, 5, 5)])
def test_batch_orbit_frames_match_oracle(gpu, oracle_mod, world, row_block, frames):
    """ceres_render_batch_device: F orbit frames (configs.BENCH_ORBIT, the bench's weak-scaling
    batch) in one launch pair, each rank's rows of each frame, == per-frame oracle renders; frame
    3 is the dragon_orbit3 fixture pose (reference Transform) and must match its PPM sha."""
    import torch
    pkg = gpu
    import ceres_raytracer_amd.distributed as D
    name = "dragon_333x217"
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"])
    axis, step = configs.BENCH_ORBIT
    b12, s3 = pkg.orbit_cameras(cam0, cfg["sun"], W, H, frames, axis=axis, step_deg=step, rotate_first=False)
    src, maxrows = D.ppm_row_permutation(H, row_block, world)
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    per_rank = []
    rays = hits = 0
    for r in range(world):
        t = pkg.Tiling(row_block, r, world)
        rows = pkg.local_rows(H, t)
        buf = torch.zeros((frames, maxrows, 3 * W), dtype=torch.uint8, device="cuda")
        tight = torch.zeros((frames * rows * 3 * W,), dtype=torch.uint8, device="cuda")
        scene.render_batch_device(b12, s3, W, H, tiling=t, d_rgb8=tight.data_ptr(), d_counters=counters.data_ptr(),
                                  stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        buf[:, :rows] = tight.view(frames, rows, 3 * W)
        c = counters.cpu().numpy()
        rays += int(c[0]); hits += int(c[1])
        per_rank.append(buf)
    idx = torch.as_tensor(src, device="cuda")
    sc = oracle_mod.prepare(cfg)
    o_rays = o_hits = 0
    for f in range(frames):
        full = torch.cat([b[f] for b in per_rank])[idx].cpu().numpy().reshape(-1)
        o = _oracle_frame(oracle_mod, sc, cfg, b12[f], s3[f])
        o_rays += o["rays"]; o_hits += o["hits"]
        np.testing.assert_array_equal(full, o["ppm"], err_msg=f"frame {f}")
        if f == 3:
            meta, _, _ = load_golden("dragon_orbit3_333x217")
            assert hashlib.sha256(pkg.ppm(W, H, full)).hexdigest() == meta["ppm_sha256"]["exact"]
    assert (rays, hits) == (o_rays, o_hits)


def test_batch_float_pixels_match_single_frames(gpu):
    """Batch float framebuffer == single-frame ceres_render_f32 per frame, bit for bit."""
    import torch
    pkg = gpu
    name = "dragon_640"
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"])
    b12, s3 = pkg.orbit_cameras(cam0, cfg["sun"], W, H, 8, axis=configs.BENCH_ORBIT[0],
                                step_deg=configs.BENCH_ORBIT[1], rotate_first=False)
    px = torch.zeros((8, H, W, 3), dtype=torch.float32, device="cuda")
    scene.render_batch_device(b12, s3, W, H, d_pixels=px.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = px.cpu().numpy()
    for f in range(8):
        ref, _, _ = scene.render(b12[f], s3[f], W, H, want_rgb8=False)
        np.testing.assert_array_equal(got[f].reshape(-1).view(np.uint32), ref.view(np.uint32), err_msg=f"frame {f}")


@pytest.mark.parametrize("W,H,row_block,world,frames", [(64, 48, 16, 3, 2), (333, 217, 7, 3, 3), (1920, 1080, 8, 8, 8),
                                                        (16, 5, 16, 4, 1)])
def test_assemble_kernel_matches_permutation(gpu, W, H, row_block, world, frames):
    """ceres_assemble_rgb8 (16-B vector and byte paths) == the host permutation of distributed.py."""
    import torch
    pkg = gpu
    import ceres_raytracer_amd.distributed as D
    src, maxrows = D.batch_row_permutation(H, row_block, world, frames)
    g = torch.randint(0, 256, (world, frames * maxrows, 3 * W), dtype=torch.uint8, device="cuda")
    out = torch.zeros((frames, H, 3 * W), dtype=torch.uint8, device="cuda")
    pkg.assemble_rgb8(g.data_ptr(), g[0].numel(), out.data_ptr(), frames, W, H, row_block, world,
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = g.view(-1, 3 * W)[torch.as_tensor(src, device="cuda")].view(frames, H, 3 * W)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("W,H,row_block,world,frames", [(64, 48, 16, 3, 2), (333, 217, 7, 3, 1), (1920, 1080, 8, 8, 1),
                                                        (97, 61, 3, 5, 1)])
def test_assemble_packed_kernel_matches_permutation(gpu, W, H, row_block, world, frames):
    """ceres_assemble_rgb8_packed (the all-to-all receive layout, no padding) == the host
    permutation of distributed.py."""
    import torch
    pkg = gpu
    import ceres_raytracer_amd.distributed as D
    src = D.packed_row_permutation(H, row_block, world, frames)
    g = torch.randint(0, 256, (frames * H, 3 * W), dtype=torch.uint8, device="cuda")
    out = torch.zeros((frames, H, 3 * W), dtype=torch.uint8, device="cuda")
    pkg.assemble_rgb8_packed(g.data_ptr(), out.data_ptr(), frames, W, H, row_block, world,
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = g[torch.as_tensor(src, device="cuda")].view(frames, H, 3 * W)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("name", ALL)
def test_batch_kernel_frame_matches_reference(gpu, name):
    """The multi-frame kernel on every fixture (edge cases included: one triangle, root leaf,
    degenerate and duplicated-leaf meshes, odd sizes, robust mode): a 3-frame batch of the fixture
    view -- the batch kernel traces a tile's shadow rays as one wave-wide packet when its rays
    share an octant (packet_any4), else one ray per lane -- gives the reference's PPM for every
    frame and 3x its rays / hits."""
    import torch
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    b12 = np.repeat(pinned_basis(meta, cfg)[None, :], 3, 0).astype(np.float32)
    s3 = np.repeat(np.asarray(pinned_sun(meta, cfg), np.float32)[None, :], 3, 0)
    rgb = torch.zeros((3, H, 3 * W), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    scene.render_batch_device(b12, s3, W, H, mode=pkg.cfg_mode(cfg), d_rgb8=rgb.data_ptr(), d_counters=cnt.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    assert (int(c[0]), int(c[1])) == (3 * meta["exact"]["rays"], 3 * meta["exact"]["hits"])
    assert int(c[6]) == 0
    head = b"P6 %d %d 255\n" % (W, H)
    for f in range(3):
        assert hashlib.sha256(head + rgb[f].cpu().numpy().tobytes()).hexdigest() == meta["ppm_sha256"]["exact"], f


def test_batch_of_64_frames_matches_single_frames(gpu):
    """The largest batch (64 frames, cameras inline in the kernel arguments): every frame's PPM
    body == a one-frame render of the same camera, whole frames and one rank of a 3-way split."""
    import torch
    pkg = gpu
    name = "dragon_333x217"
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    scene, _, _, _ = scene_for(pkg, name)
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"])
    b12, s3 = pkg.orbit_cameras(cam0, cfg["sun"], W, H, 64, axis=configs.BENCH_ORBIT[0], step_deg=5.625,
                                rotate_first=False)
    st = torch.cuda.current_stream().cuda_stream
    for til in (pkg.Tiling(H, 0, 1), pkg.Tiling(8, 2, 3)):
        rows = pkg.local_rows(H, til)
        rgb = torch.zeros((64, rows, 3 * W), dtype=torch.uint8, device="cuda")
        scene.render_batch_device(b12, s3, W, H, tiling=til, d_rgb8=rgb.data_ptr(), stream=st)
        one = torch.zeros((rows, 3 * W), dtype=torch.uint8, device="cuda")
        for f in (0, 1, 31, 32, 33, 62, 63):
            scene.render_device(b12[f], s3[f], W, H, tiling=til, d_rgb8=one.data_ptr(), stream=st)
            torch.cuda.synchronize()
            assert torch.equal(rgb[f], one), f"frame {f}, tiling {til}"


def test_large_frame_batch_matches_single_frames(gpu):
    """Frames of >= 1 Mpixel are dealt frame after frame in a batch (CERES_FRAME_MAJOR_PIXELS)
    instead of interleaved: every frame's PPM body == a one-frame render, whole frames and one
    rank of a 3-way row split."""
    import torch
    pkg = gpu
    name = "dragon_640"
    cfg = configs.CONFIGS[name]
    W, H = 2048, 2048
    scene, _, _, _ = scene_for(pkg, name)
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"])
    b12, s3 = pkg.orbit_cameras(cam0, cfg["sun"], W, H, 3, axis=configs.BENCH_ORBIT[0], step_deg=20.0,
                                rotate_first=False)
    st = torch.cuda.current_stream().cuda_stream
    for til in (pkg.Tiling(H, 0, 1), pkg.Tiling(8, 1, 3)):
        rows = pkg.local_rows(H, til)
        rgb = torch.zeros((3, rows, 3 * W), dtype=torch.uint8, device="cuda")
        scene.render_batch_device(b12, s3, W, H, tiling=til, d_rgb8=rgb.data_ptr(), stream=st)
        one = torch.zeros((rows, 3 * W), dtype=torch.uint8, device="cuda")
        for f in range(3):
            scene.render_device(b12[f], s3[f], W, H, tiling=til, d_rgb8=one.data_ptr(), stream=st)
            torch.cuda.synchronize()
            assert torch.equal(rgb[f], one), f"frame {f}, tiling {til}"
        assert int(rgb.max()) > 0


def test_batch_rejects_bad_frame_counts(gpu):
    pkg = gpu
    scene, _, _, _ = scene_for(pkg, "tri1")
    with pytest.raises(pkg.CeresError):
        scene.render_batch_device(np.zeros((65, 12), np.float32), np.zeros((65, 3), np.float32), 8, 8)
    with pytest.raises(pkg.CeresError):
        scene.render_batch_device(np.zeros((2, 12), np.float32), np.zeros((3, 3), np.float32), 8, 8)


# ./render's arithmetic: default (--fma) = the reference's CMake build, --exact = -ffp-contract=off
CLI_ARITH = {"ref": [], "exact": ["--exact"]}


@pytest.mark.parametrize("build", ["ref", "exact"])
def test_cli_orbit_frames(gpu, tmp_path, build):
    """./render --orbit ... --frames 2 writes the anim.cpp orbit frames; frame 0 = fixture pose."""
    pkg = gpu
    name = "dragon_orbit3_333x217"
    meta, _, ppm = load_golden(name)
    out = tmp_path / "orbit.ppm"
    args = configs.cli_args(configs.CONFIGS[name]) + CLI_ARITH[build]
    r = subprocess.run([pkg.CLI_PATH] + args + ["--frames", "2", "-o", str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "orbit_000.ppm").read_bytes() == ppm[build]
    assert (tmp_path / "orbit_001.ppm").exists()
    assert "Total Rays:" in r.stdout


def test_fast_reciprocal_is_exact(gpu):
    """rcp_exact() (render_hip.hip) == IEEE 1/x for all normal |x| in [2^-126, 2^126): exhaustive
    over every float bit pattern on this gfx950 (the kernels fall back to the division elsewhere)."""
    exe = os.path.join(REPO, "tools", "probes", "rcp_exhaustive")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "exact for biased exponents [1, 252]" in r.stdout, r.stdout


def test_repeat_renders_are_deterministic(gpu):
    pkg = gpu
    meta, _, _ = load_golden("dragon_1080")
    cfg = configs.CONFIGS["dragon_1080"]
    scene, _, _, _ = scene_for(pkg, "dragon_1080")
    outs = [scene.render(pinned_basis(meta, cfg), cfg["sun"], 1920, 1080, want_pixels=False)[1] for _ in range(3)]
    assert all(np.array_equal(outs[0], o) for o in outs[1:])


def test_c5_procedural_10m_triangles(gpu):
    """C5: 9,999,392 triangles at 3840x2160 (1.26 GB scene, HBM-resident): counts + PPM sha."""
    pkg = gpu
    if not os.path.exists(os.path.join(GOLDEN, "proc_c5.json")):
        pytest.skip("C5 fixture not generated")
    meta, rec, _ = load_golden("proc_c5")
    cfg = configs.CONFIGS["proc_c5"]
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh)
    del mesh, bvh
    px, rgb, st = scene.render(pinned_basis(meta, cfg), cfg["sun"], cfg["W"], cfg["H"])
    assert (st["rays"], st["hits"]) == (meta["exact"]["rays"], meta["exact"]["hits"])
    assert hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"]["exact"]
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(px.reshape(-1, 3)[pix].view(np.uint32), rec["rgb"].view(np.uint32))
    scene.close()


def test_c5_single_launch_xcd_local_order(gpu):
    """C5 as ONE whole-frame launch (ceres_render_device, the launch bench.py's roofline times): a
    DRAM-resident scene's large frame takes the XCD-local Morton tile order (ensure_tile_order);
    the PPM and the counts still equal the reference's."""
    import torch
    pkg = gpu
    meta, _, _ = load_golden("proc_c5")
    cfg = configs.CONFIGS["proc_c5"]
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh)
    del mesh, bvh
    assert scene.info()["device_bytes"] >= 64 << 20          # kDramSceneBytes: the local order applies
    rgb = torch.empty(3 * W * H, dtype=torch.uint8, device="cuda")
    c = torch.zeros(8, dtype=torch.int64, device="cuda")
    scene.render_device(pinned_basis(meta, cfg), cfg["sun"], W, H, d_rgb8=rgb.data_ptr(), d_counters=c.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = c.cpu().numpy()
    assert (int(c[0]), int(c[1])) == (meta["exact"]["rays"], meta["exact"]["hits"]) and c[6] == 0
    assert hashlib.sha256(pkg.ppm(W, H, rgb.cpu().numpy())).hexdigest() == meta["ppm_sha256"]["exact"]
    scene.close()


@pytest.mark.parametrize("gpu_bvh,build", [(False, "ref"), (False, "exact"), (True, "exact")])
def test_cli_writes_reference_ppm(gpu, tmp_path, gpu_bvh, build):
    """static.cpp's sequence: the default writes the reference CMake build's PPM byte for byte,
    --exact the contraction-free build's (bunny 640x480 is where they differ most: 20 bytes)."""
    pkg = gpu
    name = "bunny_640"
    meta, _, ppm = load_golden(name)
    out = tmp_path / "bunny.ppm"
    args = configs.cli_args(configs.CONFIGS[name]) + (["--gpu-bvh"] if gpu_bvh else []) + CLI_ARITH[build]
    r = subprocess.run([pkg.CLI_PATH] + args + ["-o", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Rays: %d\tHits: %d" % (meta[build]["rays"], meta[build]["hits"]) in r.stdout
    assert out.read_bytes() == ppm[build]


DROPIN_APP = r"""
#include <cstdio>
#include <vector>
#include "ceres/render.hpp"
// static.cpp's sequence (load :76, rotate :83-88, BVH :100-107, render :130) on the drop-in header,
// then the caller EDITS its arrays in place between two render() calls (render.hpp:86-156 reads
// them on every call): argv[3] = a triangle whose three vertex normals are flipped, argv[4] = a
// triangle whose p0 moves by 1e-3 along y.  Both float framebuffers go to argv[2].{0,1}.
int main(int argc, char** argv) {
    float* tri; float* nrm; size_t n;
    if (ceres_obj_load_arith(argv[1], &tri, &nrm, &n, CERES_DROPIN_ARITH)) return 3;
    rotate_triangles<0>(90.0f, reinterpret_cast<ceres::HostTriangle*>(tri), n);
    uint32_t* nodes; uint64_t* prim; size_t m;
    if (ceres_bvh_build_arith(tri, n, &nodes, &m, &prim, CERES_DROPIN_ARITH)) return 4;
    ceres::HostBvh bvh;
    bvh.nodes.reset(new ceres::HostBvh::Node[m]); std::memcpy(bvh.nodes.get(), nodes, 32 * m);
    bvh.primitive_indices.reset(new size_t[n]); std::memcpy(bvh.primitive_indices.get(), prim, 8 * n);
    bvh.node_count = m;
    Camera<float> cam{ceres::vec3<float>(0, -15, 2), ceres::vec3<float>(0, 1, 0), ceres::vec3<float>(0, 0, 1), 60};
    std::vector<float> px(3 * 333 * 217);
    auto* T = reinterpret_cast<ceres::HostTriangle*>(tri);
    auto* N = reinterpret_cast<std::array<ceres::vec3<float>, 3>*>(nrm);
    auto rh = render(cam, ceres::vec3<float>(-50, -20, 0), bvh, T, N, px.data(), 333, 217);
    std::string out = argv[2];
    if (FILE* f = std::fopen((out + ".0").c_str(), "wb")) { std::fwrite(px.data(), 4, px.size(), f); std::fclose(f); }
    const size_t a = std::strtoul(argv[3], nullptr, 10), b = std::strtoul(argv[4], nullptr, 10);
    for (int k = 0; k < 3; ++k) for (int c = 0; c < 3; ++c) N[a][k][c] = -N[a][k][c];
    T[b].p0[1] += 1e-3f;
    auto rh2 = render(cam, ceres::vec3<float>(-50, -20, 0), bvh, T, N, px.data(), 333, 217);
    if (FILE* f = std::fopen((out + ".1").c_str(), "wb")) { std::fwrite(px.data(), 4, px.size(), f); std::fclose(f); }
    std::printf("%d %d %d %d %d\n", rh.first, rh.second, rh2.first, rh2.second, int(CERES_DROPIN_ARITH));
    return 0;
}
"""


@pytest.mark.parametrize("arith", ["default", "exact"])
def test_dropin_render_hpp_per_call_contract(gpu, oracle_mod, tmp_path, arith):
    """A static.cpp-style program on include/ceres/render.hpp: render<float>()'s host float
    framebuffer equals the reference's (fixture records) and the oracle's bit for bit; after the
    caller edits one triangle's normals and another triangle's p0 IN PLACE (neither at a 4096th
    index), the next render() call sees the edited scene -- its framebuffer equals the oracle's
    render of the edited arrays.  Compiled with g++ -O2 -mfma (default: the reference CMake build's
    FMA arithmetic, CERES_DROPIN_ARITH) and with -DCERES_DROPIN_ARITH=CERES_ARITH_EXACT."""
    pkg = gpu
    name = "dragon_333x217"
    meta, rec, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    contract = arith == "default"
    # two visible lit triangles from the fixture's records, neither a multiple of 4096
    lit = rec["prim"][(rec["prim"] >= 0) & (rec["shadow"] == 0)]
    cand = [int(p) for p in np.unique(lit) if p % 4096 and p > 0]
    t_norm, t_move = cand[len(cand) // 3], cand[2 * len(cand) // 3]
    src = tmp_path / "app.cpp"
    src.write_text(DROPIN_APP)
    exe = tmp_path / "app"
    pkgdir = os.path.dirname(pkg.LIB_PATH)
    flags = ["-O2", "-mfma"] + ([] if contract else ["-DCERES_DROPIN_ARITH=CERES_ARITH_EXACT"])
    r = subprocess.run(["g++", "-std=c++17"] + flags + ["-I" + os.path.join(REPO, "include"), str(src), "-o", str(exe),
                        "-L" + pkgdir, "-lceres_hip", "-Wl,-rpath," + pkgdir], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    stem = str(tmp_path / "px")
    r = subprocess.run([str(exe), os.path.join(REPO, "data", "dragon.obj"), stem, str(t_norm), str(t_move)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rays, hits, rays2, hits2, ar = map(int, r.stdout.split())
    build = "ref" if contract else "exact"
    assert ar == (1 if contract else 0)
    assert (rays, hits) == (meta[build]["rays"], meta[build]["hits"])
    px0 = np.fromfile(stem + ".0", np.float32)
    px1 = np.fromfile(stem + ".1", np.float32)
    recb = load_ref_records(name) if contract else rec
    pix = recb["pixel"].astype(np.int64)
    np.testing.assert_array_equal(px0.reshape(-1, 3)[pix].view(np.uint32), recb["rgb"].view(np.uint32))
    sc = oracle_mod.prepare(cfg, contract=contract)
    o0 = oracle_mod.render(sc, cfg, want_ppm=False)
    np.testing.assert_array_equal(px0.view(np.uint32), o0["pixels"].view(np.uint32))
    sc["norm"][t_norm] = -sc["norm"][t_norm]
    sc["tri"][t_move, 1] += np.float32(1e-3)
    o1 = oracle_mod.render(sc, cfg, want_ppm=False)
    assert not np.array_equal(o0["pixels"], o1["pixels"])          # the edits are visible
    np.testing.assert_array_equal(px1.view(np.uint32), o1["pixels"].view(np.uint32))
    assert (rays2, hits2) == (o1["rays"], o1["hits"])


@pytest.mark.parametrize("world,row_block", [(1, 8), (2, 8), (3, 5), (5, 16)])
def test_render_multi_reassembles_frame(gpu, world, row_block):
    """ceres_render_multi_f32 (`./render --gpus N`): N rank scenes (all on device 0 here: the
    one-GPU box stands in for N devices; the peer copy is then device-local) render their row
    blocks, the RGB8 rows are gathered and assembled on the first device: PPM = the reference's,
    float pixels = the one-GPU render's, rays/hits = the fixture's."""
    pkg = gpu
    name = "dragon_333x217"
    meta, _, ppm = load_golden(name)
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = pkg.prepare(cfg)
    basis, sun = pinned_basis(meta, cfg), pinned_sun(meta, cfg)
    W, H = cfg["W"], cfg["H"]
    one = scene_for(pkg, name)[0]
    px1, rgb1, st1 = one.render(basis, sun, W, H)
    ranks = [pkg.Scene(mesh, bvh, device=0) for _ in range(world)]
    try:
        px, rgb, st = pkg.render_multi(ranks, basis, sun, W, H, row_block=row_block)
        assert pkg.ppm(W, H, rgb) == ppm["exact"]
        assert np.array_equal(px.view(np.uint32), px1.view(np.uint32))
        assert (st["rays"], st["hits"]) == (meta["exact"]["rays"], meta["exact"]["hits"]) == (st1["rays"], st1["hits"])
        # RGB8 only, primary-only mode
        _, rgbp, _ = pkg.render_multi(ranks, basis, sun, W, H, row_block=row_block, mode=pkg.MODE_PRIMARY,
                                      want_pixels=False)
        _, rgbp1, _ = one.render(basis, sun, W, H, mode=pkg.MODE_PRIMARY, want_pixels=False)
        assert np.array_equal(rgbp, rgbp1)
    finally:
        for sc in ranks:
            sc.close()


def test_render_multi_rejects_shared_scene(gpu):
    pkg = gpu
    name = "dragon_333x217"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    sc = scene_for(pkg, name)[0]
    with pytest.raises(pkg.CeresError, match="share a scene"):
        pkg.render_multi([sc, sc], pinned_basis(meta, cfg), pinned_sun(meta, cfg), cfg["W"], cfg["H"])


@pytest.mark.parametrize("build", ["ref", "exact"])
def test_cli_gpus_splits_frame(gpu, tmp_path, build):
    """./render --gpus 3 --row-block 5: the frame split over 3 ranks (device 0 reused on a one-GPU
    box) writes the reference's PPM and counts."""
    pkg = gpu
    name = "bunny_640"
    meta, _, ppm = load_golden(name)
    out = tmp_path / "bunny3.ppm"
    args = configs.cli_args(configs.CONFIGS[name]) + CLI_ARITH[build]
    r = subprocess.run([pkg.CLI_PATH] + args + ["--gpus", "3", "--row-block", "5", "-o", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "on 3 HIP ranks" in r.stdout
    assert "Rays: %d\tHits: %d" % (meta[build]["rays"], meta[build]["hits"]) in r.stdout
    assert out.read_bytes() == ppm[build]


def test_concurrent_streams_render_identical_frames(gpu):
    """bench.py's pattern: launches of one scene in flight on several HIP streams at once, with
    different batch shapes (1 and 3 frames, full frame and a row tiling) so their tile orders
    differ -- every output equals the same render done alone."""
    import torch
    pkg = gpu
    name = "dragon_333x217"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    scene = scene_for(pkg, name)[0]
    W, H = cfg["W"], cfg["H"]
    cam = scene_for(pkg, name)[1]
    b3, s3 = pkg.orbit_cameras(cam, cfg["sun"], W, H, 3, axis=(0.0, 0.0, 1.0), step_deg=45.0, rotate_first=False)
    b3[0] = pinned_basis(meta, cfg)
    s3[0] = pinned_sun(meta, cfg)
    jobs = [(b3[:1], s3[:1], pkg.Tiling(H, 0, 1)), (b3, s3, pkg.Tiling(H, 0, 1)), (b3, s3, pkg.Tiling(8, 1, 3)),
            (b3[:1], s3[:1], pkg.Tiling(5, 0, 2))]
    outs, refs = [], []
    for b, s, t in jobs:
        rows = pkg.local_rows(H, t)
        outs.append(torch.zeros(len(b) * 3 * W * rows, dtype=torch.uint8, device="cuda"))
        ref = torch.zeros_like(outs[-1])
        scene.render_batch_device(b, s, W, H, tiling=t, d_rgb8=ref.data_ptr())
        torch.cuda.synchronize()
        refs.append(ref.cpu())
    streams = [torch.cuda.Stream() for _ in jobs]
    for rep in range(4):
        for (b, s, t), o, st in zip(jobs, outs, streams):
            with torch.cuda.stream(st):
                o.zero_()
            scene.render_batch_device(b, s, W, H, tiling=t, d_rgb8=o.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        for o, r in zip(outs, refs):
            assert torch.equal(o.cpu(), r)


def test_tile_order_eviction_under_concurrent_streams(gpu):
    """More distinct batch shapes than the scene caches tile orders for (kMaxTileOrders = 16,
    scene_internal.hpp), launched round-robin on four streams and repeated, so least-recently-used
    orders are evicted -- their buffers RETIRED, not rewritten, while other streams' launches may
    still read them -- and, after more than kMaxRetired (64) evictions, freed in bulk behind one
    device synchronise while work is queued on the streams: every output still equals the same
    render done alone."""
    import torch
    pkg = gpu
    name = "dragon_333x217"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    b4, s4 = pkg.orbit_cameras(cam, cfg["sun"], W, H, 4, axis=(0.0, 0.0, 1.0), step_deg=30.0, rotate_first=False)
    b4[0] = pinned_basis(meta, cfg)
    s4[0] = pinned_sun(meta, cfg)
    jobs = []
    for nf in (1, 2, 3, 4):
        for t in (pkg.Tiling(H, 0, 1), pkg.Tiling(8, 0, 2), pkg.Tiling(8, 1, 2), pkg.Tiling(5, 2, 3),
                  pkg.Tiling(16, 0, 4)):
            jobs.append((b4[:nf], s4[:nf], t))
    assert len(jobs) == 20
    refs = []
    for b, s, t in jobs:
        ref = torch.zeros(len(b) * 3 * W * pkg.local_rows(H, t), dtype=torch.uint8, device="cuda")
        scene.render_batch_device(b, s, W, H, tiling=t, d_rgb8=ref.data_ptr())
        torch.cuda.synchronize()
        refs.append(ref.cpu())
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = [torch.zeros_like(r, device="cuda") for r in refs]
    for rep in range(6):
        # the same cyclic order every round: with 20 shapes for 16 slots every launch misses the LRU
        # cache, so ~120 orders are retired and the bulk free path runs at least once
        order = list(range(len(jobs)))
        for q, j in enumerate(order):
            b, s, t = jobs[j]
            st = streams[q % 4]
            with torch.cuda.stream(st):
                outs[j].zero_()
            scene.render_batch_device(b, s, W, H, tiling=t, d_rgb8=outs[j].data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        for j, (o, r) in enumerate(zip(outs, refs)):
            assert torch.equal(o.cpu(), r), f"rep {rep} job {j}"
    scene.close()


def test_fused_batch_allocates_no_shadow_queue(gpu):
    """The fused kernel keeps shadow rays on chip: a 64-frame batch must not allocate the
    two-pass path's HBM shadow-job queue (32 B x 64 per wavefront: ~150 MB here)."""
    import torch
    pkg = gpu
    name = "dragon_333x217"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, cam = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh, device=0)
    b, s = pkg.orbit_cameras(cam, cfg["sun"], W, H, 64, axis=(0.0, 0.0, 1.0), step_deg=5.0, rotate_first=False)
    out = torch.zeros(64 * 3 * W * H, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    scene.render_batch_device(b, s, W, H, d_rgb8=out.data_ptr())
    torch.cuda.synchronize()
    grown = free0 - torch.cuda.mem_get_info()[0]
    scene.close()
    assert grown < 32 << 20, f"device memory grew by {grown / 2**20:.1f} MiB for one fused batch"


@pytest.mark.parametrize("build", ["ref", "exact"])
@pytest.mark.parametrize("name", ["quad_65x49_robust", "bunny_97x61_primary_robust", "dragon_orbit3_333x217"])
def test_cli_modes_write_reference_ppm(gpu, tmp_path, name, build):
    """./render with --robust / --primary-only / --orbit (configs.cli_args) writes the
    reference's PPM byte for byte (each build's arithmetic)."""
    pkg = gpu
    meta, _, ppm = load_golden(name)
    out = tmp_path / "out.ppm"
    r = subprocess.run([pkg.CLI_PATH] + configs.cli_args(configs.CONFIGS[name]) + CLI_ARITH[build] + ["-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == ppm[build]


def test_robust_mode_rejected_for_double_scenes(gpu):
    pkg = gpu
    name = "dragon_333x217"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    mesh, bvh, cam = pkg.prepare(cfg, f64=True)
    sc = pkg.Scene(mesh, bvh, device=0)
    try:
        with pytest.raises(pkg.CeresError):
            sc.render(cam.basis(cfg["W"], cfg["H"]), np.asarray(cfg["sun"], np.float64), cfg["W"], cfg["H"],
                      mode=pkg.MODE_FULL | pkg.MODE_ROBUST)
    finally:
        sc.close()
