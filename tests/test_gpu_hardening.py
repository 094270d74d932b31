"""Round 6 hardening: the production kernels REPORT a broken
traversal-stack bound, non-finite shadow rays never reach the wave-wide packet walk, and the
batch paths whose pieces only bench rehearsals covered -- 64-frame batches split into two launches
with counters and float pixels, the background cull under a multi-rank row tiling -- equal their
one-frame / uncull'd counterparts."""
import os

import numpy as np
import pytest

import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


@pytest.fixture(scope="module")
def dragon(gpu):
    cfg = configs.CONFIGS["dragon_333x217"]
    mesh, bvh, cam = gpu.prepare(cfg, arith=1)
    sc = gpu.Scene(mesh, bvh)
    yield cfg, mesh, bvh, cam, sc
    sc.close()


def _count_build():
    import importlib.util
    pkgdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ceres-raytracer_amd")
    path = os.path.join(pkgdir, "variants", "libceres_hip_count.so")
    assert os.path.exists(path), "the diagnostic build is part of build() (make all)"
    spec = importlib.util.spec_from_file_location("ceres_count_build_t", os.path.join(pkgdir, "__init__.py"),
                                                  submodule_search_locations=[pkgdir])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.LIB_PATH = path
    mod.lib()
    return mod


def test_stack_guard_reports_an_overrun(gpu, dragon, monkeypatch):
    """guarded_trace (the diagnostic build, libceres_hip_count.so, which bench.py runs over the timed
    views): the walk without per-step clamps keeps a guard value in LDS slot stack_entries, which
    an exact bound never reaches.  CERES_DEBUG_GUARD_SLOT moves the guard down into slots deep walks
    DO write (the LDS carve-up and every index unchanged), so the guard is overwritten: the render
    must fail with CERES_ESTACK -- single frames (work-stealing kernel) and batches (packet kernel)
    alike -- and succeed again, with the product's bytes, once the guard is back in place."""
    import torch
    pkg = gpu
    cfg, mesh, bvh, cam, prod = dragon
    cb = _count_build()
    sc = cb.Scene(mesh, bvh)
    W, H = cfg["W"], cfg["H"]
    b12 = cam.basis(W, H)
    mode = pkg.MODE_FULL | pkg.MODE_FMA
    _, rgb0, st0 = prod.render(b12, cfg["sun"], W, H, mode=mode)
    monkeypatch.setenv("CERES_DEBUG_GUARD_SLOT", "2")
    with pytest.raises(cb.CeresError, match="-5"):
        sc.render(b12, cfg["sun"], W, H, mode=mode)
    F = 4
    rgb = torch.zeros(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    sc.render_batch_device(np.repeat(b12[None], F, 0), np.repeat(np.asarray(cfg["sun"], np.float32)[None], F, 0), W, H,
                           mode=mode, d_rgb8=rgb.data_ptr(), d_counters=cnt.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert int(cnt[6].item()) != 0, "the batch kernel's error word must report the overwritten guard"
    monkeypatch.delenv("CERES_DEBUG_GUARD_SLOT")
    _, rgb1, st1 = sc.render(b12, cfg["sun"], W, H, mode=mode)
    assert np.array_equal(rgb0, rgb1) and (st0["rays"], st0["hits"]) == (st1["rays"], st1["hits"])
    sc.close()


def test_counting_build_tallies_fetches(gpu, dragon):
    """The diagnostic build's fetch tallies (bench.py roofline.build_bytes): zero before a render,
    then every kind a dragon batch exercises is non-zero, the stores equal 15 B per pixel (float +
    RGB8), and the product library refuses the call (EUNSUPPORTED) instead of reporting zeros."""
    import torch
    pkg = gpu
    cfg, mesh, bvh, cam, _ = dragon
    cb = _count_build()
    sc = cb.Scene(mesh, bvh)
    W, H = cfg["W"], cfg["H"]
    F = 4
    b12 = np.repeat(cam.basis(W, H)[None], F, 0)
    s3 = np.repeat(np.asarray(cfg["sun"], np.float32)[None], F, 0)
    rgb = torch.zeros(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    px = torch.zeros(F * 3 * W * H, dtype=torch.float32, device="cuda")
    cb.fetch_counters(0, reset=True)
    assert sum(cb.fetch_counters(0, reset=False).values()) == 0
    sc.render_batch_device(b12, s3, W, H, mode=pkg.MODE_FULL | pkg.MODE_FMA, d_pixels=px.data_ptr(),
                           d_rgb8=rgb.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    c = cb.fetch_counters(0, reset=True)
    assert c["store_vector"] == 15 * F * W * H
    for k in ("bvh2_vector", "bvh4_scalar", "tri_scalar", "shade_vector", "order_scalar"):
        assert c[k] > 0, k
    assert c["bvh2_vector"] % 64 == 0 and c["tri_vector"] % 48 == 0
    with pytest.raises(pkg.CeresError, match="-6"):
        pkg.fetch_counters(0)
    sc.close()


@pytest.mark.parametrize("sun", [(np.inf, 0.0, 0.0), (0.0, -np.inf, 3.0), (np.nan, 1.0, 1.0), (1e38, -3e38, 2e38)])
def test_nonfinite_sun_takes_the_per_lane_walk(gpu, dragon, oracle_mod, sun):
    """packet_any4 relies on finite slab constants (an empty BVH4 slot then
    fails by itself).  With a non-finite sun the shadow direction is NaN / the slab constants are
    not finite; such tiles must take the per-lane loop (which tests the child word), not walk into
    n4_first(kNode4Empty).  The batch (packet) kernel, the single-frame (work-stealing) kernel and
    the oracle restatement must agree: equal PPM bytes and counts, equal floats where finite and
    NaN in the same pixels (a NaN's payload is not portable between x86 and gfx950)."""
    import torch
    pkg = gpu
    cfg, mesh, bvh, cam, sc = dragon
    W, H = cfg["W"], cfg["H"]
    b12 = cam.basis(W, H)
    s3 = np.asarray(sun, np.float32)
    mode = pkg.MODE_FULL | pkg.MODE_FMA
    px1, rgb1, st1 = sc.render(b12, s3, W, H, mode=mode)
    F = 3
    px = torch.zeros(F * 3 * W * H, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    sc.render_batch_device(np.repeat(b12[None], F, 0), np.repeat(s3[None], F, 0), W, H, mode=mode,
                           d_pixels=px.data_ptr(), d_rgb8=rgb.data_ptr(), d_counters=cnt.data_ptr(),
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    assert (int(c[0]), int(c[1]), int(c[6])) == (F * st1["rays"], F * st1["hits"], 0)
    pxb = px.cpu().numpy().reshape(F, -1)
    rgbb = rgb.cpu().numpy().reshape(F, -1)
    for f in range(F):
        assert np.array_equal(rgbb[f], rgb1.reshape(-1)), f
        a, b = pxb[f], px1.reshape(-1)
        assert np.array_equal(np.isnan(a), np.isnan(b)), f
        fin = ~np.isnan(a)
        assert np.array_equal(a[fin].view(np.uint32), b[fin].view(np.uint32)), f
    osc = oracle_mod.prepare(cfg, contract=True)
    ref = oracle_mod.render(osc, cfg, basis=b12[3:], sun=s3)
    assert (ref["rays"], ref["hits"]) == (st1["rays"], st1["hits"])
    r = ref["pixels"].reshape(-1)
    a = px1.reshape(-1)
    assert np.array_equal(np.isnan(a), np.isnan(r))
    fin = ~np.isnan(a)
    assert np.array_equal(a[fin].view(np.uint32), r[fin].view(np.uint32))


def test_batch_of_64_frames_counters_and_floats(gpu, dragon):
    """a 64-frame batch is two launches of 32 (the kernel-argument block holds 56
    frames): the first cleans the counter shards, the last sums them, each writes its float and
    RGB8 frames at its own offset.  Rays / hits = the sum of the 64 single-frame counts, and every
    frame's floats and bytes equal a one-frame render's, whole frames and one rank of a 3-way split."""
    import torch
    pkg = gpu
    cfg, mesh, bvh, cam, sc = dragon
    W, H = cfg["W"], cfg["H"]
    cam0 = pkg.Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"], arith=1)
    b12, s3 = pkg.orbit_cameras(cam0, cfg["sun"], W, H, 64, axis=configs.BENCH_ORBIT[0], step_deg=5.625,
                                rotate_first=False)
    st = torch.cuda.current_stream().cuda_stream
    mode = pkg.MODE_FULL | pkg.MODE_FMA
    for til in (pkg.Tiling(H, 0, 1), pkg.Tiling(8, 1, 3)):
        rows = pkg.local_rows(H, til)
        rgb = torch.zeros((64, rows, 3 * W), dtype=torch.uint8, device="cuda")
        px = torch.zeros((64, rows, 3 * W), dtype=torch.float32, device="cuda")
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        sc.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(), d_rgb8=rgb.data_ptr(),
                               d_counters=cnt.data_ptr(), stream=st)
        one_rgb = torch.zeros((rows, 3 * W), dtype=torch.uint8, device="cuda")
        one_px = torch.zeros((rows, 3 * W), dtype=torch.float32, device="cuda")
        one_cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        rays = hits = 0
        for f in range(64):
            sc.render_device(b12[f], s3[f], W, H, mode=mode, tiling=til, d_pixels=one_px.data_ptr(),
                             d_rgb8=one_rgb.data_ptr(), d_counters=one_cnt.data_ptr(), stream=st)
            torch.cuda.synchronize()
            rays += int(one_cnt[0].item())
            hits += int(one_cnt[1].item())
            assert torch.equal(rgb[f], one_rgb), (f, til)
            assert torch.equal(px[f].view(torch.int32), one_px.view(torch.int32)), (f, til)
        c = cnt.cpu().numpy()
        assert (int(c[0]), int(c[1]), int(c[6])) == (rays, hits, 0), til


@pytest.mark.parametrize("world", [2, 3])
def test_cull_under_row_tiling(gpu, world):
    """the background cull maps a rank's local rows to global rows (global_row) before
    testing the frame's cull rectangle.  Every rank's rows of random views (single frames and a
    16-frame batch) equal the stats scene's (which never culls), floats, bytes and counts."""
    import torch
    pkg = gpu
    from test_gpu_cull import _cameras
    cfg = configs.CONFIGS["dragon_1080"]
    mesh, bvh, _ = pkg.prepare(cfg, arith=1)
    prod, ref = pkg.Scene(mesh, bvh), pkg.Scene(mesh, bvh, stats=True)
    mode = pkg.MODE_FULL | pkg.MODE_FMA
    st = torch.cuda.current_stream().cuda_stream
    cams = _cameras(pkg, mesh, 16, 91 + world, 1, size=(333, 217))
    W, H = 333, 217
    b12 = np.stack([c[0] for c in cams])
    s3 = np.stack([c[1] for c in cams])
    for r in range(world):
        til = pkg.Tiling(8, r, world)
        rows = pkg.local_rows(H, til)
        out = {}
        for name, sc in (("prod", prod), ("ref", ref)):
            rgb = torch.zeros((16, rows, 3 * W), dtype=torch.uint8, device="cuda")
            px = torch.zeros((16, rows, 3 * W), dtype=torch.float32, device="cuda")
            cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
            sc.render_batch_device(b12, s3, W, H, mode=mode, tiling=til, d_pixels=px.data_ptr(), d_rgb8=rgb.data_ptr(),
                                   d_counters=cnt.data_ptr(), stream=st)
            one = []
            for f in (0, 5, 11):
                o_rgb = torch.zeros((rows, 3 * W), dtype=torch.uint8, device="cuda")
                sc.render_device(b12[f], s3[f], W, H, mode=mode, tiling=til, d_rgb8=o_rgb.data_ptr(), stream=st)
                one.append(o_rgb)
            torch.cuda.synchronize()
            out[name] = (rgb, px.view(torch.int32), cnt[:2].clone(), one)
        a, b = out["prod"], out["ref"]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), (world, r)
        assert torch.equal(a[2], b[2]), (world, r)
        for k in range(3):
            assert torch.equal(a[3][k], b[3][k]), (world, r, k)
    prod.close()
    ref.close()


def test_lit_record_buffer_is_capped(gpu, dragon):
    """the compacted float readback holds records for at most half the pixels; a frame
    lit above that overflows the records and falls back to the full copy in the same call.  A sparse
    frame, then a dense one (a narrow view filled by the mesh, lit from the camera) -- each call,
    including the first dense call that takes the overflow path -- equal the device framebuffer of
    the same render."""
    import torch
    pkg = gpu
    cfg, mesh, bvh, cam, sc = dragon
    W, H = cfg["W"], cfg["H"]
    mode = pkg.MODE_FULL | pkg.MODE_FMA
    tri = mesh.tri.reshape(-1, 12)
    ctr = tri[:, 0:3].mean(0)
    views = [(cam.basis(W, H), np.asarray(cfg["sun"], np.float32), False)]
    eye = (ctr + (np.asarray(cfg["eye"], np.float32) - ctr) * 0.6).astype(np.float32)
    c = pkg.Camera(eye, (ctr - eye).astype(np.float32), np.asarray(cfg["up"], np.float32), 12.0, arith=1)
    views.append((c.basis(W, H), (eye + np.float32(0.01)).astype(np.float32), True))
    for b12, sun, dense in views:
        d = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda")
        sc.render_device(b12, sun, W, H, mode=mode, d_pixels=d.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        dev = d.cpu().numpy()
        lit = float(np.mean((dev.reshape(-1, 3).view(np.uint32) != 0).any(1)))
        assert (lit > 0.5) == dense, lit
        for call in range(2):
            host, _, st = sc.render(b12, sun, W, H, mode=mode)
            assert np.array_equal(host.reshape(-1).view(np.uint32), dev.view(np.uint32)), (dense, call)
