"""The frames bench.py times, against the REFERENCE: every view of a bench step (pkg.bench_views:
the config camera + sun rotated once by f x 360 / F degrees about z, anim.cpp:76-110 /
transform.hpp:67-112) rendered the way bench.py renders it -- one ceres_render_batch_device
launch per 64 frames per rank, each rank its interleaved 8-row blocks, frames in the
FrameExchange batch order at N > 1 -- reassembled, and compared by PPM sha256 with the
reference's own render() of the same view (tests/golden/orbit/<cfg>.json, made by
oracle/_ref/ref_render{_exact,} --orbit-views): in both arithmetics, the reference CMake build's
(FMA contraction, bench.py's default) and the contraction-free one.  The step's rays / hits equal the sum of the
reference's per-view counts (render.hpp:155).  N = 1 is the bench step on one GPU; N = 2, 4, 8
are the weak-scaling steps (16N views, 22.5/N degrees apart), every rank's share rendered here
in turn on the one GPU."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden, load_orbit

import configs

pytestmark = pytest.mark.gpu

MAXF = 64          # frames per batch launch (kMaxFrames)


def _basis0(meta, cfg, build):
    b = meta["ref_basis"] if build == "ref" else meta["basis"]
    bits = [int(h, 16) for h in b["dir"] + b["u"] + b["v"]]
    return np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])


_scenes = {}


def _scene(pkg, name, arith):
    if (name, arith) not in _scenes:
        _scenes.clear()                     # one big scene resident at a time
        cfg = configs.CONFIGS[name]
        mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
        _scenes[(name, arith)] = (pkg.Scene(mesh, bvh, device=0), cam)
    return _scenes[(name, arith)]


CASES = [("bunny_640", 1), ("dragon_1080", 1), ("dragon_1080", 2), ("dragon_1080", 4), ("dragon_1080", 8),
         ("bunny_1080", 1), ("bunny_1080_primary", 1), ("dragon_4096", 1), ("dragon_4096", 8), ("proc_c5", 1),
         ("proc_c5", 8)]


@pytest.mark.parametrize("build", ["ref", "exact"])
@pytest.mark.parametrize("name,world", CASES)
def test_bench_step_frames_match_reference(pkg, name, world, build):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    import ceres_raytracer_amd.distributed as D
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    meta, _, _ = load_golden(name)
    fx = load_orbit(name)["by_step_bits"]
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    scene, cam = _scene(pkg, name, arith)
    F = 16 * world
    b12, s3, steps = pkg.bench_views(cam, cfg["sun"], W, H, F, basis0=_basis0(meta, cfg, build))
    if world > 1:
        order = D.exchange_order(F, world)
        b12, s3, steps = b12[order], s3[order], steps[order]
    row_block = 8 if world > 1 else H
    mode = pkg.cfg_mode(cfg, arith)
    st = torch.cuda.current_stream().cuda_stream
    _, maxrows = D.ppm_row_permutation(H, row_block, world)
    idx = torch.as_tensor(D.ppm_row_permutation(H, row_block, world)[0], device="cuda")
    per_rank = []
    rays = hits = 0
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    for r in range(world):
        til = pkg.Tiling(row_block, r, world)
        rows = pkg.local_rows(H, til)
        tight = torch.zeros((F, rows, 3 * W), dtype=torch.uint8, device="cuda")
        for f0 in range(0, F, MAXF):
            f1 = min(F, f0 + MAXF)
            counters.zero_()
            scene.render_batch_device(b12[f0:f1], s3[f0:f1], W, H, mode=mode, tiling=til,
                                      d_rgb8=tight[f0].data_ptr(), d_counters=counters.data_ptr(), stream=st)
            torch.cuda.synchronize()
            c = counters.cpu().numpy()
            assert c[6] == 0, "traversal stack overflow"
            rays += int(c[0]); hits += int(c[1])
        buf = torch.zeros((F, maxrows, 3 * W), dtype=torch.uint8, device="cuda")
        buf[:, :rows] = tight
        del tight
        per_rank.append(buf)
    head = b"P6 %d %d 255\n" % (W, H)
    bad = []
    ref_rays = ref_hits = 0
    for f in range(F):
        e0 = fx["%08x" % int(np.asarray(steps[f], np.float32).view(np.uint32))]
        e = e0["ref"] if build == "ref" else e0
        ref_rays += e["rays"]; ref_hits += e["hits"]
        full = torch.cat([b[f] for b in per_rank])[idx].cpu().numpy()
        if hashlib.sha256(head + full.tobytes()).hexdigest() != e["sha256"]:
            bad.append((f, e0["k"]))
    assert not bad, f"frames differing from the reference (batch frame, orbit view k): {bad}"
    assert (rays, hits) == (ref_rays, ref_hits)


FRAMES_CASES = [("dragon_1080", 2, "ref"), ("dragon_1080", 4, "exact"), ("dragon_1080", 8, "ref"),
                ("bunny_1080", 2, "ref"), ("dragon_4096", 2, "ref"), ("proc_c5", 2, "ref")]


@pytest.mark.parametrize("name,world,build", FRAMES_CASES)
def test_bench_frames_partition_matches_reference(pkg, name, world, build):
    """bench.py --collect frames (its default for C3 at every N and for the tiled C4 / C5 at N = 2):
    rank q renders batch frames q*k .. q*k+k-1 of exchange_order (orbit frames q, q+N, ...) WHOLE
    with one batch launch; its k PPM bodies are the reference's, and the ranks' rays / hits add up
    to the step's reference counts."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    import ceres_raytracer_amd.distributed as D
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    meta, _, _ = load_golden(name)
    fx = load_orbit(name)["by_step_bits"]
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    scene, cam = _scene(pkg, name, arith)
    F = 16 * world
    b12, s3, steps = pkg.bench_views(cam, cfg["sun"], W, H, F, basis0=_basis0(meta, cfg, build))
    order = D.exchange_order(F, world)
    b12, s3, steps = b12[order], s3[order], steps[order]
    mode = pkg.cfg_mode(cfg, arith)
    st = torch.cuda.current_stream().cuda_stream
    head = b"P6 %d %d 255\n" % (W, H)
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    rays = hits = 0
    bad = []
    for r in range(world):
        g = D.FrameOwner(W, H, r, world, frames=F, device="cuda", slots=1)
        mine = g.owned_frames()
        counters.zero_()
        scene.render_batch_device(b12[mine], s3[mine], W, H, mode=mode, tiling=pkg.Tiling(H, 0, 1),
                                  d_rgb8=g.local_ptr(0), d_counters=counters.data_ptr(), stream=st)
        torch.cuda.synchronize()
        c = counters.cpu().numpy()
        assert c[6] == 0, "traversal stack overflow"
        rays += int(c[0]); hits += int(c[1])
        full = g.finish(0)
        for m, f in enumerate(mine):
            e0 = fx["%08x" % int(np.asarray(steps[f], np.float32).view(np.uint32))]
            e = e0["ref"] if build == "ref" else e0
            if hashlib.sha256(head + full[m].cpu().numpy().tobytes()).hexdigest() != e["sha256"]:
                bad.append((r, f, e0["k"]))
        del g, full
    assert not bad, f"frames differing from the reference (rank, batch frame, orbit view k): {bad}"
    ref = [fx["%08x" % int(np.asarray(x, np.float32).view(np.uint32))] for x in steps]
    ref = [e["ref"] if build == "ref" else e for e in ref]
    assert (rays, hits) == (sum(e["rays"] for e in ref), sum(e["hits"] for e in ref))


BANDS_CASES = [("dragon_1080", 2, "ref"), ("dragon_1080", 8, "ref"), ("dragon_1080", 4, "exact"),
               ("dragon_4096", 8, "ref"), ("bunny_640", 4, "exact"), ("proc_c5", 4, "ref")]


@pytest.mark.parametrize("name,world,build", BANDS_CASES)
def test_bench_bands_partition_matches_reference(pkg, name, world, build):
    """bench.py --collect bands (the tiled C4 / C5 at N >= 4; C3's partition_alt): rank r renders
    band (r + f) mod N of every batch frame f (ceres_tiling.bands, one launch per 64 frames, the
    rotation carried across launches and the library's 56-frame chunks); every band placed in its
    rows of the owner's PPM body (the layout distributed.FrameBands receives in place) gives the
    reference's frame, and the ranks' rays / hits add up to the step's reference counts."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    import ceres_raytracer_amd.distributed as D
    cfg = configs.CONFIGS[name]
    W, H = cfg["W"], cfg["H"]
    meta, _, _ = load_golden(name)
    fx = load_orbit(name)["by_step_bits"]
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    scene, cam = _scene(pkg, name, arith)
    F = 16 * world
    b12, s3, steps = pkg.bench_views(cam, cfg["sun"], W, H, F, basis0=_basis0(meta, cfg, build))
    order = D.exchange_order(F, world)
    b12, s3, steps = b12[order], s3[order], steps[order]
    mode = pkg.cfg_mode(cfg, arith)
    st = torch.cuda.current_stream().cuda_stream
    bh = D.band_height(H, world)
    full = torch.zeros((F, H, 3 * W), dtype=torch.uint8, device="cuda")
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    rays = hits = 0
    for r in range(world):
        assert pkg.local_rows(H, pkg.Tiling(bh, r, world, 1)) == bh
        buf = torch.zeros((F, bh, 3 * W), dtype=torch.uint8, device="cuda")
        for f0 in range(0, F, MAXF):
            f1 = min(F, f0 + MAXF)
            counters.zero_()
            scene.render_batch_device(b12[f0:f1], s3[f0:f1], W, H, mode=mode, tiling=pkg.Tiling(bh, (r + f0) % world, world, 1),
                                      d_rgb8=buf[f0].data_ptr(), d_counters=counters.data_ptr(), stream=st)
            torch.cuda.synchronize()
            c = counters.cpu().numpy()
            assert c[6] == 0, "traversal stack overflow"
            rays += int(c[0]); hits += int(c[1])
        for f in range(F):
            b = (r + f) % world
            n = D.band_rows(H, bh, b)
            if n:
                top = H - b * bh - n
                full[f, top:top + n] = buf[f, bh - n:]
        del buf
    head = b"P6 %d %d 255\n" % (W, H)
    bad = []
    ref_rays = ref_hits = 0
    for f in range(F):
        e0 = fx["%08x" % int(np.asarray(steps[f], np.float32).view(np.uint32))]
        e = e0["ref"] if build == "ref" else e0
        ref_rays += e["rays"]; ref_hits += e["hits"]
        if hashlib.sha256(head + full[f].cpu().numpy().tobytes()).hexdigest() != e["sha256"]:
            bad.append((f, e0["k"]))
    assert not bad, f"frames differing from the reference (batch frame, orbit view k): {bad}"
    assert (rays, hits) == (ref_rays, ref_hits)


def test_band_tiling_rejects_uncovered_frames(pkg):
    """ceres_tiling.bands needs row_block * world >= height (every row in some band)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    cfg = configs.CONFIGS["bunny_640"]
    scene, cam = _scene(pkg, "bunny_640", pkg.ARITH_EXACT)
    W, H = cfg["W"], cfg["H"]
    out = torch.zeros(3 * W * H, dtype=torch.uint8, device="cuda")
    b12 = np.asarray(cam.basis(W, H), np.float32)[None]
    with pytest.raises(pkg.CeresError):
        scene.render_batch_device(b12, np.asarray(cfg["sun"], np.float32)[None], W, H, tiling=pkg.Tiling(8, 0, 4, 1),
                                  d_rgb8=out.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
