"""The background tile cull (render_hip.hip tile_misses_root) changes no pixel and no count.

Production kernels store a tile as misses when the root box's image, expanded by a margin, misses
every pixel of the tile; stats scenes (CERES_SCENE_STATS) never cull -- they trace every ray's own
root step, and their frames are the ones the parity suite pins to the reference.  Here random
cameras (inside and outside the scene box, wide and narrow fields of view, odd sizes, frames that
see the mesh at a grazing angle or from behind) render through both and every float pixel, PPM
byte and ray / hit count must agree, single frames and a 16-frame batch, full and primary-only."""
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


def _cameras(pkg, mesh, n, seed, arith, size=None):
    tri = mesh.tri.reshape(-1, 12)
    p0 = tri[:, 0:3].astype(np.float64)
    lo, hi = p0.min(0), p0.max(0)
    ctr, diag = (lo + hi) / 2, float(np.linalg.norm(hi - lo))
    rng = np.random.default_rng(seed)
    sizes = [(160, 120), (333, 217), (96, 200), (517, 77), (64, 64)]
    out = []
    for k in range(n):
        dirn = rng.normal(size=3)
        dirn /= np.linalg.norm(dirn)
        dist = diag * (rng.uniform(0.05, 0.4) if k % 7 == 0 else rng.uniform(0.6, 5.0))   # some inside the box
        eye = ctr + dirn * dist
        target = ctr + rng.uniform(-0.6, 0.6, 3) * (hi - lo)
        look = target - eye
        if k % 11 == 0:
            look = -look                                                          # facing away from the mesh
        up = rng.normal(size=3)
        fov = float(rng.uniform(15, 100))
        W, H = size or sizes[k % len(sizes)]
        cam = pkg.Camera(eye.astype(np.float32), look.astype(np.float32), up.astype(np.float32), fov, arith=arith)
        sun = (ctr + rng.normal(size=3) * diag * 4).astype(np.float32)
        out.append((cam.basis(W, H), sun, W, H))
    return out


@pytest.mark.parametrize("name", ["dragon_1080", "bunny_1080"])
@pytest.mark.parametrize("arith", [0, 1])
def test_cull_changes_nothing_single_frames(gpu, name, arith):
    pkg = gpu
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = pkg.prepare(cfg, arith=arith)
    prod, ref = pkg.Scene(mesh, bvh), pkg.Scene(mesh, bvh, stats=True)
    for mode in (pkg.MODE_FULL, pkg.MODE_PRIMARY):
        m = mode | (pkg.MODE_FMA if arith else 0)
        for k, (b12, sun, W, H) in enumerate(_cameras(pkg, mesh, 40, 17 + arith + 2 * mode, arith)):
            pa, ra, sa = prod.render(b12, sun, W, H, mode=m)
            pb, rb, sb = ref.render(b12, sun, W, H, mode=m)
            assert (sa["rays"], sa["hits"]) == (sb["rays"], sb["hits"]), (name, mode, k)
            assert np.array_equal(pa.view(np.uint32), pb.view(np.uint32)), (name, mode, k)
            assert np.array_equal(ra, rb), (name, mode, k)
    prod.close()
    ref.close()


@pytest.mark.parametrize("W,H", [(333, 217), (480, 272), (484, 270)])
def test_cull_changes_nothing_in_a_batch(gpu, W, H):
    """16 random views in one ceres_render_batch_device launch (the batch kernel: 4 tiles per wave,
    tiles of different frames in one wavefront, XCD row runs) against the stats scene's single
    frames.  Sizes: odd width (RGB8 byte stores), whole tiles with 4-byte rows (the dword RGB8 rows
    of store_tile), and 4-byte rows with ragged right and bottom tiles (both paths in one frame)."""
    import torch
    pkg = gpu
    cfg = configs.CONFIGS["dragon_1080"]
    mesh, bvh, _ = pkg.prepare(cfg, arith=1)
    prod, ref = pkg.Scene(mesh, bvh), pkg.Scene(mesh, bvh, stats=True)
    cams = [(b, s) for b, s, _, _ in _cameras(pkg, mesh, 16, 99, 1, size=(W, H))]
    b12 = np.stack([c[0] for c in cams]).astype(np.float32)
    s3 = np.stack([c[1] for c in cams]).astype(np.float32)
    px = torch.empty(16 * 3 * W * H, dtype=torch.float32, device="cuda")
    rgb = torch.empty(16 * 3 * W * H, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    prod.render_batch_device(b12, s3, W, H, mode=pkg.MODE_FULL | pkg.MODE_FMA, d_pixels=px.data_ptr(),
                             d_rgb8=rgb.data_ptr(), d_counters=cnt.data_ptr())
    torch.cuda.synchronize()
    px = px.cpu().numpy().reshape(16, -1)
    rgb = rgb.cpu().numpy().reshape(16, -1)
    rays = hits = 0
    for f in range(16):
        pb, rb, sb = ref.render(b12[f], s3[f], W, H, mode=pkg.MODE_FULL | pkg.MODE_FMA)
        rays += sb["rays"]
        hits += sb["hits"]
        assert np.array_equal(px[f].view(np.uint32), pb.view(np.uint32)), f
        assert np.array_equal(rgb[f], rb), f
    c = cnt.cpu().numpy()
    assert (int(c[0]), int(c[1])) == (rays, hits)
    prod.close()
    ref.close()
