"""CERES_MODE_QBVH4: shadow rays over a COMPRESSED BVH4 -- 64-B nodes whose
child bounds are bytes decoded as fma(q, scale, origin), rounded outwards on the host.  Not
bit-exact, so it is never the default; held here to the SURVEY §7 budget against the reference
(±1 LSB per channel, at most max(1, 1e-5 W H) pixels beyond it).  The reference's bytes are the
exact mode's own output, which the same test first checks against the reference PPM sha256.

Decoded boxes contain the exact ones and the fast slab test is monotone in the bounds
(node_intersectors.hpp:83-103), so every leaf the reference's traversal reaches is still tested:
an occluded pixel can never turn lit; only a grazing shadow ray can meet a triangle the
reference's slab tests never reach (a lit pixel turns dark).  Both directions are counted."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden, ppm_budget_ok

import configs

pytestmark = pytest.mark.gpu

CASES = ["dragon_1080", "bunny_1080", "dragon_4096", "dragon_640", "bunny_640", "dragon_333x217", "dupleaf",
         "degenerate", "quad", "tri1", "proc_101", "dragon_orbit3_333x217", "proc_c5"]


def _basis(meta, cfg):
    hx = lambda a: np.asarray([int(h, 16) for h in a], np.uint32).view(np.float32)   # noqa: E731
    eye = hx(meta["pose"]["eye"]) if "pose" in meta else np.asarray(cfg["eye"], np.float32)
    sun = hx(meta["pose"]["sun"]) if "pose" in meta else np.asarray(cfg["sun"], np.float32)
    return np.concatenate([eye, hx(meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"])]), sun


@pytest.mark.parametrize("name", CASES)
def test_qbvh4_within_budget(pkg, name):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    cfg = configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    W, H = cfg["W"], cfg["H"]
    mesh, bvh, _ = pkg.prepare(cfg)
    scene = pkg.Scene(mesh, bvh)
    del mesh, bvh
    basis, sun = _basis(meta, cfg)
    _, rgb_e, st_e = scene.render(basis, sun, W, H, want_pixels=False)
    ppm_e = pkg.ppm(W, H, rgb_e)
    assert hashlib.sha256(ppm_e).hexdigest() == meta["ppm_sha256"]["exact"]          # exact mode = the reference
    _, rgb_q, st_q = scene.render(basis, sun, W, H, mode=pkg.MODE_FULL | pkg.MODE_QBVH4, want_pixels=False)
    ok, bad = ppm_budget_ok(pkg.ppm(W, H, rgb_q), ppm_e, W, H)
    assert ok, f"{bad} pixels beyond +-1 LSB"
    _, _, sh_e, _ = scene.records(basis, sun, W, H)
    _, _, sh_q, _ = scene.records(basis, sun, W, H, mode=pkg.MODE_FULL | pkg.MODE_QBVH4)
    darkened = int(np.count_nonzero((sh_e == 0) & (sh_q == 1)))
    lightened = int(np.count_nonzero((sh_e == 1) & (sh_q == 0)))
    assert lightened == 0, "an occluded pixel turned lit: a decoded box lost an exact box's hit"
    assert np.array_equal(sh_e == -1, sh_q == -1)                  # the primary pass is untouched
    assert st_q["rays"] == st_e["rays"] and st_q["hits"] - st_e["hits"] == darkened
    assert darkened <= max(1, int(1e-5 * W * H))
    scene.close()


def test_qbvh4_rejects_robust_and_stats(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    cfg = configs.CONFIGS["dragon_333x217"]
    meta, _, _ = load_golden("dragon_333x217")
    mesh, bvh, _ = pkg.prepare(cfg)
    basis, sun = _basis(meta, cfg)
    scene = pkg.Scene(mesh, bvh)
    with pytest.raises(pkg.CeresError):
        scene.render(basis, sun, 64, 48, mode=pkg.MODE_FULL | pkg.MODE_QBVH4 | pkg.MODE_ROBUST)
    scene.close()
    st = pkg.Scene(mesh, bvh, stats=True)
    with pytest.raises(pkg.CeresError):
        st.render(basis, sun, 64, 48, mode=pkg.MODE_FULL | pkg.MODE_QBVH4)
    st.close()
