"""The shadow BVH4's traversal-stack bounds (render_hip.hip scene creation; scene_host.cpp
build_shadow_bvh4 / order_shadow_bvh4) against an independent restatement over the reference BVH.

The BVH4 record of a BVH2 node takes its children, each replaced by its own two children when both
of their boxes lie inside its box; a record pushes all but one of its passing inner children.
* nearest-first walks (the work-stealing loop): a record may descend into any passing child with
  every other one pushed, so the bound is the sum over a root-leaf path of (inner children - 1);
* first-passing-child walks (trace_any4, packet_any4, the stealing loop of LDS-bound scenes): the
  child in slot j of k starts with at most max(k-1-j, j-1) of its record's entries below it, and
  the host orders each record's inner children so the largest subtree needs take the smallest
  weights; this test recomputes that optimum.
Both must equal what the library reports, and the frames those stacks serve must stay the
reference's (every parity test renders through them; a bound that is too small raises the
traversal-overflow error instead of returning a frame)."""
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


def _bounds(nodes):
    nd = np.asarray(nodes).reshape(-1, 8)
    box = nd[:, :6].view(np.float32)
    cnt, first = nd[:, 6], nd[:, 7]
    assert cnt.max() <= 31            # no piece nodes in these scenes

    def inside(c, p):
        return bool(np.all(box[c, 0::2] >= box[p, 0::2]) and np.all(box[c, 1::2] <= box[p, 1::2]))

    def inner_entries(x):
        out = []
        c = int(first[x])
        for s in (c, c + 1):
            if cnt[s]:
                continue
            g = int(first[s])
            if inside(g, s) and inside(g + 1, s):
                out += [q for q in (g, g + 1) if cnt[q] == 0]
            else:
                out.append(s)
        return out

    if cnt[0]:
        return 1, 1
    order, st = [], [0]
    kids = {}
    while st:
        x = st.pop()
        order.append(x)
        kids[x] = inner_entries(x)
        st.extend(kids[x])
    near, firstb = {}, {}
    for x in reversed(order):
        ch = kids[x]
        k = len(ch)
        if not k:
            near[x] = firstb[x] = 0
            continue
        near[x] = (k - 1) + max(near[c] for c in ch)
        w = sorted(max(k - 1 - j, j - 1) for j in range(k))
        need = sorted((firstb[c] for c in ch), reverse=True)
        firstb[x] = max(a + b for a, b in zip(w, need))
    return max(1, near[0]), max(1, min(near[0], firstb[0]))


@pytest.mark.parametrize("name", ["dragon_1080", "bunny_1080", "proc_101"])
def test_shadow_stack_bounds_match_restatement(gpu, name):
    """Build order (these scenes' stacks fit the LDS budget): both walks use the nearest-first
    bound.  CERES_SCENE_FIRST_ORDER (what C5 gets automatically): the inner children ordered,
    the first-passing-child bound the optimum above."""
    pkg = gpu
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = pkg.prepare(cfg, arith=1)
    near, firstb = _bounds(bvh.nodes)
    assert firstb <= near
    for first_order, expect in ((False, (near, near)), (True, (near, firstb))):
        scene = pkg.Scene(mesh, bvh, first_order=first_order)
        info = scene.info()
        assert (info["shadow_stack_nearest"], info["shadow_stack_first"]) == expect, first_order
        scene.close()


@pytest.mark.parametrize("name", ["dragon_1080", "bunny_1080", "dragon_333x217", "dupleaf", "dragon_orbit3_333x217"])
def test_first_order_frames_equal_reference(gpu, name):
    """A first-order scene renders single frames with the stealing loop taking the first passing
    child under the smaller stack bound, and 16-frame batches with the ordered records: every PPM
    byte and the ray / hit counts must still be the reference CMake build's (a bound too small
    would raise the traversal-overflow error)."""
    import hashlib
    import torch
    from test_gpu_fma import ref_basis, ref_sun
    from conftest import load_golden
    pkg = gpu
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    mesh, bvh, _ = pkg.prepare(cfg, arith=1)
    scene = pkg.Scene(mesh, bvh, first_order=True)
    W, H = cfg["W"], cfg["H"]
    mode = pkg.cfg_mode(cfg, 1)
    b12, sun = ref_basis(meta), ref_sun(meta)
    px, rgb, st = scene.render(b12, sun, W, H, mode=mode)
    assert hashlib.sha256(pkg.ppm(W, H, rgb)).hexdigest() == meta["ppm_sha256"]["ref"]
    assert (st["rays"], st["hits"]) == (meta["ref"]["rays"], meta["ref"]["hits"])
    F = 16
    d_rgb = torch.empty(F * 3 * W * H, dtype=torch.uint8, device="cuda")
    d_px = torch.empty(F * 3 * W * H, dtype=torch.float32, device="cuda")
    scene.render_batch_device(np.repeat(b12[None], F, 0), np.repeat(np.asarray(sun)[None], F, 0), W, H, mode=mode,
                              d_pixels=d_px.data_ptr(), d_rgb8=d_rgb.data_ptr())
    torch.cuda.synchronize()
    frames = d_rgb.cpu().numpy().reshape(F, -1)
    for f in range(F):
        assert hashlib.sha256(pkg.ppm(W, H, frames[f])).hexdigest() == meta["ppm_sha256"]["ref"], f
    scene.close()


def test_c5_first_order_bound_fits_the_primary_stack(gpu):
    """C5: its nearest-first bound (37 entries x 3 B x 64 lanes + mailboxes = 7.9 KB per wave)
    costs waves, so the scene is ordered automatically: the first-passing-child bound (27) fits the
    primary stack's LDS (depth + 1 entries) and its single-frame launches hold a wave more per
    SIMD."""
    pkg = gpu
    cfg = configs.CONFIGS["proc_c5"]
    mesh, bvh, _ = pkg.prepare(cfg, arith=1)
    scene = pkg.Scene(mesh, bvh)
    info = scene.info()
    assert info["shadow_stack_first"] < info["shadow_stack_nearest"]
    assert info["shadow_stack_first"] <= info["stack_entries"] + 1
    scene.close()
