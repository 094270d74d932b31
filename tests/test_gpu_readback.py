"""ceres_render_f32's host float framebuffer (render.hpp:86-89: every pixel of the caller's buffer
is written) through the compacted readback: only the lit pixels cross the host link and the host
writes the zeros.  The caller's buffer is pre-filled with garbage before every call, and every
float must equal the device framebuffer of the same view rendered by ceres_render_device (no host
copy logic involved); dense frames (most pixels lit) switch to the full copy, and the next sparse
frames must come out right as well."""
import ctypes

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


def _host_render(pkg, scene, b12, sun, W, H, mode):
    px = np.full(3 * W * H, np.nan, np.float32)
    px.view(np.uint32)[::7] = 0xdeadbeef
    rgb = np.full(3 * W * H, 0xab, np.uint8)
    st = pkg._Stats()
    b = np.ascontiguousarray(b12, np.float32)
    s = np.ascontiguousarray(sun, np.float32)
    pkg._check(pkg.lib().ceres_render_f32(scene._h, b.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                          s.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), int(mode),
                                          px.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                          rgb.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), W, H, ctypes.byref(st)))
    return px, rgb, (st.rays, st.hits)


def _device_render(pkg, scene, b12, sun, W, H, mode):
    import torch
    px = torch.empty(3 * W * H, dtype=torch.float32, device="cuda")
    rgb = torch.empty(3 * W * H, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    scene.render_device(b12, sun, W, H, mode=mode, d_pixels=px.data_ptr(), d_rgb8=rgb.data_ptr(), d_counters=cnt.data_ptr())
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    return px.cpu().numpy(), rgb.cpu().numpy(), (int(c[0]), int(c[1]))


def test_compacted_readback_equals_device_framebuffer(gpu):
    pkg = gpu
    cfg = configs.CONFIGS["bunny_1080"]
    mesh, bvh, cam = pkg.prepare(cfg, arith=1)
    scene = pkg.Scene(mesh, bvh)
    mode = pkg.cfg_mode(cfg, 1)
    W, H = 480, 272
    sparse = cam.basis(W, H)
    # a close-up that fills the frame with the sun behind the camera: ~90 % of the pixels lit (the
    # full-copy path on the following calls)
    close = pkg.Camera(np.float32([0.015, 0.11, -0.12]), cfg["dir"], cfg["up"], 40.0, arith=1).basis(W, H)
    views = [(sparse, cfg["sun"]), (close, (0.0, 0.1, -5.0))]
    lit_fracs = []
    for k, v in enumerate([0, 1, 1, 0, 0] + [0] * 30 + [1, 0]):
        b12, sun = views[v][0], np.asarray(views[v][1], np.float32)
        hp, hr, hc = _host_render(pkg, scene, b12, sun, W, H, mode)
        dp, dr, dc = _device_render(pkg, scene, b12, sun, W, H, mode)
        assert hc == dc, k
        assert np.array_equal(hp.view(np.uint32), dp.view(np.uint32)), k
        assert np.array_equal(hr, dr), k
        lit_fracs.append(float(np.mean(np.any(dp.reshape(-1, 3) != 0, axis=1))))
    assert min(lit_fracs) < 0.5 < max(lit_fracs), lit_fracs   # both paths taken
    scene.close()
