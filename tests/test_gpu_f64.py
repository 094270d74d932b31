"""render<double> on the GPU (render64.hip) against the reference's own double builds
(tests/golden/f64/, oracle/_ref/ref_render_f64{,_exact}): PPM sha256 equal, rays/hits equal, and
per-pixel hit records {prim, t, u, v, shadow} and colours bit-identical (t/u/v as doubles).
The shading's std::pow(double, 24) is evaluated as a correctly rounded x^24 and narrowed to
float like blinn_phong_spec's return type (render.hpp:52-54)."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

import configs

pytestmark = pytest.mark.gpu

F64 = os.path.join(GOLDEN, "f64")
NAMES = sorted(f[:-5] for f in os.listdir(F64) if f.endswith(".json"))


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


def _hex64(hx):
    return np.asarray([int(h, 16) for h in hx], np.uint64).view(np.float64)


def load(name, build="exact"):
    meta = json.load(open(os.path.join(F64, name + ".json")))
    rec = dict(np.load(os.path.join(F64, name + (".ref" if build == "ref" else "") + ".records.npz")))
    p = os.path.join(F64, name + ".exact.ppm.gz")
    ppm = gzip.decompress(open(p, "rb").read()) if os.path.exists(p) and build == "exact" else None
    return meta, rec, ppm


@pytest.mark.parametrize("build", ["exact", "ref"])
@pytest.mark.parametrize("name", NAMES)
def test_f64_frame_matches_reference(gpu, name, build):
    """build "exact": the -ffp-contract=off double build; "ref": the reference's own CMake build of
    anim.cpp -d (-O3 -mavx2 -mfma: GCC's FMA contraction; scene prepared with CERES_ARITH_FMA,
    rendered with CERES_MODE_FMA) -- round 5."""
    pkg = gpu
    meta, rec, ppm = load(name, build)
    cfg = configs.CONFIGS[name]
    arith = 1 if build == "ref" else 0
    mesh, bvh, _ = pkg.prepare(cfg, f64=True, arith=arith)
    scene = pkg.Scene(mesh, bvh)
    bb, pose = (meta["ref_basis"], meta["ref_pose"]) if build == "ref" else (meta["basis"], meta["pose"])
    basis = np.concatenate([_hex64(pose["eye"]), _hex64(bb["dir"] + bb["u"] + bb["v"])])
    sun = _hex64(pose["sun"])
    mode = (pkg.MODE_PRIMARY if cfg["mode"] == "primary" else pkg.MODE_FULL) | (pkg.MODE_FMA if arith else 0)
    W, H = cfg["W"], cfg["H"]
    px, rgb, st = scene.render(basis, sun, W, H, mode=mode)
    assert (st["rays"], st["hits"]) == (meta[build]["rays"], meta[build]["hits"])
    body = pkg.ppm(W, H, rgb)
    assert hashlib.sha256(body).hexdigest() == meta["ppm_sha256"][build]
    if ppm is not None:
        assert body == ppm
    pix = rec["pixel"].astype(np.int64)
    np.testing.assert_array_equal(px.reshape(-1, 3)[pix].view(np.uint64), rec["rgb"].view(np.uint64))
    prim, tuv, sh, st2 = scene.records(basis, sun, W, H, mode=mode)
    np.testing.assert_array_equal(prim[pix], rec["prim"])
    hit = rec["prim"] >= 0
    for k, key in enumerate("tuv"):
        np.testing.assert_array_equal(tuv[pix, k][hit].view(np.uint64), rec[key][hit].view(np.uint64))
    if mode & 0xf == pkg.MODE_FULL:
        np.testing.assert_array_equal(sh[pix], rec["shadow"])
    scene.close()


def test_f64_and_f32_scenes_reject_each_others_calls(gpu):
    pkg = gpu
    cfg = configs.CONFIGS["tri1"]
    m64, b64, c64 = pkg.prepare(cfg, f64=True)
    m32, b32, c32 = pkg.prepare(cfg)
    s64, s32 = pkg.Scene(m64, b64), pkg.Scene(m32, b32)
    import ctypes
    px = np.empty(3 * 16, np.float32)
    st = pkg._Stats()
    b = c32.basis(4, 4)
    with pytest.raises(pkg.CeresError):
        pkg._check(pkg.lib().ceres_render_f32(s64._h, pkg._p(b, ctypes.c_float), pkg._p(np.zeros(3, np.float32), ctypes.c_float),
                                              0, pkg._p(px, ctypes.c_float), None, 4, 4, ctypes.byref(st)))
    pxd = np.empty(3 * 16, np.float64)
    bd = c64.basis(4, 4)
    with pytest.raises(pkg.CeresError):
        pkg._check(pkg.lib().ceres_render_f64(s32._h, pkg._p(bd, ctypes.c_double), pkg._p(np.zeros(3), ctypes.c_double),
                                              0, pkg._p(pxd, ctypes.c_double), None, 4, 4, ctypes.byref(st)))
    s64.close()
    s32.close()


@pytest.mark.parametrize("name", ["bunny_640", "quad"])
@pytest.mark.parametrize("flag", ["", "--exact"])
def test_cli_double_writes_reference_ppm(gpu, tmp_path, name, flag):
    """./render --double (anim.cpp's -d): the reference's double-precision PPM, byte for byte -- by
    default the reference CMake build's (--fma), with --exact the contraction-free build's (quad:
    the two builds' PPMs differ by one byte)."""
    import subprocess
    pkg = gpu
    build = "exact" if flag else "ref"
    meta, _, _ = load(name)
    out = tmp_path / "b.ppm"
    args = configs.cli_args(configs.CONFIGS[name]) + ["--double", "-o", str(out)] + ([flag] if flag else [])
    r = subprocess.run([pkg.CLI_PATH] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Rays: %d\tHits: %d" % (meta[build]["rays"], meta[build]["hits"]) in r.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == meta["ppm_sha256"][build]


@pytest.mark.parametrize("contract", [False, True])
def test_dropin_render_hpp_double_runs(gpu, tmp_path, contract):
    """A static.cpp-style program with Scalar = double on include/ceres/render.hpp, compiled the
    contraction-free way and the way the reference's CMake build compiles anim.cpp (-O2 -mfma:
    CERES_DROPIN_ARITH = CERES_ARITH_FMA)."""
    import subprocess
    from conftest import REPO
    pkg = gpu
    meta, _, _ = load("dragon_333x217")
    src = tmp_path / "app.cpp"
    src.write_text(r'''
#include <cstdio>
#include <vector>
#include "ceres/render.hpp"
int main(int argc, char** argv) {
    double* tri; double* nrm; size_t n;
    if (ceres_obj_load_f64_arith(argv[1], &tri, &nrm, &n, CERES_DROPIN_ARITH)) return 3;
    rotate_triangles<0>(90.0, reinterpret_cast<ceres::HostTriangle64*>(tri), n);
    uint64_t* nodes; uint64_t* prim; size_t m;
    if (ceres_bvh_build_f64_arith(tri, n, &nodes, &m, &prim, CERES_DROPIN_ARITH)) return 4;
    ceres::HostBvh64 bvh;
    bvh.nodes.reset(new ceres::HostBvh64::Node[m]); std::memcpy(bvh.nodes.get(), nodes, 64 * m);
    bvh.primitive_indices.reset(new size_t[n]); std::memcpy(bvh.primitive_indices.get(), prim, 8 * n);
    bvh.node_count = m;
    Camera<double> cam{ceres::vec3<double>(0, -15, 2), ceres::vec3<double>(0, 1, 0), ceres::vec3<double>(0, 0, 1), 60};
    std::vector<double> px(3 * 333 * 217);
    auto rh = render(cam, ceres::vec3<double>(-50, -20, 0), bvh, reinterpret_cast<ceres::HostTriangle64*>(tri),
                     reinterpret_cast<std::array<ceres::vec3<double>, 3>*>(nrm), px.data(), 333, 217);
    std::printf("%d %d\n", rh.first, rh.second);
    return 0;
}
''')
    exe = tmp_path / "app"
    pkgdir = os.path.dirname(pkg.LIB_PATH)
    flags = ["-O2", "-mfma", "-DCERES_DROPIN_QUIET"] if contract else ["-O1"]
    r = subprocess.run(["g++", "-std=c++17", *flags, "-I" + os.path.join(REPO, "include"), str(src), "-o", str(exe),
                        "-L" + pkgdir, "-lceres_hip", "-Wl,-rpath," + pkgdir], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), os.path.join(REPO, "data", "dragon.obj")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    build = "ref" if contract else "exact"
    assert tuple(map(int, r.stdout.split())) == (meta[build]["rays"], meta[build]["hits"])
