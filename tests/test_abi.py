"""The C-ABI library loads, exports every symbol include/ceres_render.h declares, and fails
loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "ceres_render.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ceres_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_api(pkg):
    names = declared_functions()
    assert set(names) == set(pkg.EXPORTED_SYMBOLS), names


def test_library_exports_every_declared_symbol(pkg):
    L = ctypes.CDLL(pkg.LIB_PATH)
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(r"\bT %s\b" % name, out), name


def test_kernels_are_gfx950_code_objects(pkg):
    """The shipped .so carries gfx950 device code (hipcc --offload-arch=gfx950)."""
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"ceres_fused" in blob and b"ceres_primary" in blob


def test_no_cpu_fallback_without_gpu(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    mesh, bvh, _ = pkg.prepare(pkg.configs.CONFIGS["tri1"])
    with pytest.raises(pkg.CeresError):
        pkg.Scene(mesh, bvh)


def test_cli_usage_and_loud_failure(pkg):
    r = subprocess.run([pkg.CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    r = subprocess.run([pkg.CLI_PATH, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 2
    import torch
    if not torch.cuda.is_available():
        r = subprocess.run([pkg.CLI_PATH, os.path.join(REPO, "tests", "golden", "tri1.obj"), "--size", "8", "8",
                            "-o", os.devnull], capture_output=True, text=True)
        assert r.returncode == 1 and "error" in r.stderr


def test_dropin_header_compiles_with_own_types(tmp_path):
    """include/ceres/render.hpp compiles against the self-contained ceres:: types (render.hpp API)."""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include "ceres/render.hpp"
int main() {
    ceres::HostBvh bvh; std::vector<ceres::HostTriangle> tris(1);
    std::vector<std::array<ceres::vec3<float>, 3>> norms(1);
    Camera<float> cam{ceres::vec3<float>(0, -15, 2), ceres::vec3<float>(0, 1, 0), ceres::vec3<float>(0, 0, 1), 60};
    std::vector<float> px(3 * 4 * 4);
    rotate_triangles<0>(90.0f, tris.data(), tris.size());
    if (false) render(cam, ceres::vec3<float>(-50, -20, 0), bvh, tris.data(), norms.data(), px.data(), 4, 4);
    ceres::HostBvh64 bvh64; std::vector<ceres::HostTriangle64> tris64(1);
    std::vector<std::array<ceres::vec3<double>, 3>> norms64(1);
    Camera<double> cam64{ceres::vec3<double>(-150, -20, 0), ceres::vec3<double>(1, -0.1, 0), ceres::vec3<double>(0, -1, 0), 60};
    std::vector<double> px64(3 * 4 * 4);
    rotate_triangles<1>(45.0, tris64.data(), tris64.size());
    if (false) render(cam64, ceres::vec3<double>(-500, 300, 10), bvh64, tris64.data(), norms64.data(), px64.data(), 4, 4);
    return 0;
}
''')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I" + os.path.join(REPO, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("flags,warns", [(["-O2", "-mfma"], None), (["-O0", "-mfma"], "CERES_ARITH_EXACT"),
                                         (["-O2", "-mfma", "-DCERES_DROPIN_VERBOSE"], "CERES_ARITH_FMA"),
                                         (["-O2"], None),
                                         (["-O2", "-mfma", "-DCERES_DROPIN_ARITH=CERES_ARITH_EXACT"], None),
                                         (["-O0", "-mfma", "-DCERES_DROPIN_QUIET"], None)])
def test_dropin_auto_arith_warns(tmp_path, flags, warns):
    """the header cannot see -ffp-contract, so an AMBIGUOUS automatic choice with FMA
    enabled (no optimisation, or clang) is announced with a #warning naming the choice; the
    reference CMake configuration (GCC -O -mfma: FMA, the right pick) is silent unless
    CERES_DROPIN_VERBOSE asks, so -Werror builds of the default drop-in compile; an explicit
    CERES_DROPIN_ARITH (or CERES_DROPIN_QUIET) silences the rest, and without FMA there is nothing
    to guess."""
    src = tmp_path / "w.cpp"
    src.write_text('#include "ceres/render.hpp"\nint main() { return CERES_DROPIN_ARITH; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", *flags, "-I" + os.path.join(REPO, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    if warns is None:
        assert "#warning" not in r.stderr and "warning" not in r.stderr, r.stderr
    else:
        assert "auto-selected " + warns in r.stderr, r.stderr


@pytest.mark.skipif(not os.path.isdir("/root/reference/lib/bvh"), reason="reference sources only in the build container")
def test_dropin_header_compiles_with_reference_types(tmp_path):
    """Drop-in proof: the reference's own static.cpp call pattern compiles against ceres/render.hpp
    with the reference's lib/bvh types (read in place, nothing copied)."""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include <bvh/bvh.hpp>
#include <bvh/triangle.hpp>
#include "ceres/render.hpp"
using Scalar = float;
using Vector3 = bvh::Vector3<Scalar>;
int main() {
    bvh::Bvh<Scalar> bvh; std::vector<bvh::Triangle<Scalar>> triangles(1);
    std::vector<std::array<Vector3, 3>> tri_norms(1);
    Camera<Scalar> camera = { Vector3(0.0, -15.0, 2.0), Vector3(0, 1, 0), Vector3(0, 0, 1), 60 };   // static.cpp:39-44
    Vector3 sun_position = Vector3(-50.0, -20.0, 0.0);
    rotate_triangles<0>(Scalar(90), triangles.data(), triangles.size());
    std::vector<Scalar> pixels(3 * 16);
    if (false) { auto [rays, hits] = render(camera, sun_position, bvh, triangles.data(), tri_norms.data(), pixels.data(), 4, 4); (void)rays; (void)hits; }
    Vector3 e = camera.eye; (void)e;    // anim.cpp:87 style round trip
    return 0;
}
''')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I/root/reference/lib", "-I" + os.path.join(REPO, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # anim.cpp -d: the same calls with Scalar = double (anim.cpp:146-155, camera as double literals)
    src.write_text(src.read_text().replace("using Scalar = float;", "using Scalar = double;")
                   .replace("Vector3(0.0, -15.0, 2.0), Vector3(0, 1, 0), Vector3(0, 0, 1)",
                            "Vector3(-150.0, -20.0, 0.0), Vector3(1, -0.1, 0), Vector3(0, -1, 0)"))
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I/root/reference/lib", "-I" + os.path.join(REPO, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_scene_accepts_leaf_too_large_for_packed_word(pkg):
    """The shadow BVH4 packs a child in one word (Node4::child: first << 5 | count, at most 31
    triangles), but the reference builder makes bigger leaves when centroids cannot be split
    (binned_sah_builder.hpp:199-232).  Such a leaf becomes a node of equal-box pieces, so the host
    layout accepts it: without a GPU, scene creation gets past the relayout and the BVH4 and fails
    only at the device step.  (The GPU parity of such scenes: the `dupleaf` fixture.)"""
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_parity.py (dupleaf)")
    n = 41
    tri = np.zeros((n, 12), np.float32)                  # {p0, e1, e2, n}: any finite values
    tri[:, 3] = 1.0
    tri[:, 8] = 1.0
    nor = np.zeros((n, 9), np.float32)
    nodes = np.zeros(3, dtype=[("b", np.float32, 6), ("count", np.uint32), ("first", np.uint32)])
    nodes["b"][:] = [-1, 1, -1, 1, -1, 1]
    nodes[0]["count"], nodes[0]["first"] = 0, 1           # root: children 1 and 2
    nodes[1]["count"], nodes[1]["first"] = 40, 0          # a leaf of 40 triangles
    nodes[2]["count"], nodes[2]["first"] = 1, 40
    prim = np.arange(n, dtype=np.uint64)
    L = pkg.lib()
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))     # noqa: E731
    h = L.ceres_scene_create(fp(tri), n, fp(nor), nodes.ctypes.data_as(ctypes.c_void_p), 3,
                             prim.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0, 0)
    assert not h
    err = L.ceres_last_error()
    assert b"BVH4" not in err and b"device" in err, err


def test_scene_accepts_big_leaf_beside_uncollapsed_inner_pairs(pkg):
    """the shadow BVH4's tree check must not count piece nodes.  Root = {a leaf of 1000
    coincident-centroid triangles (-> ~20 piece nodes), an inner node whose two children are inner
    nodes again}: 4 sibling pairs, 3 collapsed records + the pieces.  Without a GPU, scene creation
    gets past the relayout and the BVH4 (no "do not form a tree") and fails only at the device step."""
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    n = 1004
    tri = np.zeros((n, 12), np.float32)
    tri[:, 3] = 1.0
    tri[:, 8] = 1.0
    nor = np.zeros((n, 9), np.float32)
    nodes = np.zeros(9, dtype=[("b", np.float32, 6), ("count", np.uint32), ("first", np.uint32)])
    nodes["b"][:] = [-1, 1, -1, 1, -1, 1]
    nodes[0]["first"] = 1                                         # root -> 1, 2
    nodes[1]["count"], nodes[1]["first"] = 1000, 0                # the big leaf
    nodes[2]["first"] = 3                                         # inner -> 3, 4 (both inner)
    nodes[3]["first"] = 5
    nodes[4]["first"] = 7
    for k, first in zip((5, 6, 7, 8), (1000, 1001, 1002, 1003)):
        nodes[k]["count"], nodes[k]["first"] = 1, first
    prim = np.arange(n, dtype=np.uint64)
    L = pkg.lib()
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))     # noqa: E731
    h = L.ceres_scene_create(fp(tri), n, fp(nor), nodes.ctypes.data_as(ctypes.c_void_p), nodes.shape[0],
                             prim.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0, 0)
    assert not h
    err = L.ceres_last_error()
    assert b"tree" not in err and b"BVH4" not in err and b"device" in err, err


def test_content_hash(pkg):
    """ceres_content_hash (the drop-in's per-call scene check): deterministic, and any single changed
    byte -- in a full 32-B block, in the <32-B tail, in any 256-KiB chunk -- changes it."""
    import numpy as np
    L = pkg.lib()
    rng = np.random.default_rng(7)
    for size in (1, 7, 31, 33, 1000, (256 << 10) + 5, 3 << 20):
        a = rng.integers(0, 256, size, dtype=np.uint8)
        h0 = L.ceres_content_hash(a.ctypes.data_as(ctypes.c_void_p), size)
        assert h0 == L.ceres_content_hash(a.ctypes.data_as(ctypes.c_void_p), size)
        for pos in {0, size // 2, size - 1, max(0, size - 9)}:
            b = a.copy()
            b[pos] ^= 1
            assert L.ceres_content_hash(b.ctypes.data_as(ctypes.c_void_p), size) != h0, (size, pos)
        if size > 1:
            assert L.ceres_content_hash(a.ctypes.data_as(ctypes.c_void_p), size - 1) != h0
