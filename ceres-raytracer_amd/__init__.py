"""ceres_raytracer_amd -- MI355X-native CERES hot path, Python host mirror over the C ABI.

This module mirrors the reference's render interface (include/render.hpp of
iracigt/ceres-raytracer) for Python callers, tests and bench.py:

    Camera(eye, dir, up, fov)                 render.hpp:16-22
    load_obj(path) -> Mesh                    obj_norms.hpp:120-127 (triangles + tri_norms)
    rotate_triangles(mesh, axis, degrees)     render.hpp:24-44
    build_bvh(mesh) -> Bvh                    binned_sah_builder.hpp:39-234 (static.cpp:100-107)
    build_bvh_gpu(mesh) -> Bvh                the same BVH, built by gfx950 kernels
    Scene(mesh, bvh, device)                  the (bvh, triangles, tri_norms) arguments, on the GPU
    render(camera, sun, scene, W, H) -> (pixels, rays, hits)   render.hpp:86-156

Everything runs through libceres_hip.so (include/ceres_render.h): host scene preparation in
C++, the hot path in hand-written gfx950 HIP kernels.  There is no CPU fallback: rendering
without the library or without a gfx950 device raises CeresError.
"""
import ctypes
import os
import sys

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# CERES_LIB: an A/B build of the same library (tools/ab.py, `make variant`); default the in-tree one
LIB_PATH = os.environ.get("CERES_LIB") or os.path.join(_PKG, "libceres_hip.so")
CLI_PATH = os.path.join(_PKG, "render")

if _PKG not in sys.path:
    sys.path.insert(0, _PKG)
import configs  # noqa: E402,F401  (re-exported)

MODE_FULL, MODE_PRIMARY = 0, 1
MODE_ROBUST = 0x10          # OR-ed: RobustNodeIntersector traversal (node_intersectors.hpp:54-79)
MODE_QBVH4 = 0x20           # OR-ed: compressed shadow BVH4 (8-bit child bounds; budget-gated, not exact)
MODE_FMA = 0x40             # OR-ed: the reference CMake build's arithmetic (GCC FMA contraction)
# Arithmetic of the host scene prep (CERES_ARITH_*): the reference without contraction, or as its
# own CMake build (g++ -O3 -mavx2 -mfma) compiles it; pair ARITH_FMA scenes with MODE_FMA renders
ARITH_EXACT, ARITH_FMA = 0, 1


def cfg_mode(cfg, arith=ARITH_EXACT):
    """The C-ABI mode of a configs.CONFIGS entry (| MODE_FMA for the reference-flag arithmetic)."""
    return ((MODE_PRIMARY if cfg["mode"] == "primary" else MODE_FULL) | (MODE_ROBUST if cfg.get("robust") else 0)
            | (MODE_FMA if arith else 0))
SCENE_STATS = 1
SCENE_FIRST_ORDER = 2

EXPORTED_SYMBOLS = (
    "ceres_obj_load", "ceres_proc_mesh", "ceres_rotate_triangles", "ceres_bvh_build", "ceres_bvh_build_gpu",
    "ceres_bvh_build_device", "ceres_obj_load_gpu", "ceres_obj_parse_device", "ceres_rotate_triangles_device",
    "ceres_device_free", "ceres_camera_basis", "ceres_obj_load_f64", "ceres_proc_mesh_f64", "ceres_rotate_triangles_f64",
    "ceres_bvh_build_f64", "ceres_camera_basis_f64", "ceres_orbit_cameras_f64", "ceres_scene_create_f64",
    "ceres_render_f64", "ceres_render_records_f64", "ceres_obj_load_f64_arith", "ceres_proc_mesh_f64_arith",
    "ceres_rotate_triangles_f64_arith", "ceres_bvh_build_f64_arith", "ceres_camera_basis_f64_arith",
    "ceres_orbit_cameras_f64_arith",
    "ceres_free", "ceres_scene_create", "ceres_scene_create_device", "ceres_scene_destroy", "ceres_scene_info", "ceres_scene_shadow_stacks", "ceres_render_f32",
    "ceres_render_device", "ceres_render_batch_device", "ceres_render_multi_f32", "ceres_device_count", "ceres_assemble_rgb8_packed", "ceres_render_records", "ceres_tiling_local_rows",
    "ceres_scene_set_timing", "ceres_scene_read_timing", "ceres_scene_wave_log", "ceres_fetch_counters",
    "ceres_cpu_scene_create", "ceres_cpu_scene_destroy", "ceres_render_cpu_f32", "ceres_cpu_scene_create_f64",
    "ceres_render_cpu_f64",
    "ceres_orbit_cameras", "ceres_assemble_rgb8",
    "ceres_kernel_names", "ceres_last_error", "ceres_version",
    "ceres_obj_load_arith", "ceres_proc_mesh_arith", "ceres_rotate_triangles_arith", "ceres_bvh_build_arith",
    "ceres_camera_basis_arith", "ceres_orbit_cameras_arith", "ceres_content_hash",
    "ceres_bvh_build_gpu_arith", "ceres_bvh_build_device_arith", "ceres_obj_load_gpu_arith",
    "ceres_obj_parse_device_arith", "ceres_rotate_triangles_device_arith",
)


class CeresError(RuntimeError):
    pass


class _Stats(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_uint64), ("hits", ctypes.c_uint64), ("primary_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("node_pairs", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64),
                ("ms", ctypes.c_double)]


class Tiling(ctypes.Structure):
    """ceres_tiling: bands = 0 -- row blocks dealt round-robin; bands = 1 -- frame f of a call renders
    the contiguous band (rank + f) mod world of row_block rows (distributed.FrameBands)."""
    _fields_ = [("row_block", ctypes.c_uint32), ("rank", ctypes.c_uint32), ("world", ctypes.c_uint32),
                ("bands", ctypes.c_uint32)]


_lib = None
_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p


def build(verbose=False):
    """Compile libceres_hip.so and ./render for gfx950 (hipcc), in-tree."""
    import subprocess
    r = subprocess.run(["make", "-C", os.path.join(_PKG, "csrc"), "-j4", "all"], capture_output=True, text=True)
    if verbose or r.returncode:
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr)
    if r.returncode:
        raise CeresError("build of libceres_hip.so failed")


def lib():
    """Load libceres_hip.so (import torch first when present so one HIP runtime is shared)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CeresError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    L.ceres_last_error.restype = ctypes.c_char_p
    L.ceres_version.restype = ctypes.c_char_p
    L.ceres_kernel_names.restype = ctypes.c_char_p
    L.ceres_obj_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz)]
    L.ceres_proc_mesh.argtypes = [ctypes.c_int, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz)]
    L.ceres_rotate_triangles.argtypes = [_fp, _sz, ctypes.c_int, ctypes.c_float]
    L.ceres_bvh_build.argtypes = [_fp, _sz, ctypes.POINTER(_u32p), ctypes.POINTER(_sz), ctypes.POINTER(_u64p)]
    L.ceres_bvh_build_gpu.argtypes = [_fp, _sz, ctypes.POINTER(_u32p), ctypes.POINTER(_sz), ctypes.POINTER(_u64p),
                                      ctypes.c_int]
    L.ceres_bvh_build_device.argtypes = [_vp, _sz, _vp, _vp, ctypes.POINTER(_sz), _vp]
    L.ceres_obj_load_gpu.argtypes = [ctypes.c_char_p, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz),
                                     ctypes.c_int]
    L.ceres_obj_parse_device.argtypes = [_vp, _sz, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_sz), _vp]
    L.ceres_rotate_triangles_device.argtypes = [_vp, _sz, ctypes.c_int, ctypes.c_float, _vp]
    L.ceres_device_free.argtypes = [_vp]
    L.ceres_device_free.restype = None
    L.ceres_camera_basis.argtypes = [_fp, _fp, _fp, ctypes.c_float, _sz, _sz, _fp]
    L.ceres_obj_load_f64.argtypes = [ctypes.c_char_p, ctypes.POINTER(_dp), ctypes.POINTER(_dp), ctypes.POINTER(_sz)]
    L.ceres_proc_mesh_f64.argtypes = [ctypes.c_int, ctypes.POINTER(_dp), ctypes.POINTER(_dp), ctypes.POINTER(_sz)]
    L.ceres_rotate_triangles_f64.argtypes = [_dp, _sz, ctypes.c_int, ctypes.c_double]
    L.ceres_bvh_build_f64.argtypes = [_dp, _sz, ctypes.POINTER(_u64p), ctypes.POINTER(_sz), ctypes.POINTER(_u64p)]
    L.ceres_camera_basis_f64.argtypes = [_dp, _dp, _dp, ctypes.c_double, _sz, _sz, _dp]
    L.ceres_orbit_cameras_f64.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, _sz, _sz, _dp, ctypes.c_double,
                                          ctypes.c_uint32, ctypes.c_int, _dp, _dp, _dp]
    L.ceres_obj_load_f64_arith.argtypes = [ctypes.c_char_p, ctypes.POINTER(_dp), ctypes.POINTER(_dp), ctypes.POINTER(_sz),
                                           ctypes.c_int]
    L.ceres_proc_mesh_f64_arith.argtypes = [ctypes.c_int, ctypes.POINTER(_dp), ctypes.POINTER(_dp), ctypes.POINTER(_sz),
                                            ctypes.c_int]
    L.ceres_rotate_triangles_f64_arith.argtypes = [_dp, _sz, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    L.ceres_bvh_build_f64_arith.argtypes = [_dp, _sz, ctypes.POINTER(_u64p), ctypes.POINTER(_sz), ctypes.POINTER(_u64p),
                                            ctypes.c_int]
    L.ceres_camera_basis_f64_arith.argtypes = [_dp, _dp, _dp, ctypes.c_double, _sz, _sz, _dp, ctypes.c_int]
    L.ceres_orbit_cameras_f64_arith.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, _sz, _sz, _dp, ctypes.c_double,
                                                ctypes.c_uint32, ctypes.c_int, _dp, _dp, _dp, ctypes.c_int]
    L.ceres_scene_create_f64.argtypes = [_dp, _sz, _dp, _vp, _sz, _u64p, ctypes.c_int, ctypes.c_uint32]
    L.ceres_scene_create_f64.restype = _vp
    L.ceres_render_f64.argtypes = [_vp, _dp, _dp, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_uint8), _sz, _sz,
                                   ctypes.POINTER(_Stats)]
    L.ceres_render_records_f64.argtypes = [_vp, _dp, _dp, ctypes.c_int, _sz, _sz, ctypes.POINTER(ctypes.c_int32), _dp,
                                           ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(_Stats)]
    L.ceres_orbit_cameras.argtypes = [_fp, _fp, _fp, _fp, ctypes.c_float, _sz, _sz, _fp, ctypes.c_float,
                                      ctypes.c_uint32, ctypes.c_int, _fp, _fp, _fp]
    L.ceres_free.argtypes = [_vp]
    L.ceres_free.restype = None
    L.ceres_scene_create.argtypes = [_fp, _sz, _fp, _vp, _sz, _u64p, ctypes.c_int, ctypes.c_uint32]
    L.ceres_scene_create.restype = _vp
    L.ceres_scene_create_device.argtypes = [_vp, _sz, _vp, _vp, _sz, _vp, ctypes.c_int, ctypes.c_uint32, _vp]
    L.ceres_scene_create_device.restype = _vp
    L.ceres_scene_destroy.argtypes = [_vp]
    L.ceres_scene_destroy.restype = None
    L.ceres_scene_info.argtypes = [_vp, _u32p, _u32p, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]
    L.ceres_scene_shadow_stacks.argtypes = [_vp, _u32p, _u32p]
    L.ceres_render_f32.argtypes = [_vp, _fp, _fp, ctypes.c_int, _fp, ctypes.POINTER(ctypes.c_uint8), _sz, _sz,
                                   ctypes.POINTER(_Stats)]
    L.ceres_render_device.argtypes = [_vp, _fp, _fp, ctypes.c_int, _sz, _sz, ctypes.POINTER(Tiling), _vp, _vp, _vp, _vp]
    L.ceres_render_batch_device.argtypes = [_vp, ctypes.c_uint32, _fp, _fp, ctypes.c_int, _sz, _sz,
                                            ctypes.POINTER(Tiling), _vp, _vp, _vp, _vp]
    L.ceres_render_multi_f32.argtypes = [ctypes.POINTER(_vp), ctypes.c_uint32, ctypes.c_uint32, _fp, _fp, ctypes.c_int, _fp,
                                         ctypes.POINTER(ctypes.c_uint8), _sz, _sz, ctypes.POINTER(_Stats)]
    L.ceres_assemble_rgb8_packed.argtypes = [_vp, _vp, ctypes.c_uint32, _sz, _sz, ctypes.c_uint32, ctypes.c_uint32, _vp]
    L.ceres_assemble_rgb8.argtypes = [_vp, _sz, _vp, ctypes.c_uint32, _sz, _sz, ctypes.c_uint32, ctypes.c_uint32, _vp]
    L.ceres_render_records.argtypes = [_vp, _fp, _fp, ctypes.c_int, _sz, _sz, ctypes.POINTER(ctypes.c_int32), _fp,
                                       ctypes.POINTER(ctypes.c_int8), ctypes.POINTER(_Stats)]
    L.ceres_tiling_local_rows.argtypes = [_sz, ctypes.POINTER(Tiling)]
    L.ceres_tiling_local_rows.restype = _sz
    L.ceres_scene_set_timing.argtypes = [_vp, ctypes.c_int]
    L.ceres_scene_read_timing.argtypes = [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          _u64p]
    L.ceres_scene_wave_log.argtypes = [_vp, _u64p, _sz, ctypes.POINTER(_sz)]
    L.ceres_fetch_counters.argtypes = [ctypes.c_int, _u64p, ctypes.c_int]
    L.ceres_cpu_scene_create.argtypes = [_fp, _sz, _fp, _vp, _sz, _u64p]
    L.ceres_cpu_scene_create.restype = _vp
    L.ceres_cpu_scene_destroy.argtypes = [_vp]
    L.ceres_cpu_scene_destroy.restype = None
    L.ceres_render_cpu_f32.argtypes = [_vp, _fp, _fp, ctypes.c_int, _fp, ctypes.POINTER(ctypes.c_uint8), _sz, _sz,
                                       ctypes.POINTER(_Stats), ctypes.c_int]
    L.ceres_cpu_scene_create_f64.argtypes = [_dp, _sz, _dp, _vp, _sz, _u64p]
    L.ceres_cpu_scene_create_f64.restype = _vp
    L.ceres_render_cpu_f64.argtypes = [_vp, _dp, _dp, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_uint8), _sz, _sz,
                                       ctypes.POINTER(_Stats), ctypes.c_int]
    L.ceres_content_hash.argtypes = [_vp, _sz]
    L.ceres_content_hash.restype = ctypes.c_uint64
    L.ceres_obj_load_arith.argtypes = L.ceres_obj_load.argtypes + [ctypes.c_int]
    L.ceres_proc_mesh_arith.argtypes = L.ceres_proc_mesh.argtypes + [ctypes.c_int]
    L.ceres_rotate_triangles_arith.argtypes = L.ceres_rotate_triangles.argtypes + [ctypes.c_int]
    L.ceres_bvh_build_arith.argtypes = L.ceres_bvh_build.argtypes + [ctypes.c_int]
    L.ceres_camera_basis_arith.argtypes = L.ceres_camera_basis.argtypes + [ctypes.c_int]
    L.ceres_orbit_cameras_arith.argtypes = L.ceres_orbit_cameras.argtypes + [ctypes.c_int]
    L.ceres_bvh_build_gpu_arith.argtypes = L.ceres_bvh_build_gpu.argtypes + [ctypes.c_int]
    L.ceres_bvh_build_device_arith.argtypes = L.ceres_bvh_build_device.argtypes + [ctypes.c_int]
    L.ceres_obj_load_gpu_arith.argtypes = L.ceres_obj_load_gpu.argtypes + [ctypes.c_int]
    L.ceres_obj_parse_device_arith.argtypes = L.ceres_obj_parse_device.argtypes + [ctypes.c_int]
    L.ceres_rotate_triangles_device_arith.argtypes = L.ceres_rotate_triangles_device.argtypes + [ctypes.c_int]
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise CeresError(f"ceres error {rc}: {lib().ceres_last_error().decode()}")


def _p(a, t):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(t))


def _take(ptr, count, dtype):
    if count == 0:
        lib().ceres_free(ctypes.cast(ptr, _vp))
        return np.zeros(0, dtype)
    a = np.ctypeslib.as_array(ptr, shape=(count,)).copy().view(dtype)
    lib().ceres_free(ctypes.cast(ptr, _vp))
    return a


class Camera:
    """render.hpp:16-22 -- eye, dir, up, fov (degrees); Camera<float> or, with dtype=np.float64,
    Camera<double> (anim.cpp -d)."""

    def __init__(self, eye, dir, up, fov, dtype=np.float32, arith=ARITH_EXACT):
        self.dtype = np.dtype(dtype)
        self.eye = np.asarray(eye, self.dtype)
        self.dir = np.asarray(dir, self.dtype)
        self.up = np.asarray(up, self.dtype)
        self.fov = float(fov)
        self.arith = int(arith)                      # float cameras: CERES_ARITH_* of the basis

    def basis(self, W, H):
        """render.hpp:91-97 on the host (libm stays on the host): {eye, dir, image_u, image_v}."""
        if self.dtype == np.float64:
            out = np.zeros(9, np.float64)
            _check(lib().ceres_camera_basis_f64_arith(_p(self.eye, ctypes.c_double), _p(self.dir, ctypes.c_double),
                                                      _p(self.up, ctypes.c_double), self.fov, W, H,
                                                      _p(out, ctypes.c_double), self.arith))
            return np.concatenate([self.eye, out])
        out = np.zeros(9, np.float32)
        _check(lib().ceres_camera_basis_arith(_p(self.eye, ctypes.c_float), _p(self.dir, ctypes.c_float),
                                              _p(self.up, ctypes.c_float), self.fov, W, H, _p(out, ctypes.c_float),
                                              self.arith))
        return np.concatenate([self.eye, out]).astype(np.float32)


class Mesh:
    """Triangles (n x 12 = bvh::Triangle<S>) and per-triangle vertex normals (n x 9); S = float
    (f32 arrays) or double (f64 arrays, render<double>)."""

    def __init__(self, tri, norm):
        dt = np.float64 if np.asarray(tri).dtype == np.float64 else np.float32
        self.tri = np.ascontiguousarray(tri, dt).reshape(-1, 12)
        self.norm = np.ascontiguousarray(norm, dt).reshape(-1, 9)

    @property
    def f64(self):
        return self.tri.dtype == np.float64

    def __len__(self):
        return self.tri.shape[0]


class Bvh:
    """bvh::Bvh<S>: nodes (m x 8 u32 = Node<float>, or m x 8 u64 = Node<double>: 6 doubles +
    2 u64) and primitive_indices (u64)."""

    def __init__(self, nodes, prim):
        dt = np.uint64 if np.asarray(nodes).dtype == np.uint64 else np.uint32
        self.nodes = np.ascontiguousarray(nodes, dt).reshape(-1, 8)
        self.prim = np.ascontiguousarray(prim, np.uint64)


def load_obj(path, arith=ARITH_EXACT):
    t, n, cnt = _fp(), _fp(), _sz()
    _check(lib().ceres_obj_load_arith(os.fsencode(path), ctypes.byref(t), ctypes.byref(n), ctypes.byref(cnt), int(arith)))
    c = cnt.value
    return Mesh(_take(t, c * 12, np.float32).reshape(c, 12), _take(n, c * 9, np.float32).reshape(c, 9))


def load_obj_f64(path, arith=ARITH_EXACT):
    """obj::load_from_file<double> (anim.cpp -d): strtof coordinates widened to double."""
    t, n, cnt = _dp(), _dp(), _sz()
    _check(lib().ceres_obj_load_f64_arith(os.fsencode(path), ctypes.byref(t), ctypes.byref(n), ctypes.byref(cnt),
                                          int(arith)))
    c = cnt.value
    return Mesh(_take(t, c * 12, np.float64).reshape(c, 12), _take(n, c * 9, np.float64).reshape(c, 9))


def proc_mesh_f64(n, arith=ARITH_EXACT):
    t, nn, cnt = _dp(), _dp(), _sz()
    _check(lib().ceres_proc_mesh_f64_arith(int(n), ctypes.byref(t), ctypes.byref(nn), ctypes.byref(cnt), int(arith)))
    c = cnt.value
    return Mesh(_take(t, c * 12, np.float64).reshape(c, 12), _take(nn, c * 9, np.float64).reshape(c, 9))


def load_obj_gpu(path, device=0, arith=ARITH_EXACT):
    """load_obj with the text parsed on the GPU (ceres_obj_load_gpu): the same bits."""
    t, n, cnt = _fp(), _fp(), _sz()
    _check(lib().ceres_obj_load_gpu_arith(os.fsencode(path), ctypes.byref(t), ctypes.byref(n), ctypes.byref(cnt),
                                          int(device), int(arith)))
    c = cnt.value
    return Mesh(_take(t, c * 12, np.float32).reshape(c, 12), _take(n, c * 9, np.float32).reshape(c, 9))


def parse_obj_device(d_text, length, stream=0, arith=ARITH_EXACT):
    """ceres_obj_parse_device on a device text buffer (int pointer): returns (d_tri48, d_norm36, n_tri)
    device pointers (free with device_free)."""
    t, n, cnt = _vp(), _vp(), _sz()
    _check(lib().ceres_obj_parse_device_arith(d_text, length, ctypes.byref(t), ctypes.byref(n), ctypes.byref(cnt),
                                              stream or None, int(arith)))
    return t.value or 0, n.value or 0, cnt.value


def rotate_triangles_device(d_tri48, n_tri, axis, degrees, stream=0, arith=ARITH_EXACT):
    ax = {"x": 0, "y": 1, "z": 2}[axis] if isinstance(axis, str) else int(axis)
    _check(lib().ceres_rotate_triangles_device_arith(d_tri48, n_tri, ax, float(degrees), stream or None, int(arith)))


def device_free(d_ptr):
    lib().ceres_device_free(d_ptr or None)


def proc_mesh(n, arith=ARITH_EXACT):
    t, nn, cnt = _fp(), _fp(), _sz()
    _check(lib().ceres_proc_mesh_arith(int(n), ctypes.byref(t), ctypes.byref(nn), ctypes.byref(cnt), int(arith)))
    c = cnt.value
    return Mesh(_take(t, c * 12, np.float32).reshape(c, 12), _take(nn, c * 9, np.float32).reshape(c, 9))


def rotate_triangles(mesh, axis, degrees, arith=ARITH_EXACT):
    ax = {"x": 0, "y": 1, "z": 2}[axis] if isinstance(axis, str) else int(axis)
    if mesh.f64:
        _check(lib().ceres_rotate_triangles_f64_arith(_p(mesh.tri, ctypes.c_double), len(mesh), ax, float(degrees),
                                                      int(arith)))
    else:
        _check(lib().ceres_rotate_triangles_arith(_p(mesh.tri, ctypes.c_float), len(mesh), ax, float(degrees),
                                                  int(arith)))
    return mesh


def build_bvh(mesh, arith=ARITH_EXACT):
    if mesh.f64:
        nodes, prim, m = _u64p(), _u64p(), _sz()
        _check(lib().ceres_bvh_build_f64_arith(_p(mesh.tri, ctypes.c_double), len(mesh), ctypes.byref(nodes),
                                               ctypes.byref(m), ctypes.byref(prim), int(arith)))
        return Bvh(_take(nodes, m.value * 8, np.uint64).reshape(-1, 8), _take(prim, len(mesh), np.uint64))
    nodes, prim, m = _u32p(), _u64p(), _sz()
    _check(lib().ceres_bvh_build_arith(_p(mesh.tri, ctypes.c_float), len(mesh), ctypes.byref(nodes), ctypes.byref(m),
                                       ctypes.byref(prim), int(arith)))
    return Bvh(_take(nodes, m.value * 8, np.uint32).reshape(-1, 8), _take(prim, len(mesh), np.uint64))


def build_bvh_gpu(mesh, device=0, arith=ARITH_EXACT):
    """The same binned-SAH BVH as build_bvh, built on the GPU (ceres_bvh_build_gpu)."""
    nodes, prim, m = _u32p(), _u64p(), _sz()
    _check(lib().ceres_bvh_build_gpu_arith(_p(mesh.tri, ctypes.c_float), len(mesh), ctypes.byref(nodes),
                                           ctypes.byref(m), ctypes.byref(prim), int(device), int(arith)))
    return Bvh(_take(nodes, m.value * 8, np.uint32).reshape(-1, 8), _take(prim, len(mesh), np.uint64))


def build_bvh_device(d_tri48, n_tri, d_nodes32, d_prim32, stream=0, arith=ARITH_EXACT):
    """ceres_bvh_build_device on device pointers (ints); returns the node count."""
    m = _sz()
    _check(lib().ceres_bvh_build_device_arith(d_tri48, n_tri, d_nodes32, d_prim32, ctypes.byref(m), stream or None,
                                              int(arith)))
    return m.value


class CpuScene:
    """The CPU path's scene (ceres_cpu_scene_create): render<float>() on host cores, chosen
    explicitly (./render --cpu); the GPU classes never fall back to it."""

    def __init__(self, mesh, bvh):
        L = lib()
        self.f64 = mesh.f64
        if self.f64:
            self._h = L.ceres_cpu_scene_create_f64(_p(mesh.tri, ctypes.c_double), len(mesh), _p(mesh.norm, ctypes.c_double),
                                                   bvh.nodes.ctypes.data_as(_vp), bvh.nodes.shape[0],
                                                   _p(bvh.prim, ctypes.c_uint64))
        else:
            self._h = L.ceres_cpu_scene_create(_p(mesh.tri, ctypes.c_float), len(mesh), _p(mesh.norm, ctypes.c_float),
                                               bvh.nodes.ctypes.data_as(_vp), bvh.nodes.shape[0],
                                               _p(bvh.prim, ctypes.c_uint64))
        if not self._h:
            raise CeresError("ceres_cpu_scene_create: " + L.ceres_last_error().decode())

    def close(self):
        if getattr(self, "_h", None):
            lib().ceres_cpu_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, basis12, sun, W, H, mode=MODE_FULL, threads=0, want_pixels=True, want_rgb8=True):
        """ceres_render_cpu_f32 / _f64: (pixels [H*W*3] f32|f64 | None, rgb8 | None, stats dict)."""
        dt, ct = (np.float64, ctypes.c_double) if self.f64 else (np.float32, ctypes.c_float)
        b = np.ascontiguousarray(basis12, dt)
        s = np.ascontiguousarray(sun, dt)
        px = np.empty(3 * W * H, dt) if want_pixels else None
        rgb = np.empty(3 * W * H, np.uint8) if want_rgb8 else None
        st = _Stats()
        fn = lib().ceres_render_cpu_f64 if self.f64 else lib().ceres_render_cpu_f32
        _check(fn(self._h, _p(b, ct), _p(s, ct), int(mode), _p(px, ct), _p(rgb, ctypes.c_uint8), W, H, ctypes.byref(st),
                  int(threads)))
        return px, rgb, dict(rays=st.rays, hits=st.hits, primary_rays=st.primary_rays, shadow_rays=st.shadow_rays,
                             node_pairs=st.node_pairs, tri_tests=st.tri_tests, ms=st.ms)


class Scene:
    """A scene resident in HBM of one device (ceres_scene_create)."""

    def __init__(self, mesh, bvh, device=0, stats=False, first_order=False, _handle=None):
        L = lib()
        if _handle is not None:                      # Scene.from_device
            self._h, self.device, self.n_tri = _handle
            self.f64 = False
            return
        self.f64 = mesh.f64
        flags = (SCENE_STATS if stats else 0) | (SCENE_FIRST_ORDER if first_order else 0)
        if self.f64:
            self._h = L.ceres_scene_create_f64(_p(mesh.tri, ctypes.c_double), len(mesh), _p(mesh.norm, ctypes.c_double),
                                               bvh.nodes.ctypes.data_as(_vp), bvh.nodes.shape[0],
                                               _p(bvh.prim, ctypes.c_uint64), int(device), flags)
        else:
            self._h = L.ceres_scene_create(_p(mesh.tri, ctypes.c_float), len(mesh), _p(mesh.norm, ctypes.c_float),
                                           bvh.nodes.ctypes.data_as(_vp), bvh.nodes.shape[0],
                                           _p(bvh.prim, ctypes.c_uint64), int(device), flags)
        if not self._h:
            raise CeresError("ceres_scene_create: " + L.ceres_last_error().decode())
        self.device = device
        self.n_tri = len(mesh)

    @classmethod
    def from_device(cls, d_tri48, n_tri, d_norm36, d_nodes32, n_nodes, d_prim32, device=0, stats=False, stream=0):
        """ceres_scene_create_device: a scene from arrays already in HBM (int device pointers)."""
        L = lib()
        h = L.ceres_scene_create_device(d_tri48, n_tri, d_norm36, d_nodes32, n_nodes, d_prim32, int(device),
                                        SCENE_STATS if stats else 0, stream or None)
        if not h:
            raise CeresError("ceres_scene_create_device: " + L.ceres_last_error().decode())
        return cls(None, None, _handle=(h, device, n_tri))

    def info(self):
        d, s, n, b = ctypes.c_uint32(), ctypes.c_uint32(), _sz(), _sz()
        _check(lib().ceres_scene_info(self._h, ctypes.byref(d), ctypes.byref(s), ctypes.byref(n), ctypes.byref(b)))
        near, first = ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().ceres_scene_shadow_stacks(self._h, ctypes.byref(near), ctypes.byref(first)))
        return dict(depth=d.value, stack_entries=s.value, n_pairs=n.value, device_bytes=b.value,
                    shadow_stack_nearest=near.value, shadow_stack_first=first.value)

    def close(self):
        if getattr(self, "_h", None):
            lib().ceres_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, basis12, sun, W, H, mode=MODE_FULL, want_pixels=True, want_rgb8=True):
        """ceres_render_f32 / ceres_render_f64 (double scenes): host buffers out; returns
        (pixels [H*W*3] f32|f64 | None, rgb8 | None, stats dict)."""
        dt, ct = (np.float64, ctypes.c_double) if self.f64 else (np.float32, ctypes.c_float)
        b = np.ascontiguousarray(basis12, dt)
        s = np.ascontiguousarray(sun, dt)
        px = np.empty(3 * W * H, dt) if want_pixels else None
        rgb = np.empty(3 * W * H, np.uint8) if want_rgb8 else None
        st = _Stats()
        fn = lib().ceres_render_f64 if self.f64 else lib().ceres_render_f32
        _check(fn(self._h, _p(b, ct), _p(s, ct), int(mode), _p(px, ct), _p(rgb, ctypes.c_uint8), W, H, ctypes.byref(st)))
        return px, rgb, dict(rays=st.rays, hits=st.hits, primary_rays=st.primary_rays, shadow_rays=st.shadow_rays,
                             node_pairs=st.node_pairs, tri_tests=st.tri_tests, ms=st.ms)

    def records(self, basis12, sun, W, H, mode=MODE_FULL):
        """ceres_render_records(_f64): per-pixel (prim [W*H] i32, tuv [W*H,3] f32|f64, shadow [W*H] i8, stats)."""
        dt, ct = (np.float64, ctypes.c_double) if self.f64 else (np.float32, ctypes.c_float)
        b = np.ascontiguousarray(basis12, dt)
        s = np.ascontiguousarray(sun, dt)
        prim = np.empty(W * H, np.int32)
        tuv = np.empty(3 * W * H, dt)
        sh = np.empty(W * H, np.int8)
        st = _Stats()
        fn = lib().ceres_render_records_f64 if self.f64 else lib().ceres_render_records
        _check(fn(self._h, _p(b, ct), _p(s, ct), int(mode), W, H, _p(prim, ctypes.c_int32), _p(tuv, ct),
                  _p(sh, ctypes.c_int8), ctypes.byref(st)))
        return prim, tuv.reshape(-1, 3), sh, dict(rays=st.rays, hits=st.hits, node_pairs=st.node_pairs,
                                                  tri_tests=st.tri_tests)

    def render_device(self, basis12, sun, W, H, mode=MODE_FULL, tiling=None, d_pixels=0, d_rgb8=0, d_counters=0,
                      stream=0):
        """ceres_render_device: device pointers (ints, e.g. torch data_ptr()), async on `stream`."""
        b = np.ascontiguousarray(basis12, np.float32)
        s = np.ascontiguousarray(sun, np.float32)
        t = ctypes.byref(tiling) if tiling is not None else None
        _check(lib().ceres_render_device(self._h, _p(b, ctypes.c_float), _p(s, ctypes.c_float), int(mode), W, H, t,
                                         d_pixels or None, d_rgb8 or None, d_counters or None, stream or None))

    def render_batch_device(self, basis12, sun3, W, H, mode=MODE_FULL, tiling=None, d_pixels=0, d_rgb8=0,
                            d_counters=0, stream=0):
        """ceres_render_batch_device: F frames (basis12 [F,12], sun3 [F,3]) in one launch pair.
        Frame f's rows are at offset f*3*W*local_rows of d_pixels / d_rgb8."""
        b = np.ascontiguousarray(basis12, np.float32).reshape(-1, 12)
        s = np.ascontiguousarray(sun3, np.float32).reshape(-1, 3)
        if b.shape[0] != s.shape[0]:
            raise CeresError("render_batch_device: %d cameras but %d suns" % (b.shape[0], s.shape[0]))
        t = ctypes.byref(tiling) if tiling is not None else None
        _check(lib().ceres_render_batch_device(self._h, b.shape[0], _p(b, ctypes.c_float), _p(s, ctypes.c_float),
                                               int(mode), W, H, t, d_pixels or None, d_rgb8 or None,
                                               d_counters or None, stream or None))

    def set_timing(self, on):
        _check(lib().ceres_scene_set_timing(self._h, 1 if on else 0))

    def wave_log(self, max_waves=1 << 16):
        """Diagnostic per-wavefront records of the last full-mode render (stats scenes), one row per
        8x8 tile: start / after primary / end (100-MHz ticks), longest primary chain, shadow-loop
        trips, primary hits, primary and shadow node pairs of the wavefront."""
        out = np.zeros(8 * max_waves, np.uint64)
        n = _sz()
        _check(lib().ceres_scene_wave_log(self._h, _p(out, ctypes.c_uint64), max_waves, ctypes.byref(n)))
        return out[: 8 * n.value].reshape(-1, 8)

    def read_timing(self):
        """(kernel ms summed over the renders since set_timing, 0.0, renders)."""
        p, q, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        _check(lib().ceres_scene_read_timing(self._h, ctypes.byref(p), ctypes.byref(q), ctypes.byref(n)))
        return p.value, q.value, n.value


def source_sha16(repo=None):
    """sha256 (16 hex digits) of the sources libceres_hip.so is built from, in the Makefile's order
    (build_info.o: include/*.h and include/ceres/*.hpp sorted by path, then csrc/*.cpp *.hip *.hpp
    sorted by name); ceres_version() carries the value the loaded library was built with."""
    import glob
    import hashlib
    repo = repo or os.path.dirname(_PKG)
    inc = sorted(glob.glob(os.path.join(repo, "include", "*.h")) + glob.glob(os.path.join(repo, "include", "ceres", "*.hpp")))
    csrc = os.path.join(_PKG, "csrc")
    names = sorted(n for n in os.listdir(csrc) if n.endswith((".cpp", ".hip", ".hpp")))
    h = hashlib.sha256()
    for f in inc + [os.path.join(csrc, n) for n in names]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def native_provenance():
    """Which native library this process loaded and whether it was built from the sources in this
    tree: {lib, sha256 of the .so, sources_sha16 it was built with, sources_sha16 of the tree, match}."""
    import hashlib
    v = lib().ceres_version().decode()
    built = v.rsplit(" src ", 1)[1] if " src " in v else None
    with open(LIB_PATH, "rb") as fh:
        so_sha = hashlib.sha256(fh.read()).hexdigest()
    now = source_sha16()
    return {"lib": os.path.relpath(LIB_PATH, os.path.dirname(_PKG)), "version": v, "so_sha256": so_sha,
            "built_from_sources_sha16": built, "tree_sources_sha16": now, "built_from_this_tree": built == now}


FETCH_KINDS = ("bvh2_vector", "bvh4_vector", "bvh4_scalar", "tri_vector", "tri_scalar", "shade_vector",
               "store_vector", "order_scalar")
COUNT_LIB_PATH = os.path.join(_PKG, "variants", "libceres_hip_count.so")


def fetch_counters(device=0, reset=True):
    """Bytes moved by the kernels' own fetch sites since the last reset (the counting build only,
    `make count`; the product library raises CeresError EUNSUPPORTED): {kind: bytes}, vector kinds
    per lane, scalar kinds per wavefront (include/ceres_render.h ceres_fetch_counters)."""
    out = np.zeros(8, np.uint64)
    _check(lib().ceres_fetch_counters(int(device), _p(out, ctypes.c_uint64), 1 if reset else 0))
    return {k: int(v) for k, v in zip(FETCH_KINDS, out)}


def render_multi(scenes, basis12, sun, W, H, row_block=8, mode=MODE_FULL, want_pixels=True, want_rgb8=True):
    """ceres_render_multi_f32: one frame split over len(scenes) ranks (one Scene per rank, e.g. one
    per device) in this process; returns (pixels, rgb8, stats) like Scene.render."""
    b = np.ascontiguousarray(basis12, np.float32)
    s = np.ascontiguousarray(sun, np.float32)
    px = np.empty(3 * W * H, np.float32) if want_pixels else None
    rgb = np.empty(3 * W * H, np.uint8) if want_rgb8 else None
    hs = (_vp * len(scenes))(*[sc._h for sc in scenes])
    st = _Stats()
    _check(lib().ceres_render_multi_f32(hs, len(scenes), int(row_block), _p(b, ctypes.c_float), _p(s, ctypes.c_float),
                                        int(mode), _p(px, ctypes.c_float), _p(rgb, ctypes.c_uint8), W, H,
                                        ctypes.byref(st)))
    return px, rgb, dict(rays=st.rays, hits=st.hits, primary_rays=st.primary_rays, shadow_rays=st.shadow_rays,
                         node_pairs=st.node_pairs, tri_tests=st.tri_tests, ms=st.ms)


def orbit_cameras(camera, sun, W, H, n_frames, axis=(0, 1, 0), step_deg=None, rotate_first=True, want_dirs=False):
    """anim.cpp:76-88 orbit: eye, dir and sun rotated by step_deg (default 360/n_frames, as
    anim.cpp) about `axis` per frame.  Returns (basis12 [F,12] f32, sun3 [F,3] f32) and, with
    want_dirs, the rotated camera dirs [F,3] as a third element."""
    n = int(n_frames)
    step = np.float32(360.0) / np.float32(n) if step_deg is None else np.float32(step_deg)
    b = np.zeros((n, 12), np.float32)
    s3 = np.zeros((n, 3), np.float32)
    d3 = np.zeros((n, 3), np.float32)
    ax = np.asarray(axis, np.float32)
    sn = np.asarray(sun, np.float32)
    _check(lib().ceres_orbit_cameras_arith(_p(camera.eye, ctypes.c_float), _p(camera.dir, ctypes.c_float),
                                           _p(camera.up, ctypes.c_float), _p(sn, ctypes.c_float), camera.fov, W, H,
                                           _p(ax, ctypes.c_float), float(step), n, 1 if rotate_first else 0,
                                           _p(b, ctypes.c_float), _p(s3, ctypes.c_float), _p(d3, ctypes.c_float),
                                           camera.arith))
    return (b, s3, d3) if want_dirs else (b, s3)


def bench_views(camera, sun, W, H, F, basis0=None):
    """The F views of one bench.py step: frame f = the camera + sun rotated once by
    configs.orbit_step(f, F) degrees about configs.BENCH_AXIS (anim.cpp:76-88, Transform::rotate
    transform.hpp:67-112); frame 0 unrotated, with `basis0` (the fixture's pinned basis12) when
    given.  Returns (basis12 [F,12] f32, sun3 [F,3] f32, step_deg [F] f32); the reference PPM of
    every such view is pinned in tests/golden/orbit/<cfg>.json by its step bits."""
    F = int(F)
    b12 = np.zeros((F, 12), np.float32)
    s3 = np.zeros((F, 3), np.float32)
    steps = np.asarray([configs.orbit_step(f, F) for f in range(F)], np.float32)
    b12[0] = camera.basis(W, H) if basis0 is None else np.asarray(basis0, np.float32)
    s3[0] = np.asarray(sun, np.float32)
    for f in range(1, F):
        b, s = orbit_cameras(camera, sun, W, H, 2, axis=configs.BENCH_AXIS, step_deg=float(steps[f]),
                             rotate_first=False)
        b12[f], s3[f] = b[1], s[1]
    return b12, s3, steps


def pose(cfg, frame=0, arith=ARITH_EXACT):
    """(Camera, sun) of a config: configs with "orbit": (axis, step_deg, count) are the anim.cpp
    orbit pose after count + frame rotations; otherwise the config's camera rotated `frame`
    times by configs.BENCH_ORBIT."""
    cam = Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"], arith=arith)
    axis, step = (cfg["orbit"][0], cfg["orbit"][1]) if cfg.get("orbit") else configs.BENCH_ORBIT
    n = (cfg["orbit"][2] if cfg.get("orbit") else 0) + int(frame)
    if n == 0:
        return cam, np.asarray(cfg["sun"], np.float32)
    b, s3, d3 = orbit_cameras(cam, cfg["sun"], cfg["W"], cfg["H"], n + 1, axis=axis, step_deg=step,
                              rotate_first=False, want_dirs=True)
    return Camera(b[n, :3], d3[n], cfg["up"], cfg["fov"], arith=arith), s3[n].copy()


def pose_f64(cfg, arith=ARITH_EXACT):
    """(Camera<double>, sun) of a config: its values as double literals (anim.cpp writes its
    camera as double literals), orbited with Transform<double> when the config has "orbit"."""
    cam = Camera(cfg["eye"], cfg["dir"], cfg["up"], cfg["fov"], dtype=np.float64, arith=arith)
    sun = np.asarray(cfg["sun"], np.float64)
    if not cfg.get("orbit"):
        return cam, sun
    (axis, step, n) = cfg["orbit"]
    b = np.zeros((n + 1, 12), np.float64)
    s3 = np.zeros((n + 1, 3), np.float64)
    d3 = np.zeros((n + 1, 3), np.float64)
    ax = np.asarray(axis, np.float64)
    _check(lib().ceres_orbit_cameras_f64_arith(_p(cam.eye, ctypes.c_double), _p(cam.dir, ctypes.c_double),
                                               _p(cam.up, ctypes.c_double), _p(sun, ctypes.c_double), cam.fov, cfg["W"],
                                               cfg["H"], _p(ax, ctypes.c_double), float(step), n + 1, 0,
                                               _p(b, ctypes.c_double), _p(s3, ctypes.c_double), _p(d3, ctypes.c_double),
                                               int(arith)))
    return Camera(b[n, :3], d3[n], cfg["up"], cfg["fov"], dtype=np.float64, arith=arith), s3[n].copy()


def assemble_rgb8(d_gathered, rank_stride, d_out, frames, W, H, row_block, world, stream=0):
    """ceres_assemble_rgb8 (device pointers): rank-major gathered batch rows -> F PPM bodies."""
    _check(lib().ceres_assemble_rgb8(d_gathered, rank_stride, d_out, int(frames), W, H, int(row_block), int(world),
                                     stream or None))


def assemble_rgb8_packed(d_gathered, d_out, frames, W, H, row_block, world, stream=0):
    """ceres_assemble_rgb8_packed (device pointers): packed rank-major rows -> F PPM bodies."""
    _check(lib().ceres_assemble_rgb8_packed(d_gathered, d_out, int(frames), W, H, int(row_block), int(world),
                                            stream or None))


def local_rows(H, tiling):
    return lib().ceres_tiling_local_rows(H, ctypes.byref(tiling))


def row_map(H, row_block, world):
    """For each rank, the global rows j of its local rows k (ceres_tiling)."""
    out = []
    nb = (H + row_block - 1) // row_block
    for r in range(world):
        rows = []
        for b in range(r, nb, world):
            rows.extend(range(b * row_block, min(H, (b + 1) * row_block)))
        out.append(np.asarray(rows, np.int64))
    return out


def prepare(cfg, f64=False, arith=ARITH_EXACT):
    """Scene prep of the reference app for a config (configs.CONFIGS entry): mesh, bvh, camera
    (at the config's orbit pose; pose(cfg) also gives the sun).  f64: the render<double>
    pipeline (anim.cpp -d) -- double mesh / BVH, camera at the config's pose in double.
    arith = ARITH_FMA: every step in the reference CMake build's arithmetic (render with MODE_FMA)."""
    if f64:
        mesh = proc_mesh_f64(cfg["proc"], arith) if cfg.get("proc") else load_obj_f64(configs.obj_path(cfg), arith)
        if len(mesh) == 0:
            raise CeresError("The given scene is empty or cannot be loaded")
        if cfg.get("rotate"):
            rotate_triangles(mesh, cfg["rotate"][0], cfg["rotate"][1], arith)
        return mesh, build_bvh(mesh, arith), pose_f64(cfg, arith)[0]
    mesh = proc_mesh(cfg["proc"], arith) if cfg.get("proc") else load_obj(configs.obj_path(cfg), arith)
    if len(mesh) == 0:
        raise CeresError("The given scene is empty or cannot be loaded")
    if cfg.get("rotate"):
        rotate_triangles(mesh, cfg["rotate"][0], cfg["rotate"][1], arith)
    bvh = build_bvh(mesh, arith)
    cam, _ = pose(cfg, arith=arith)
    return mesh, bvh, cam


def render(camera, sun, scene, W, H, mode=MODE_FULL):
    """render<float>() (render.hpp:86-156): returns (pixels [3*W*H] f32, rays, hits)."""
    px, _, st = scene.render(camera.basis(W, H), sun, W, H, mode=mode, want_rgb8=False)
    return px, st["rays"], st["hits"]


def ppm(W, H, rgb8):
    """P6 file bytes exactly as static.cpp:135-147 writes them."""
    return b"P6 %d %d 255\n" % (W, H) + np.asarray(rgb8, np.uint8).tobytes()
