"""ctypes front-end of the CPU restatement (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / reported CPU baseline -- never as the product path.
See oracle/oracle.cpp for what is restated from which reference file:line, and
tests/test_oracle_golden.py for how it is pinned to the reference's own outputs.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_render")
REF_BIN_EXACT = os.path.join(HERE, "_ref", "ref_render_exact")

_lib = None
_fp = ctypes.POINTER(ctypes.c_float)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t


def build():
    subprocess.run(["make", "-C", HERE, "oracle"], check=True, capture_output=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_load_obj.argtypes = [ctypes.c_char_p, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz),
                                      ctypes.c_int]
        L.oracle_load_obj_text.argtypes = [ctypes.c_char_p, _sz, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz),
                                           ctypes.c_int]
        L.oracle_proc_mesh.argtypes = [ctypes.c_int, ctypes.POINTER(_fp), ctypes.POINTER(_fp), ctypes.POINTER(_sz), ctypes.c_int]
        L.oracle_rotate.argtypes = [_fp, _sz, ctypes.c_int, ctypes.c_float, ctypes.c_int]
        L.oracle_rotate.restype = None
        L.oracle_build_bvh.argtypes = [_fp, _sz, ctypes.POINTER(_u32p), ctypes.POINTER(_sz), ctypes.POINTER(_u64p), ctypes.c_int]
        L.oracle_camera_basis.argtypes = [_fp, _fp, _fp, ctypes.c_float, _sz, _sz, _fp, ctypes.c_int]
        L.oracle_camera_basis.restype = None
        L.oracle_orbit.argtypes = [_fp, ctypes.c_float, ctypes.c_int, _fp, _fp, _fp, ctypes.c_int]
        L.oracle_orbit.restype = None
        L.oracle_render.argtypes = [_fp, _fp, _sz, _u32p, _sz, _u64p, _fp, _fp, _fp, ctypes.c_int, _sz, _sz,
                                    _fp, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int32), _fp,
                                    ctypes.POINTER(ctypes.c_int8), _u64p, ctypes.c_int, _u32p]
        L.oracle_bvh_canonical.argtypes = [_u32p, _sz, _u64p, _sz, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                           ctypes.POINTER(_sz)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_free.restype = None
        _lib = L
    return _lib


def canonical_bvh_sha(nodes, prim):
    """sha256 of the numbering-independent DFS serialisation of a BVH (nodes: m x 8 u32, prim: u64);
    equal to tests/golden/make_golden.canonical_bvh_sha, computed in C."""
    import hashlib
    nodes = np.ascontiguousarray(nodes, np.uint32).reshape(-1, 8)
    prim = np.ascontiguousarray(prim, np.uint64)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = _sz()
    _check(lib().oracle_bvh_canonical(_ptr(nodes, ctypes.c_uint32), nodes.shape[0], _ptr(prim, ctypes.c_uint64),
                                      prim.size, ctypes.byref(out), ctypes.byref(n)))
    try:
        return hashlib.sha256(ctypes.string_at(out, n.value)).hexdigest()
    finally:
        lib().oracle_free(out)


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t)) if a is not None else None


def _check(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + lib().oracle_last_error().decode())


def _take(p, count, dtype):
    if count == 0:
        return np.zeros(0, dtype=dtype)
    a = np.ctypeslib.as_array(p, shape=(count,)).copy().view(dtype)
    lib().oracle_free(ctypes.cast(p, ctypes.c_void_p))
    return a


def load_mesh(path=None, proc=0, contract=False):
    """obj_norms.hpp:120 load_from_file (or the C5 procedural mesh): (tri48 [n,12] f32, norm36 [n,9] f32).
    contract=True: the arithmetic of the reference's own CMake build (GCC FMA contraction)."""
    L = lib()
    t, nrm, n = _fp(), _fp(), _sz()
    if proc:
        _check(L.oracle_proc_mesh(int(proc), ctypes.byref(t), ctypes.byref(nrm), ctypes.byref(n), int(contract)))
    else:
        _check(L.oracle_load_obj(path.encode(), ctypes.byref(t), ctypes.byref(nrm), ctypes.byref(n), int(contract)))
    n = n.value
    tri = _take(t, n * 12, np.float32).reshape(n, 12)
    nor = _take(nrm, n * 9, np.float32).reshape(n, 9)
    return tri, nor


def rotate(tri, axis, degrees, contract=False):
    ax = {"x": 0, "y": 1, "z": 2}[axis] if isinstance(axis, str) else int(axis)
    lib().oracle_rotate(_ptr(tri, ctypes.c_float), tri.shape[0], ax, float(degrees), int(contract))
    return tri


def build_bvh(tri, contract=False):
    """Binned SAH (binned_sah_builder.hpp:39-234): nodes [m,8] u32 (bvh.hpp Node), prim u64."""
    L = lib()
    nodes, prim, m = _u32p(), _u64p(), _sz()
    _check(L.oracle_build_bvh(_ptr(tri, ctypes.c_float), tri.shape[0], ctypes.byref(nodes), ctypes.byref(m),
                              ctypes.byref(prim), int(contract)))
    m = m.value
    return _take(nodes, m * 8, np.uint32).reshape(m, 8), _take(prim, tri.shape[0], np.uint64)


def camera_basis(eye, dir, up, fov, W, H, contract=False):
    out = np.zeros(9, np.float32)
    f3 = lambda v: np.asarray(v, np.float32)  # noqa: E731
    e, d, u = f3(eye), f3(dir), f3(up)
    lib().oracle_camera_basis(_ptr(e, ctypes.c_float), _ptr(d, ctypes.c_float), _ptr(u, ctypes.c_float),
                              float(fov), W, H, _ptr(out, ctypes.c_float), int(contract))
    return out


def orbit(axis, step_deg, count, eye, dir, sun, contract=False):
    """anim.cpp:76-88: eye, dir, sun after `count` Transform rotations (oracle restatement)."""
    f3 = lambda v: np.array(v, np.float32)  # noqa: E731
    a, e, d, s = f3(axis), f3(eye), f3(dir), f3(sun)
    lib().oracle_orbit(_ptr(a, ctypes.c_float), float(np.float32(step_deg)), int(count), _ptr(e, ctypes.c_float),
                       _ptr(d, ctypes.c_float), _ptr(s, ctypes.c_float), int(contract))
    return e, d, s


def pose(cfg, frame=0, contract=False):
    """(eye, dir, sun) of a config; configs with "orbit": (axis, step_deg, count) are rotated
    count + frame times like anim.cpp's camera/sun."""
    eye, dir, sun = cfg["eye"], cfg["dir"], cfg["sun"]
    n = (cfg["orbit"][2] if cfg.get("orbit") else 0) + frame
    if n:
        axis, step = (cfg["orbit"][0], cfg["orbit"][1]) if cfg.get("orbit") else (cfg["orbit_axis"], cfg["orbit_step"])
        return orbit(axis, step, n, eye, dir, sun, contract)
    f3 = lambda v: np.array(v, np.float32)  # noqa: E731
    return f3(eye), f3(dir), f3(sun)


def prepare(cfg, contract=False):
    """Scene prep of the reference app (obj load, rotate, BVH build, camera basis) for a config dict;
    contract=True: with the reference-flag (GCC FMA contraction) arithmetic."""
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "ceres-raytracer_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    import configs as _c
    tri, nor = load_mesh(_c.obj_path(cfg), cfg.get("proc", 0), contract)
    if cfg.get("rotate"):
        rotate(tri, cfg["rotate"][0], cfg["rotate"][1], contract)
    nodes, prim = build_bvh(tri, contract)
    eye, dir, sun = pose(cfg, 0, contract)
    basis = camera_basis(eye, dir, cfg["up"], cfg["fov"], cfg["W"], cfg["H"], contract)
    return dict(tri=tri, norm=nor, nodes=nodes, prim=prim, basis=basis, eye=eye, sun=sun, contract=bool(contract))


def render(scene, cfg, basis=None, want_pixels=True, want_ppm=True, want_records=False, threads=0, want_pairs=False,
           eye=None, sun=None):
    """oracle_render of one frame; basis (9 floats), eye and sun default to the config's pose."""
    L = lib()
    W, H = cfg["W"], cfg["H"]
    basis = scene["basis"] if basis is None else np.asarray(basis, np.float32)
    eye = np.asarray(scene.get("eye", cfg["eye"]) if eye is None else eye, np.float32)
    sun = np.asarray(scene.get("sun", cfg["sun"]) if sun is None else sun, np.float32)
    px = np.zeros(3 * W * H, np.float32) if want_pixels else None
    ppm = np.zeros(3 * W * H, np.uint8) if want_ppm else None
    rp = np.zeros(W * H, np.int32) if want_records else None
    tuv = np.zeros(3 * W * H, np.float32) if want_records else None
    rs = np.zeros(W * H, np.int8) if want_records else None
    counts = np.zeros(6, np.uint64)
    pairs = np.zeros(2 * W * H, np.uint32) if want_pairs else None
    tri, nor, nodes, prim = scene["tri"], scene["norm"], scene["nodes"], scene["prim"]
    _check(L.oracle_render(_ptr(tri, ctypes.c_float), _ptr(nor, ctypes.c_float), tri.shape[0],
                           _ptr(nodes, ctypes.c_uint32), nodes.shape[0], _ptr(prim, ctypes.c_uint64),
                           _ptr(eye, ctypes.c_float), _ptr(basis, ctypes.c_float), _ptr(sun, ctypes.c_float),
                           (1 if cfg["mode"] == "primary" else 0) | (0x10 if cfg.get("robust") else 0)
                           | (0x20 if scene.get("contract") else 0), W, H,
                           _ptr(px, ctypes.c_float),
                           _ptr(ppm, ctypes.c_uint8), _ptr(rp, ctypes.c_int32), _ptr(tuv, ctypes.c_float),
                           _ptr(rs, ctypes.c_int8), _ptr(counts, ctypes.c_uint64), int(threads),
                           _ptr(pairs, ctypes.c_uint32)))
    out = dict(rays=int(counts[0]), hits=int(counts[1]), primary_pairs=int(counts[2]), primary_tests=int(counts[3]),
               shadow_pairs=int(counts[4]), shadow_tests=int(counts[5]), pixels=px, ppm=ppm)
    if want_records:
        out.update(prim=rp, tuv=tuv.reshape(-1, 3), shadow=rs)
    if want_pairs:
        out["pairs_per_pixel"] = pairs.reshape(-1, 2)      # (primary, shadow) node-pair visits
    return out


def ppm_bytes(W, H, body):
    return b"P6 %d %d 255\n" % (W, H) + body.tobytes()


def hexbits(a):
    return ["0x%08x" % int(x) for x in np.asarray(a, np.float32).view(np.uint32)]
