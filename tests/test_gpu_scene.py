"""Device-resident scene preparation (SURVEY.md §8(f) f1 + f2): OBJ text -> GPU parse -> GPU
rotation -> GPU binned-SAH BVH -> GPU relayout (ceres_scene_create_device) -> render, with no
host round trip.  The device relayout numbers its records differently from the host one, so
the bar is the rendered frame: PPM sha256 equal to the reference fixture, rays/hits equal, and
the float framebuffer bit-identical to the host-built scene's; scene shape (BVH depth, BVH4
stack bound) equal to the host relayout's.  Malformed BVHs fail loudly."""
import hashlib
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import REPO, load_golden

import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


def _hexf(hx):
    return np.asarray([int(h, 16) for h in hx], np.uint32).view(np.float32)


def basis_of(meta, cfg, build="exact"):
    pose, basis = (meta["ref_pose"], meta["ref_basis"]) if build == "ref" else (meta["pose"], meta["basis"])
    return np.concatenate([_hexf(pose["eye"]), _hexf(basis["dir"] + basis["u"] + basis["v"])])


def sun_of(meta, cfg, build="exact"):
    return _hexf((meta["ref_pose"] if build == "ref" else meta["pose"])["sun"])


def device_scene(pkg, d_tri, n, d_norm, arith=0):
    """GPU BVH + GPU relayout over device triangles/normals (int pointers)."""
    import torch
    d_nodes = torch.empty((2 * n - 1) * 8 if n > 1 else 8, dtype=torch.int32, device="cuda:0")
    d_prim = torch.empty(n, dtype=torch.int32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    m = pkg.build_bvh_device(d_tri, n, d_nodes.data_ptr(), d_prim.data_ptr(), stream, arith)
    scene = pkg.Scene.from_device(d_tri, n, d_norm, d_nodes.data_ptr(), m, d_prim.data_ptr(), stream=stream)
    return scene, m


@pytest.mark.parametrize("name", ["dragon_1080", "bunny_640", "bunny_1080_primary", "degenerate", "tri1", "quad",
                                  "proc_101", "dragon_orbit3_333x217", "dragon_4096", "dupleaf"])
def test_device_scene_renders_reference_frame(gpu, name):
    import torch
    pkg = gpu
    cfg = configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    mesh, bvh, _ = pkg.prepare(cfg)
    d_tri = torch.from_numpy(mesh.tri.reshape(-1).copy()).to("cuda:0")
    d_norm = torch.from_numpy(mesh.norm.reshape(-1).copy()).to("cuda:0")
    scene, m = device_scene(pkg, d_tri.data_ptr(), len(mesh), d_norm.data_ptr())
    host_scene = pkg.Scene(mesh, bvh)
    try:
        assert m == meta["n_nodes"]
        a, b = scene.info(), host_scene.info()
        assert (a["depth"], a["stack_entries"], a["n_pairs"]) == (b["depth"], b["stack_entries"], b["n_pairs"])
        mode = pkg.cfg_mode(cfg)
        basis, sun = basis_of(meta, cfg), sun_of(meta, cfg)
        px, rgb, st = scene.render(basis, sun, cfg["W"], cfg["H"], mode=mode)
        hpx, _, _ = host_scene.render(basis, sun, cfg["W"], cfg["H"], mode=mode)
        assert (st["rays"], st["hits"]) == (meta["exact"]["rays"], meta["exact"]["hits"])
        assert hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"]["exact"]
        assert np.array_equal(px.view(np.uint32), hpx.view(np.uint32))
    finally:
        scene.close()
        host_scene.close()


@pytest.mark.parametrize("build", ["ref", "exact"])
def test_obj_text_to_frame_on_device(gpu, build):
    """dragon.obj text in HBM -> parse -> rotate -> BVH -> scene -> C3 frame, all on the GPU; in the
    reference CMake build's arithmetic (build "ref": CERES_ARITH_FMA + CERES_MODE_FMA) and the
    contraction-free one."""
    import torch
    pkg = gpu
    name = "dragon_1080"
    cfg = configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    arith = 1 if build == "ref" else 0
    text = open(configs.obj_path(cfg), "rb").read()
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    d_tri, d_norm, n = pkg.parse_obj_device(d_text.data_ptr(), len(text), stream, arith)
    try:
        pkg.rotate_triangles_device(d_tri, n, cfg["rotate"][0], cfg["rotate"][1], stream, arith)
        scene, _ = device_scene(pkg, d_tri, n, d_norm, arith)
        _, rgb, st = scene.render(basis_of(meta, cfg, build), sun_of(meta, cfg, build), cfg["W"], cfg["H"],
                                  mode=pkg.cfg_mode(cfg, arith), want_pixels=False)
        scene.close()
    finally:
        pkg.device_free(d_tri)
        pkg.device_free(d_norm)
    assert n == meta["n_tri"]
    assert (st["rays"], st["hits"]) == (meta[build]["rays"], meta[build]["hits"])
    assert hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"][build]


@pytest.mark.parametrize("build", ["ref", "exact"])
def test_c5_obj_text_to_frame_on_device(gpu, build):
    """C5: the 10M-triangle heightfield as OBJ text -> device pipeline -> the reference's 4K frame."""
    import torch
    pkg = gpu
    name = "proc_c5"
    arith = 1 if build == "ref" else 0
    cfg = configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c5.obj")
        subprocess.run([os.path.join(REPO, "tools", "probes", "proc_obj"), str(cfg["proc"]), p], check=True)
        text = open(p, "rb").read()
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to("cuda:0")
    del text
    stream = torch.cuda.current_stream().cuda_stream
    d_tri, d_norm, n = pkg.parse_obj_device(d_text.data_ptr(), d_text.numel(), stream, arith)
    del d_text
    try:
        scene, m = device_scene(pkg, d_tri, n, d_norm, arith)
        _, rgb, st = scene.render(basis_of(meta, cfg, build), sun_of(meta, cfg, build), cfg["W"], cfg["H"],
                                  mode=pkg.cfg_mode(cfg, arith), want_pixels=False)
        scene.close()
    finally:
        pkg.device_free(d_tri)
        pkg.device_free(d_norm)
    assert (n, m) == (meta["n_tri"], meta["ref_n_nodes" if arith else "n_nodes"])
    assert (st["rays"], st["hits"]) == (meta[build]["rays"], meta[build]["hits"])
    assert hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"][build]


def test_device_scene_rejects_malformed_bvh(gpu):
    import torch
    pkg = gpu
    mesh, bvh, _ = pkg.prepare(configs.CONFIGS["proc_101"])
    d_tri = torch.from_numpy(mesh.tri.reshape(-1).copy()).to("cuda:0")
    d_norm = torch.from_numpy(mesh.norm.reshape(-1).copy()).to("cuda:0")
    d_prim = torch.from_numpy(bvh.prim.astype(np.uint32).view(np.int32)).to("cuda:0")
    inner = np.flatnonzero(bvh.nodes[:, 6] == 0)
    leaves = np.flatnonzero(bvh.nodes[:, 6] != 0)
    bad = []
    n1 = bvh.nodes.copy(); n1[inner[3], 7] = n1.shape[0] + 5; bad.append(n1)          # child index out of range
    n2 = bvh.nodes.copy(); n2[inner[5], 7] = n2[inner[4], 7]; bad.append(n2)          # two parents share children
    n3 = bvh.nodes.copy(); n3[leaves[0], 6] = len(mesh) + 1; bad.append(n3)           # leaf range out of bounds
    for nodes in bad:
        d_nodes = torch.from_numpy(nodes.view(np.int32).reshape(-1).copy()).to("cuda:0")
        with pytest.raises(pkg.CeresError):
            pkg.Scene.from_device(d_tri.data_ptr(), len(mesh), d_norm.data_ptr(), d_nodes.data_ptr(), nodes.shape[0],
                                  d_prim.data_ptr())
    p = bvh.prim.astype(np.uint32).copy(); p[7] = len(mesh) + 3
    with pytest.raises(pkg.CeresError):
        pkg.Scene.from_device(d_tri.data_ptr(), len(mesh), d_norm.data_ptr(),
                              torch.from_numpy(bvh.nodes.view(np.int32).reshape(-1).copy()).to("cuda:0").data_ptr(),
                              bvh.nodes.shape[0], torch.from_numpy(p.view(np.int32)).to("cuda:0").data_ptr())
