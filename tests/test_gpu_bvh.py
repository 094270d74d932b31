"""GPU BVH build: the gfx950 binned-SAH builder (csrc/bvh_build.hip) must
produce the reference's BVH -- BinnedSahBuilder<Bvh,16> (binned_sah_builder.hpp:39-234) --
bit for bit: the same topology, node boxes (sign of zero included) and primitive_indices,
compared through the numbering-independent canonical sha256 of tests/golden/make_golden.py
against (a) the fixtures the reference itself produced and (b) the host builder on
adversarial meshes (duplicates, signed zeros, flat axes, sizes around the small-subtree
threshold of 512 primitives).  A frame rendered over the GPU-built BVH must equal the
reference PPM."""
import hashlib
import time

import numpy as np
import pytest

from conftest import golden_names, load_golden, ref_scene_hashes

import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


def canon(bvh):
    import oracle
    return oracle.canonical_bvh_sha(bvh.nodes, bvh.prim)


def _mesh(pkg, cfg, arith=0):
    mesh = pkg.proc_mesh(cfg["proc"], arith) if cfg.get("proc") else pkg.load_obj(configs.obj_path(cfg), arith)
    if cfg.get("rotate"):
        pkg.rotate_triangles(mesh, cfg["rotate"][0], cfg["rotate"][1], arith)
    return mesh


# one config per distinct mesh (+ rotation)
_MESHES = {}
for _n in golden_names():
    _c = configs.CONFIGS[_n]
    _MESHES.setdefault((_c["obj"], _c["proc"], _c["rotate"]), _n)
MESH_CONFIGS = sorted(_MESHES.values())


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
@pytest.mark.parametrize("name", MESH_CONFIGS)
def test_gpu_bvh_matches_reference_fixture(gpu, name, arith):
    """Both reference builds: the contraction-free one and the CMake-flag one, whose SAH costs
    (binned_sah_builder.hpp:98,109,179) contract into FMA -- the FMA flavour of the GPU builder."""
    pkg = gpu
    meta, _, _ = load_golden(name)
    mesh = _mesh(pkg, configs.CONFIGS[name], arith)
    bvh = pkg.build_bvh_gpu(mesh, arith=arith)
    assert bvh.nodes.shape[0] == meta["ref_n_nodes" if arith else "n_nodes"]
    assert canon(bvh) == ref_scene_hashes(meta, arith)[2]
    assert sorted(bvh.prim.tolist()) == list(range(len(mesh)))


def _soup(rng, n, kind):
    """Adversarial triangle soups as bvh::Triangle<float> rows {p0, e1 = p0 - p1, e2 = p2 - p0, n}."""
    if kind == "uniform":
        p = rng.random((n, 3, 3), dtype=np.float32) * 10 - 5
    elif kind == "grid":                          # many equal coordinates, exact zeros of both signs
        p = rng.integers(-3, 4, size=(n, 3, 3)).astype(np.float32)
        p[rng.random((n, 3, 3)) < 0.3] = -0.0
    elif kind == "flat":                          # every triangle in z = 0 (flat axis: 1/0 bin scale)
        p = rng.random((n, 3, 3), dtype=np.float32)
        p[..., 2] = np.where(rng.random((n, 3)) < 0.5, np.float32(0.0), np.float32(-0.0))
    elif kind == "dups":                          # few distinct triangles, repeated (one-sided partitions)
        base = rng.random((7, 3, 3), dtype=np.float32)
        p = base[rng.integers(0, 7, size=n)]
    elif kind == "clustered":                     # tight clusters far apart (deep, unbalanced splits)
        c = rng.random((5, 3), dtype=np.float32) * 1e4
        p = c[rng.integers(0, 5, size=n)][:, None, :] + rng.random((n, 3, 3), dtype=np.float32) * 1e-3
    else:
        raise ValueError(kind)
    p0, p1, p2 = p[:, 0], p[:, 1], p[:, 2]
    e1 = p0 - p1
    e2 = p2 - p0
    nrm = np.cross(e1, e2).astype(np.float32)
    return np.concatenate([p0, e1, e2, nrm], axis=1).astype(np.float32)


@pytest.mark.parametrize("kind,n", [("uniform", 1), ("uniform", 2), ("uniform", 17), ("uniform", 512),
                                    ("uniform", 513), ("uniform", 1500), ("uniform", 70000), ("grid", 600),
                                    ("grid", 20000), ("flat", 3000), ("dups", 5000), ("dups", 300),
                                    ("clustered", 40000)])
def test_gpu_bvh_matches_host_builder(gpu, kind, n):
    pkg = gpu
    rng = np.random.default_rng(1234 + n)
    tri = _soup(rng, n, kind)
    mesh = pkg.Mesh(tri, np.zeros((n, 9), np.float32))
    for arith in (0, 1):
        host = pkg.build_bvh(mesh, arith=arith)
        dev = pkg.build_bvh_gpu(mesh, arith=arith)
        assert dev.nodes.shape == host.nodes.shape, arith
        assert np.array_equal(dev.prim, host.prim), arith    # primitive_indices: same permutation, same order
        assert canon(dev) == canon(host), arith


def test_render_over_gpu_bvh_matches_reference(gpu):
    pkg = gpu
    name = "dragon_1080"
    meta, _, _ = load_golden(name)
    cfg = configs.CONFIGS[name]
    mesh = _mesh(pkg, cfg)
    bvh = pkg.build_bvh_gpu(mesh)
    scene = pkg.Scene(mesh, bvh)
    bits = [int(h, 16) for h in meta["basis"]["dir"] + meta["basis"]["u"] + meta["basis"]["v"]]
    basis = np.concatenate([np.asarray(cfg["eye"], np.float32), np.asarray(bits, np.uint32).view(np.float32)])
    _, rgb, st = scene.render(basis, cfg["sun"], cfg["W"], cfg["H"], want_pixels=False)
    assert (st["rays"], st["hits"]) == (meta["exact"]["rays"], meta["exact"]["hits"])
    assert hashlib.sha256(pkg.ppm(cfg["W"], cfg["H"], rgb)).hexdigest() == meta["ppm_sha256"]["exact"]
    scene.close()


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
def test_gpu_bvh_c5_matches_reference_and_is_faster(gpu, arith):
    """C5 (9,999,392 triangles): canonical topology equal to the reference's; timing reported."""
    import torch
    pkg = gpu
    meta, _, _ = load_golden("proc_c5")
    mesh = _mesh(pkg, configs.CONFIGS["proc_c5"], arith)
    n = len(mesh)
    d_tri = torch.from_numpy(mesh.tri.reshape(-1)).to("cuda:0")
    d_nodes = torch.empty((2 * n - 1) * 8, dtype=torch.int32, device="cuda:0")
    d_prim = torch.empty(n, dtype=torch.int32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    pkg.build_bvh_device(d_tri.data_ptr(), n, d_nodes.data_ptr(), d_prim.data_ptr(), stream, arith)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = pkg.build_bvh_device(d_tri.data_ptr(), n, d_nodes.data_ptr(), d_prim.data_ptr(), stream, arith)
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) * 1e3
    nodes = d_nodes[: m * 8].cpu().numpy().view(np.uint32).reshape(-1, 8)
    prim = d_prim.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert m == meta["ref_n_nodes" if arith else "n_nodes"]
    import oracle
    assert oracle.canonical_bvh_sha(nodes, prim) == ref_scene_hashes(meta, arith)[2]
    t0 = time.perf_counter()
    pkg.build_bvh(mesh, arith=arith)
    host_ms = (time.perf_counter() - t0) * 1e3
    print(f"C5 BVH build: gpu {gpu_ms:.1f} ms, host {host_ms:.1f} ms ({n} triangles, {m} nodes)")
    assert gpu_ms < host_ms
