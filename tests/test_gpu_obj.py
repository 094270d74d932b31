"""GPU OBJ loading: csrc/obj_parse.hip must return the reference loader's
bits -- obj::load_from_stream (obj_norms.hpp:57-118): fan-triangulated Triangle records and
per-corner vertex normals summed in face order -- and rotate_triangles (render.hpp:24-44) on
device triangles must equal the host rotation.  Checked against the reference fixtures
(tri48/norm36 sha256 of every golden mesh), the oracle's std::istream loader and the host
loader on adversarial text (CRLF, tabs, comments, vt/vn/o/g lines, i/t/n forms with spaces,
relative indices, NUL bytes, junk numbers, hex floats, long mantissas, over-long lines), and
on the C5 heightfield written as OBJ text (tools/probes/proc_obj)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import ref_scene_hashes, REPO, golden_names, load_golden

import configs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device (no CPU fallback exists)")
    return pkg


def same(a, b):
    return a.tri.shape == b.tri.shape and np.array_equal(a.tri.view(np.uint32), b.tri.view(np.uint32)) and \
        np.array_equal(a.norm.view(np.uint32), b.norm.view(np.uint32))


OBJ_CONFIGS = sorted({configs.CONFIGS[n]["obj"]: n for n in golden_names() if configs.CONFIGS[n]["obj"]}.values())


@pytest.mark.parametrize("arith", [0, 1], ids=["exact", "fma"])
@pytest.mark.parametrize("name", OBJ_CONFIGS)
def test_gpu_obj_matches_reference_fixture(gpu, name, arith):
    """GPU parse + GPU rotation == the reference's loaded and rotated scene (fixture hashes), in
    both builds' arithmetic (the CMake-flag build contracts the triangle normals, the vertex-normal
    normalisation and the rotation)."""
    import torch
    pkg = gpu
    cfg = configs.CONFIGS[name]
    meta, _, _ = load_golden(name)
    path = configs.obj_path(cfg)
    host = pkg.load_obj(path, arith)
    dev = pkg.load_obj_gpu(path, arith=arith)
    assert same(dev, host)
    # rotate on the device (torch-owned HBM), compare with the reference's rotated triangles
    d_tri = torch.from_numpy(dev.tri.reshape(-1).copy()).to("cuda:0")
    if cfg.get("rotate"):
        pkg.rotate_triangles_device(d_tri.data_ptr(), len(dev), cfg["rotate"][0], cfg["rotate"][1],
                                    torch.cuda.current_stream().cuda_stream, arith)
    torch.cuda.synchronize()
    tri = d_tri.cpu().numpy()
    norm = dev.norm
    n = len(dev)
    assert n == meta["n_tri"]
    tri_h, norm_h, _ = ref_scene_hashes(meta, arith)
    assert hashlib.sha256(tri.tobytes()).hexdigest() == tri_h
    assert hashlib.sha256(norm.tobytes()).hexdigest() == norm_h


def _num(rng):
    k = rng.integers(0, 12)
    x = float(rng.normal() * 10.0 ** int(rng.integers(-6, 5)))
    if k < 6:
        return "%.*g" % (int(rng.integers(1, 12)), x)
    if k == 6:
        return "%.*e" % (int(rng.integers(0, 10)), x)
    if k == 7:
        return float(np.float32(x)).hex()                         # hex float
    if k == 8:
        return "%.40f" % x                                         # long mantissa
    if k == 9:
        return "".join(str(d) for d in rng.integers(0, 10, int(rng.integers(1, 30)))) + "e-" + str(rng.integers(0, 30))
    if k == 10:
        return ["abc", "-", ".", "+.5", "1e", "0x", "-0", "00012", "1.5e+3x"][int(rng.integers(0, 9))]
    return "%d" % int(x)


def _face_ref(rng, nv):
    i = int(rng.integers(1, nv + 1))
    ref = str(i) if rng.random() < 0.6 else str(i - nv - 1)       # absolute or relative (-1 = last)
    form = rng.integers(0, 5)
    if form == 1:
        ref += "/%d" % rng.integers(1, 9)
    elif form == 2:
        ref += "//%d" % rng.integers(1, 9)
    elif form == 3:
        ref += "/%d/%d" % (rng.integers(1, 9), rng.integers(1, 9))
    elif form == 4:
        ref += " / %d / %d" % (rng.integers(1, 9), rng.integers(1, 9))
    return ref


def make_obj(rng, n_lines):
    out, nv = [], 0
    ws = [" ", "\t", "  ", " \t "]
    for _ in range(n_lines):
        r = rng.random()
        pre = ws[int(rng.integers(0, 4))] if rng.random() < 0.2 else ""
        post = ws[int(rng.integers(0, 4))] if rng.random() < 0.2 else ""
        eol = "\r\n" if rng.random() < 0.2 else "\n"
        if r < 0.45 or nv < 3:
            nums = [_num(rng) for _ in range(int(rng.integers(2, 5)))]
            line = "v" + ws[int(rng.integers(0, 4))] + " ".join(nums)
            nv += 1
        elif r < 0.8:
            k = int(rng.integers(3, 7))
            line = "f " + (ws[int(rng.integers(0, 4))]).join(_face_ref(rng, nv) for _ in range(k))
        elif r < 0.85:
            line = "# comment " + _num(rng)
        elif r < 0.9:
            line = ["vn 0 1 0", "vt 0.5 0.5", "o thing", "g grp", "s off", "usemtl m", "v", "f", "vv 1 2 3", ""][
                int(rng.integers(0, 10))]
        elif r < 0.93:
            line = "v 1 2\x003 4"                                   # NUL ends the C string
        else:
            line = ""
        out.append(pre + line + post + eol)
    return "".join(out).encode()


@pytest.mark.parametrize("seed", range(6))
def test_gpu_obj_matches_oracle_on_adversarial_text(gpu, oracle_mod, tmp_path, seed):
    pkg = gpu
    rng = np.random.default_rng(seed)
    p = tmp_path / "adv.obj"
    data = make_obj(rng, int(rng.integers(50, 5000)))
    if seed == 5:
        data = data[: len(data) // 2] + b"# " + b"y" * 1500 + b"\n" + data[len(data) // 2:]   # reading stops here
    if seed == 4:
        data = data.rstrip(b"\n")                                    # no final newline
    p.write_bytes(data)
    dev = pkg.load_obj_gpu(str(p))
    host = pkg.load_obj(str(p))
    t, n = oracle_mod.load_mesh(str(p))
    ora = pkg.Mesh(t, n)
    assert len(dev) > 0
    assert same(dev, ora), "GPU parse differs from the std::istream restatement"
    assert same(dev, host)


def test_gpu_obj_errors_and_empty(gpu, tmp_path):
    pkg = gpu
    assert len(pkg.load_obj_gpu(str(tmp_path / "missing.obj"))) == 0
    p = tmp_path / "e.obj"
    p.write_bytes(b"")
    assert len(pkg.load_obj_gpu(str(p))) == 0
    p.write_bytes(b"# only comments\n\n   \n")
    assert len(pkg.load_obj_gpu(str(p))) == 0
    for bad in (b"v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n", b"v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
                b"v 0 0 0\nv 1 0 0\nf 1 2 -3\n", b"v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 -x\n"):
        p.write_bytes(bad)
        with pytest.raises(pkg.CeresError):
            pkg.load_obj_gpu(str(p))
    # a face may only reference vertices read before it (relative and absolute)
    p.write_bytes(b"v 0 0 0\nv 1 0 0\nf 1 2 3\nv 0 1 0\n")
    with pytest.raises(pkg.CeresError):
        pkg.load_obj_gpu(str(p))


@pytest.mark.parametrize("n", [101, 601])
def test_gpu_obj_proc_heightfield_roundtrip(gpu, tmp_path, n):
    """The C5 heightfield as OBJ text parses to exactly ceres_proc_mesh's triangles and normals."""
    pkg = gpu
    p = tmp_path / "proc.obj"
    subprocess.run([os.path.join(REPO, "tools", "probes", "proc_obj"), str(n), str(p)], check=True)
    assert same(pkg.load_obj_gpu(str(p)), pkg.proc_mesh(n))
