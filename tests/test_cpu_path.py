"""The product's CPU path (ceres_render_cpu_f32 / _f64, `./render --cpu [--double]`; SURVEY.md §7
step 3: "config 1 works with no GPU") against the reference's own outputs.  No GPU needed: these
run in the CPU suite.

Every golden config (C1-C5 and the edge cases; render<double>: every f64 fixture), both
arithmetics: the PPM bytes equal the reference build's, rays / hits equal render()'s return pair,
and the traversal counters equal the reference's Statistics (single_ray_traverser.hpp:132-135,
primary + shadow) that make_golden.py recorded.  The float framebuffer equals the oracle's bit for
bit.  The path is chosen only explicitly: the GPU
entry points still fail without a device (test_abi.py)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import load_golden

CLI_ARITH = {"ref": [], "exact": ["--exact"]}
SMALL = ["tri1", "quad", "quad_65x49_robust", "degenerate", "degenerate_65x49_robust", "dupleaf", "bunny_1x1",
         "bunny_640", "bunny_97x61_primary", "bunny_97x61_primary_robust", "bunny_orbit7_160x120", "bunny_rotz_160x120",
         "dragon_333x217", "dragon_333x217_robust", "dragon_orbit3_333x217", "dragon_640", "proc_101",
         "bunny_1080", "bunny_1080_primary", "dragon_1080", "dragon_1080_robust", "dragon_4096"]


def run_cli(pkg, name, build, tmp_path, extra=()):
    cfg = pkg.configs.CONFIGS[name]
    out = tmp_path / f"{name}_{build}.ppm"
    r = subprocess.run([pkg.CLI_PATH] + pkg.configs.cli_args(cfg) + CLI_ARITH[build] + ["--cpu", "--json", "-o", str(out)]
                       + list(extra), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    st = {}
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            st.update(json.loads(line))
    return out.read_bytes(), st, r.stdout


def check(meta, build, data, st):
    m = meta[build]
    assert hashlib.sha256(data).hexdigest() == meta["ppm_sha256"][build]
    assert (st["rays"], st["hits"]) == (m["rays"], m["hits"])
    assert st["node_pairs"] == m["primary_pairs"] + m["shadow_pairs"]
    assert st["tri_tests"] == m["primary_tests"] + m["shadow_tests"]
    assert st["shadow_rays"] == m["shadow_rays"]


@pytest.mark.parametrize("build", ["ref", "exact"])
@pytest.mark.parametrize("name", SMALL)
def test_cli_cpu_writes_reference_ppm(pkg, tmp_path, name, build):
    meta, _, ppm = load_golden(name)
    data, st, stdout = run_cli(pkg, name, build, tmp_path)
    check(meta, build, data, st)
    if build in ppm:
        assert data == ppm[build]
    assert "on the CPU" in stdout


def test_cli_cpu_c5(pkg, tmp_path):
    """C5 (the 10M-triangle procedural heightfield, 3840x2160) in the reference CMake build's arithmetic."""
    meta, _, _ = load_golden("proc_c5")
    data, st, _ = run_cli(pkg, "proc_c5", "ref", tmp_path)
    check(meta, "ref", data, st)


def test_cpu_threads_do_not_change_the_image(pkg, tmp_path):
    one, st1, _ = run_cli(pkg, "dragon_640", "ref", tmp_path, ["--threads", "1"])
    many, st8, _ = run_cli(pkg, "dragon_640", "ref", tmp_path, ["--threads", "8"])
    assert one == many and (st1["rays"], st1["hits"], st1["node_pairs"]) == (st8["rays"], st8["hits"], st8["node_pairs"])


@pytest.mark.parametrize("build", ["ref", "exact"])
@pytest.mark.parametrize("name", ["bunny_640", "dragon_333x217_robust", "bunny_97x61_primary"])
def test_cpu_float_framebuffer_equals_oracle(pkg, oracle_mod, name, build):
    """ceres_render_cpu_f32's float pixels (render.hpp:107 layout) against the oracle's, bit for bit."""
    cfg = pkg.configs.CONFIGS[name]
    arith = pkg.ARITH_FMA if build == "ref" else pkg.ARITH_EXACT
    mesh, bvh, cam = pkg.prepare(cfg, arith=arith)
    _, sun = pkg.pose(cfg, arith=arith)
    W, H = cfg["W"], cfg["H"]
    sc = pkg.CpuScene(mesh, bvh)
    try:
        px, rgb, st = sc.render(cam.basis(W, H), sun, W, H, mode=pkg.cfg_mode(cfg, arith))
    finally:
        sc.close()
    scene = oracle_mod.prepare(cfg, contract=build == "ref")
    ref = oracle_mod.render(scene, cfg)
    assert np.array_equal(px.view(np.uint32), ref["pixels"].view(np.uint32))
    assert np.array_equal(rgb, ref["ppm"])
    assert (st["rays"], st["hits"]) == (ref["rays"], ref["hits"])
    assert st["node_pairs"] == ref["primary_pairs"] + ref["shadow_pairs"]


def test_cpu_path_errors(pkg, tmp_path):
    cfg = pkg.configs.CONFIGS["tri1"]
    mesh, bvh, cam = pkg.prepare(cfg)
    _, sun = pkg.pose(cfg)
    sc = pkg.CpuScene(mesh, bvh)
    try:
        b = cam.basis(8, 8)
        with pytest.raises(pkg.CeresError):                          # a GPU-only mode
            sc.render(b, sun, 8, 8, mode=pkg.MODE_FULL | pkg.MODE_QBVH4)
        with pytest.raises(pkg.CeresError):
            sc.render(b, sun, 8, 8, mode=7)
        with pytest.raises(pkg.CeresError):
            sc.render(b, sun, 0, 8)
    finally:
        sc.close()
    obj = os.path.join(os.path.dirname(__file__), "golden", "tri1.obj")
    for flags in (["--gpus", "2"], ["--qbvh"], ["--gpu-bvh"]):
        r = subprocess.run([pkg.CLI_PATH, obj, "--size", "8", "8", "--cpu", "-o", os.devnull] + flags,
                           capture_output=True, text=True)
        assert r.returncode == 2 and "--cpu" in r.stderr, flags


F64 = os.path.join(os.path.dirname(__file__), "golden", "f64")
F64_NAMES = sorted(n[:-5] for n in os.listdir(F64) if n.endswith(".json"))


@pytest.mark.parametrize("build", ["ref", "exact"])
@pytest.mark.parametrize("name", F64_NAMES)
def test_cli_cpu_double_writes_reference_ppm(pkg, tmp_path, name, build):
    """./render --cpu --double (anim.cpp -d on the host): every render<double> fixture of the
    reference (tests/golden/f64, made by oracle/_ref/ref_render_f64{,_exact}) -- PPM bytes, rays,
    hits and the reference's traversal statistics, both arithmetics."""
    meta = json.load(open(os.path.join(F64, name + ".json")))
    data, st, stdout = run_cli(pkg, name, build, tmp_path, ["--double"])
    check(meta, build, data, st)
    assert "on the CPU" in stdout


def test_cpu_double_scene_api(pkg):
    """CpuScene over a double mesh: ceres_render_cpu_f64's double framebuffer quantises to the
    fixture's PPM; a float render call on it (and ROBUST) is refused."""
    import ctypes
    name = "bunny_640"
    meta = json.load(open(os.path.join(F64, name + ".json")))
    cfg = pkg.configs.CONFIGS[name]
    mesh, bvh, cam = pkg.prepare(cfg, f64=True, arith=pkg.ARITH_FMA)
    W, H = cfg["W"], cfg["H"]
    sc = pkg.CpuScene(mesh, bvh)
    try:
        px, rgb, st = sc.render(cam.basis(W, H), np.asarray(cfg["sun"], np.float64), W, H, mode=pkg.cfg_mode(cfg, pkg.ARITH_FMA))
        assert px.dtype == np.float64
        assert hashlib.sha256(pkg.ppm(W, H, rgb)).hexdigest() == meta["ppm_sha256"]["ref"]
        assert (st["rays"], st["hits"]) == (meta["ref"]["rays"], meta["ref"]["hits"])
        with pytest.raises(pkg.CeresError):
            sc.render(cam.basis(W, H), np.asarray(cfg["sun"], np.float64), W, H, mode=pkg.MODE_FULL | pkg.MODE_ROBUST)
        b = np.zeros(12, np.float32)
        s = np.zeros(3, np.float32)
        rc = pkg.lib().ceres_render_cpu_f32(sc._h, pkg._p(b, ctypes.c_float), pkg._p(s, ctypes.c_float), 0, None, None, 4, 4,
                                            None, 0)
        assert rc != 0
    finally:
        sc.close()
