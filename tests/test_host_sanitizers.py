"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer ("run host code
under -fsanitize=address,undefined").

tools/probes/host_sanitize.cpp drives the product's host C++ (scene_host.cpp: OBJ loader,
rotate_triangles, binned-SAH BVH build, camera basis, anim.cpp orbit, BVH2 -> GPU relayout and
the exact BVH4 collapse, float and double) on the reference meshes, the tiny fixtures and
adversarial OBJ text; any ASan/UBSan report (leaks included) fails the test.  CPU only.
"""
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, REPO

CSRC = os.path.join(REPO, "ceres-raytracer_amd", "csrc")

ADVERSARIAL = {
    # index past the vertex list: an error code, not a crash (obj_norms.hpp:90 asserts)
    "bad_index.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n",
    # negative (relative) indices, v/vt/vn forms, CRLF, tabs, comments, blank and unknown lines
    "mixed.obj": "# c\r\nv 0 0 0\r\nv 1 0 0\r\n\tv 0 1 0\r\nvt 0 0\r\nvn 0 0 1\r\n\r\nf -3/1/1 -2/1/1 -1/1/1\r\ng x\r\ns off\r\n",
    # a 40-gon fan and a zero-area triangle (NaN normals)
    "fan.obj": "".join("v %r %r 0\n" % (i * 0.1, (i * 7 % 5) * 0.1) for i in range(40)) + "f " +
               " ".join(str(i + 1) for i in range(40)) + "\nf 1 1 1\n",
    # no faces, no vertices
    "empty.obj": "# nothing here\n",
    # hex floats, inf/nan literals, exponents at the float range edge
    "numbers.obj": "v 0x1p-3 1e-45 -0\nv inf 1e38 3.4028235e38\nv nan -1e-39 2\nf 1 2 3\n",
}


@pytest.fixture(scope="module")
def sanitized_driver(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("san") / "host_sanitize"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fopenmp", "-ffp-contract=off", "-I" + os.path.join(REPO, "include"),
           "-I" + CSRC, "-D__HIP_PLATFORM_AMD__", os.path.join(REPO, "tools", "probes", "host_sanitize.cpp"),
           os.path.join(CSRC, "scene_host.cpp"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return str(out)


def test_host_code_is_sanitizer_clean(sanitized_driver, tmp_path):
    objs = [os.path.join(REPO, "data", "bunny.obj"), os.path.join(REPO, "data", "dragon.obj")]
    objs += [os.path.join(GOLDEN, n) for n in ("tri1.obj", "quad.obj", "degenerate.obj")]
    for name, text in ADVERSARIAL.items():
        p = tmp_path / name
        p.write_text(text)
        objs.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="4")
    r = subprocess.run([sanitized_driver] + objs, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "host code clean" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "bad_index.obj: load error" in r.stdout
    assert "empty.obj: empty" in r.stdout
