"""CPU check of the GPU OBJ parser's number conversion (csrc/strtof_exact.hpp): the reference
reads vertex coordinates with glibc strtof and face indices with strtol (obj_norms.hpp:36-50,
78-80); tools/probes/strtof_fuzz compiles the same __host__ __device__ code for the CPU and
compares value bits and consumed length with glibc on fixed hard cases (float midpoints,
subnormal and overflow boundaries, 40-digit mantissas, hex floats, inf/nan forms) and random
strings."""
import os
import subprocess

import pytest

from conftest import REPO

FUZZ = os.path.join(REPO, "tools", "probes", "strtof_fuzz")


@pytest.mark.parametrize("seed", [1, 7])
def test_strtof_strtol_match_glibc(seed):
    if not os.path.exists(FUZZ):
        pytest.fail("tools/probes/strtof_fuzz missing: run __graft_entry__.build()")
    r = subprocess.run([FUZZ, "400000", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
