"""CPU proof behind CERES_FAST_PIXQUOT (render_hip.hip pix_quot, primary_dir's render.hpp:109-110
quotient 2 * (i + 0.5) / n): for every image size n <= 65536, every pixel index i < n and EVERY
reciprocal estimate within one ulp of 1/n (so whatever v_rcp_f32 returns), one correction step
q = fma(fma(-n, q0, a), r0, q0) gives the correctly rounded quotient.  6.4e9 checks, ~6 s on 8
threads (tools/probes/pixquot_cpu_check.c)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_fast_pixel_quotient_exact_for_any_one_ulp_reciprocal(tmp_path):
    exe = tmp_path / "pixquot_cpu"
    src = os.path.join(REPO, "tools", "probes", "pixquot_cpu_check.c")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", src, "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pairs x estimates 6442549248 mismatches 0" in r.stdout, r.stdout
