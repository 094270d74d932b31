"""pow24f (csrc/pow24.hpp, used by the GPU shading) == (float)glibc pow((double)x, 24.0).

Exhaustive over every float with 2^-12 <= |x| < 64 (both signs; outside that range the float
result is +0 or +inf), plus random bit patterns -- the reference's blinn_phong_spec
(render.hpp:51-54) evaluates std::pow(float, int) in double.
"""
import os
import subprocess

from conftest import PKG_DIR

SRC = r'''
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include "pow24.hpp"
static bool same(float a, float b) { uint32_t x, y; std::memcpy(&x, &a, 4); std::memcpy(&y, &b, 4); return x == y || (std::isnan(a) && std::isnan(b)); }
int main() {
    long bad = 0, n = 0;
    for (uint32_t u = 0x39800000u; u < 0x42800000u; ++u) {
        float x; std::memcpy(&x, &u, 4);
        for (float y : {x, -x}) { n++; if (!same(ceres::pow24f(y), (float)std::pow((double)y, 24.0))) bad++; }
    }
    std::mt19937 rng(7);
    for (int i = 0; i < 20000000; ++i) {
        uint32_t u = rng(); float x; std::memcpy(&x, &u, 4);
        n++; if (!same(ceres::pow24f(x), (float)std::pow((double)x, 24.0))) bad++;
    }
    for (float x : {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, 1e-30f, 64.0f, 64.00001f}) { n++; if (!same(ceres::pow24f(x), (float)std::pow((double)x, 24.0))) bad++; }
    std::printf("%ld %ld\n", bad, n);
    return bad != 0;
}
'''


def test_pow24_matches_glibc_pow_exhaustively(tmp_path):
    src = tmp_path / "p.cpp"
    src.write_text(SRC)
    exe = tmp_path / "p"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-I" + os.path.join(PKG_DIR, "csrc"),
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    bad, n = map(int, r.stdout.split())
    assert bad == 0 and n > 300_000_000
