// pow24.hpp -- (float)std::pow((double)x, 24) without the general pow (render.hpp:53).
//
// The reference's Blinn-Phong term calls std::pow(float, int), which promotes to the double
// pow(double, double) and narrows the result to float.  Evaluating that general double pow
// on the GPU costs ~700 f64 instructions per call (3 calls per lit pixel).  x^24 is computed
// here as x^2 (exact in double) -> x^4 -> x^8 -> x^16 -> x^16 * x^8 in double-double
// arithmetic (error ~2^-100 relative), rounded once to double -- i.e. the correctly rounded
// pow -- and then narrowed to float exactly like the reference.
// tests/test_pow24.py checks it against glibc's pow for EVERY float with 2^-12 <= |x| < 64
// (below that the float result is +0, above it +inf) plus random bit patterns.
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define CERES_HD __host__ __device__ __forceinline__
#else
#define CERES_HD inline
#endif

namespace ceres {

CERES_HD void dd_square(double h, double l, double& H, double& L) {
    const double p = h * h;
    double e = std::fma(h, h, -p);
    e = std::fma(2.0 * h, l, e);
    H = p + e;
    L = e - (H - p);
}

CERES_HD void dd_mul(double ah, double al, double bh, double bl, double& H, double& L) {
    const double p = ah * bh;
    double e = std::fma(ah, bh, -p);
    e = std::fma(ah, bl, e);
    e = std::fma(al, bh, e);
    H = p + e;
    L = e - (H - p);
}

CERES_HD float pow24f(float xf) {
    const double x = xf;
    if (!(std::fabs(x) <= 64.0)) return std::isnan(xf) ? xf : INFINITY;   // |x|^24 > 2^144 -> +inf in float
    const double x2 = x * x;                                               // exact (48-bit product)
    double h4, l4, h8, l8, h16, l16, h24, l24;
    dd_square(x2, 0.0, h4, l4);
    dd_square(h4, l4, h8, l8);
    dd_square(h8, l8, h16, l16);
    dd_mul(h16, l16, h8, l8, h24, l24);
    return static_cast<float>(h24 + l24);
}

}  // namespace ceres
