// pow24.hpp -- (float)std::pow((double)x, 24) without the general pow (render.hpp:53).
//
// The reference's Blinn-Phong term calls std::pow(float, int), which promotes to the double
// pow(double, double) and narrows the result to float.  Evaluating that general double pow
// on the GPU costs ~700 f64 instructions per call (3 calls per lit pixel).
//
// pow24f (float input, the float render path): x^2 (exact in double: a 48-bit product), then
// x^4, x^8, x^16 and x^16 * x^8 in plain double -- four roundings, a relative error below 2^-51,
// so the double result can differ from the correctly rounded x^24 only in its last bits, and
// narrowing to float hides that unless the exact value lies within 2^-51 of a float rounding
// boundary.  No float does: tests/test_pow24.py checks pow24f against glibc's correctly rounded
// pow for EVERY float with 2^-12 <= |x| < 64 (below that the float result is +0, above it +inf)
// plus random bit patterns -- 0 mismatches (round 3; the previous double-double evaluation, 31
// f64 instructions per call against these 5 multiplications, gave the same bits).
//
// dd_square / dd_mul (double-double, error ~2^-100) stay for the double render path
// (render64.hip), whose input is a double and cannot be checked exhaustively.
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
    const double x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8;
    return static_cast<float>(x16 * x8);
}

}  // namespace ceres
