// strtof_fuzz.cpp -- CPU check of csrc/strtof_exact.hpp (the GPU OBJ parser's strtof/strtol)
// against glibc's strtof/strtol, which the reference calls (obj_norms.hpp:36-50,78-80).
// Random decimal / hex / special strings plus a fixed list of hard cases (float midpoints,
// subnormals, overflow boundaries, long mantissas).  Prints "ok N" or the first mismatch.
#include <cerrno>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "strtof_exact.hpp"

using namespace ceres::txt;

static int check(const std::string& s) {
    char* ep = nullptr;
    const float ref = std::strtof(s.c_str(), &ep);
    const long ref_n = long(ep - s.c_str());
    float got = 0.f;
    const long n = strtof_exact(Cursor{s.data(), s.data() + s.size()}, &got);
    uint32_t a, b;
    std::memcpy(&a, &ref, 4); std::memcpy(&b, &got, 4);
    if (a != b || n != ref_n) {
        std::printf("MISMATCH strtof \"%s\": glibc %08x (%ld chars) exact %08x (%ld chars)\n", s.c_str(), a, ref_n, b, n);
        return 1;
    }
    long lv = 0;
    char* ep2 = nullptr;
    const long lref = std::strtol(s.c_str(), &ep2, 10);
    const long ln = strtol10(Cursor{s.data(), s.data() + s.size()}, &lv);
    if (lv != lref || ln != long(ep2 - s.c_str())) {
        std::printf("MISMATCH strtol \"%s\": glibc %ld (%ld) exact %ld (%ld)\n", s.c_str(), lref, long(ep2 - s.c_str()), lv, ln);
        return 1;
    }
    return 0;
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? std::atol(argv[1]) : 2000000;
    std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 12345);
    long total = 0;
    const char* fixed[] = {
        "0", "-0", "+0", "1", "-1", ".5", "5.", ".", "-.", "e5", "1e", "1e+", "1e-", "1e5x", "  \t 3.25",
        "inf", "-INF", "Infinity", "infinit", "nan", "-NaN", "nan(123)", "nan(0x7f)", "nan(abc)", "nan(", "nan()",
        "0x", "0x.", "0x1", "0X1P3", "0x1.8p-3", "0x.8", "0x1p", "0x1p+", "0xAbC.dEfp7", "0x1.fffffep127",
        "0x1.ffffffp127", "0x1p128", "0x1p-149", "0x1p-150", "0x1.8p-150", "0x1p-151", "0x0.0000000000000001p0",
        "0x1.000001p0", "0x1.0000008p0", "0x1.0000018p0", "0x1.00000080000000000001p0",
        "3.4028234663852886e38", "3.4028235677973366e38", "3.4028235677973367e38", "3.40282357e38", "1e39",
        "1.4012984643e-45", "7.006492321624085e-46", "7.006492321624086e-46", "7.0064923216240854e-46",
        "1.1754943508222875e-38", "1.1754942807573643e-38", "2.5e-45", "1e-46", "1e-50",
        "0.100000001490116119384765625", "0.1000000014901161193847656250000000000001",
        "0.10000000149011611938476562", "16777217", "16777216.5", "16777217.0000000000000000000001",
        "33554435", "9007199254740993", "1.00000005960464477539062", "1.000000059604644775390625",
        "1.0000000596046447753906250000001", "-0.0168008", "0.00000000000000000000000000000000000001",
        "123456789012345678901234567890", "1e-7", "0.0000001", "340282346638528859811704183484516925440",
        "1e+38", "1e-38", "0e10000000000", "1e-10000000000", "1e10000000000", "00000000000000000000001",
        "-  1", "- 1", "+-1", "12345678901234567890123", "-9223372036854775808", "9223372036854775808",
        "-9223372036854775809", "2147483648", "1/2/3", "7//8",
    };
    for (const char* f : fixed) { if (check(f)) return 1; ++total; }
    auto digits = [&](int n) { std::string s; for (int i = 0; i < n; ++i) s += char('0' + rng() % 10); return s; };
    for (long it = 0; it < iters; ++it) {
        std::string s;
        const int kind = int(rng() % 10);
        if (kind < 5) {                           // float printed with random precision (OBJ-like)
            const uint32_t bits = uint32_t(rng());
            float f; std::memcpy(&f, &bits, 4);
            if (!std::isfinite(f)) continue;
            char buf[128];
            const int prec = int(rng() % 12) + 1;
            std::snprintf(buf, sizeof buf, (rng() & 1) ? "%.*g" : "%.*e", prec, double(f));
            s = buf;
        } else if (kind < 7) {                    // exact midpoints between floats, +- tiny
            const uint32_t bits = uint32_t(rng()) & 0x7f7fffffu;
            float f; std::memcpy(&f, &bits, 4);
            float g = std::nextafter(f, 1e39f);
            const double mid = (double(f) + double(g)) / 2.0;
            char buf[128];
            std::snprintf(buf, sizeof buf, "%.*g", int(rng() % 30) + 10, mid);
            s = buf;
            if (rng() & 1) s += digits(int(rng() % 5));
        } else if (kind < 8) {                    // long random decimal
            s = digits(int(rng() % 40) + 1);
            if (rng() & 1) s.insert(rng() % (s.size() + 1), ".");
            if (rng() & 1) s += "e" + std::to_string(int(rng() % 100) - 60);
        } else if (kind < 9) {                    // hex float
            char buf[64];
            std::snprintf(buf, sizeof buf, "%a", std::ldexp(double(rng() >> 11) / 9007199254740992.0, int(rng() % 300) - 160));
            s = buf;
        } else {                                  // integers (face indices) and junk
            s = std::to_string(long(rng() % 2000000) - 1000000);
            if (rng() % 3 == 0) s += "/" + std::to_string(rng() % 100);
            if (rng() % 5 == 0) s = digits(int(rng() % 25) + 1);
        }
        if (rng() % 4 == 0) s = "-" + s;
        if (check(s)) return 1;
        ++total;
    }
    std::printf("ok %ld\n", total);
    return 0;
}
