// strtof_exact.hpp -- glibc-compatible strtof / strtol for the GPU OBJ parser (C locale).
//
// obj_norms.hpp:78-80 reads vertex coordinates with std::strtof and face indices with
// std::strtol (obj_norms.hpp:30-53).  The GPU parser must produce the same bits, so this is a
// from-scratch, correctly rounded decimal/hex -> binary32 conversion with glibc's grammar:
// leading isspace, optional sign, "inf"/"infinity"/"nan"/"nan(chars)" (case-insensitive),
// hexadecimal "0x" mantissas with optional binary exponent, decimal mantissas with optional
// exponent; endptr = nptr when nothing converts.  Round-to-nearest-even, overflow to +-inf,
// gradual underflow.
//
// Algorithm: up to 19 significant digits in a u64; exact single-operation fast paths (float,
// then double with a midpoint check against double rounding); otherwise an exact big-integer
// comparison of the decimal value with the binary midpoints around a double-precision guess.
// __host__ __device__ so the same code is fuzzed against glibc on the CPU
// (tools/probes/strtof_fuzz.cpp) and runs in the parser kernels.
#pragma once
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define CERES_HD __host__ __device__
#else
#define CERES_HD
#endif

namespace ceres {
namespace txt {

CERES_HD inline bool is_space(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
CERES_HD inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
CERES_HD inline int hex_val(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
CERES_HD inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? char(c - 'A' + 'a') : c; }

// A bounded C string: characters at [p, e) then an implicit NUL.
struct Cursor {
    const char* p;
    const char* e;
    CERES_HD char at(long i = 0) const { return (p + i < e && p + i >= p) ? p[i] : '\0'; }
};

CERES_HD inline float bits_to_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
CERES_HD inline uint32_t float_to_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
CERES_HD inline uint64_t double_to_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

// ---- small unsigned big integer (little-endian 32-bit limbs) -----------------------------
struct Big {
    static constexpr int kLimbs = 48;       // 1536 bits: covers 120 digits x 10^+-200 scalings
    uint32_t v[kLimbs];
    int n;
    CERES_HD void set(uint64_t x) {
        n = 0;
        while (x) { v[n++] = uint32_t(x); x >>= 32; }
    }
    CERES_HD void mul_small(uint32_t m) {
        uint64_t carry = 0;
        for (int i = 0; i < n; ++i) {
            const uint64_t t = uint64_t(v[i]) * m + carry;
            v[i] = uint32_t(t);
            carry = t >> 32;
        }
        if (carry && n < kLimbs) v[n++] = uint32_t(carry);
    }
    CERES_HD void add_small(uint32_t a) {
        uint64_t carry = a;
        for (int i = 0; i < n && carry; ++i) {
            const uint64_t t = uint64_t(v[i]) + carry;
            v[i] = uint32_t(t);
            carry = t >> 32;
        }
        if (carry && n < kLimbs) v[n++] = uint32_t(carry);
    }
    CERES_HD void mul_pow5(int e) {
        while (e >= 13) { mul_small(1220703125u); e -= 13; }     // 5^13
        uint32_t m = 1;
        while (e-- > 0) m *= 5;
        if (m != 1) mul_small(m);
    }
    CERES_HD void shl(int s) {
        if (n == 0 || s <= 0) return;
        const int w = s / 32, b = s % 32;
        int nn = n + w + 1;
        if (nn > kLimbs) nn = kLimbs;
        for (int i = nn - 1; i >= 0; --i) {
            const int src = i - w;
            uint32_t hi = (src >= 0 && src < n) ? v[src] : 0u;
            uint32_t lo = (src - 1 >= 0 && src - 1 < n) ? v[src - 1] : 0u;
            v[i] = b ? (hi << b) | (lo >> (32 - b)) : hi;
        }
        n = nn;
        while (n > 0 && v[n - 1] == 0) --n;
    }
};
CERES_HD inline int big_cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int i = a.n - 1; i >= 0; --i)
        if (a.v[i] != b.v[i]) return a.v[i] < b.v[i] ? -1 : 1;
    return 0;
}

// Decimal mantissa digits in [m0, m1) (digits and at most one '.'), value = D x 10^exp10.
// Collects up to max_sig significant digits into *sig (u64) or *big; returns the decimal
// exponent of the last collected digit and whether a dropped digit was nonzero.
struct DecDigits {
    const char* m0;
    const char* m1;
    long exp10;                 // explicit exponent part
};

CERES_HD inline void collect_u64(const DecDigits& d, uint64_t& sig, int& nsig, long& e10, bool& sticky) {
    sig = 0; nsig = 0; sticky = false;
    long adj = 0;
    bool frac = false, started = false;
    for (const char* q = d.m0; q < d.m1; ++q) {
        if (*q == '.') { frac = true; continue; }
        const int dg = *q - '0';
        if (!started && dg == 0) { if (frac) --adj; continue; }
        started = true;
        if (nsig < 19) { sig = sig * 10 + uint64_t(dg); ++nsig; if (frac) --adj; }
        else { if (dg) sticky = true; if (!frac) ++adj; }
    }
    e10 = d.exp10 + adj;
}

CERES_HD inline void collect_big(const DecDigits& d, int max_sig, Big& big, long& e10, bool& sticky) {
    big.set(0);
    sticky = false;
    long adj = 0;
    int nsig = 0;
    bool frac = false, started = false;
    for (const char* q = d.m0; q < d.m1; ++q) {
        if (*q == '.') { frac = true; continue; }
        const int dg = *q - '0';
        if (!started && dg == 0) { if (frac) --adj; continue; }
        started = true;
        if (nsig < max_sig) { big.mul_small(10); big.add_small(uint32_t(dg)); ++nsig; if (frac) --adj; }
        else { if (dg) sticky = true; if (!frac) ++adj; }
    }
    e10 = d.exp10 + adj;
}

// float candidate f = k * 2^q (k <= 2^24, q >= -149)
struct Cand { uint64_t k; int q; };
CERES_HD inline Cand cand_from_float(float f) {          // f finite, >= 0
    const uint32_t u = float_to_bits(f);
    const uint32_t be = u >> 23, fr = u & 0x7fffffu;
    if (be == 0) return {fr, -149};
    return {uint64_t(fr) | 0x800000u, int(be) - 150};
}
CERES_HD inline uint32_t cand_bits(Cand c) {             // may overflow to inf
    if (c.k == 0) return 0;
    if (c.k < 0x800000u) return uint32_t(c.k);             // subnormal (q == -149)
    const int be = c.q + 150;
    if (be >= 255) return 0x7f800000u;
    return (uint32_t(be) << 23) | uint32_t(c.k & 0x7fffffu);
}
CERES_HD inline Cand cand_up(Cand c) {
    c.k += 1;
    if (c.k == (1u << 24)) { c.k = 1u << 23; c.q += 1; }
    return c;
}
CERES_HD inline Cand cand_down(Cand c) {
    if (c.k == (1u << 23) && c.q > -149) { c.k = (1u << 24) - 1; c.q -= 1; }
    else c.k -= 1;
    return c;
}
// compare D * 10^e10 (+ sticky) with M * 2^Q; returns -1, 0, +1
CERES_HD inline int cmp_dec_bin(const Big& D, long e10, bool sticky, uint64_t M, int Q) {
    Big a = D, b;
    b.set(M);
    if (e10 >= 0) a.mul_pow5(int(e10)); else b.mul_pow5(int(-e10));
    const long d = e10 - long(Q);                          // powers of two: a has 2^e10, b has 2^Q
    if (d >= 0) a.shl(int(d)); else b.shl(int(-d));
    const int c = big_cmp(a, b);
    if (c == 0 && sticky) return 1;
    return c;
}

CERES_HD inline uint32_t round_decimal_slow(const DecDigits& dd, double approx) {
    Big D;
    long e10;
    bool sticky;
    collect_big(dd, 120, D, e10, sticky);
    float f0 = float(approx);
    if (!(f0 >= 0.0f)) f0 = 0.0f;
    if (f0 > 3.4028234663852886e38f) f0 = 3.4028234663852886e38f;   // start from FLT_MAX when the guess overflowed
    Cand c = cand_from_float(f0);
    for (int it = 0; it < 64; ++it) {
        // upper midpoint (c, c+1): (2k+1) 2^(q-1)
        const int up = cmp_dec_bin(D, e10, sticky, 2 * c.k + 1, c.q - 1);
        if (up > 0 || (up == 0 && (c.k & 1))) {
            if (cand_bits(c) == 0x7f7fffffu) return 0x7f800000u;        // beyond FLT_MAX's upper midpoint
            c = cand_up(c);
            continue;
        }
        if (c.k == 0) break;
        // lower midpoint (c-1, c)
        int lo;
        if (c.k == (1u << 23) && c.q > -149) lo = cmp_dec_bin(D, e10, sticky, (uint64_t(1) << 25) - 1, c.q - 2);
        else lo = cmp_dec_bin(D, e10, sticky, 2 * c.k - 1, c.q - 1);
        if (lo < 0 || (lo == 0 && (c.k & 1))) { c = cand_down(c); continue; }
        break;
    }
    return cand_bits(c);
}

CERES_HD inline double pow10_approx(long e) {          // only a starting guess for the exact path
    double r = 1.0, b = 10.0;
    long x = e < 0 ? -e : e;
    while (x) { if (x & 1) r *= b; b *= b; x >>= 1; }
    return e < 0 ? 1.0 / r : r;
}

// magnitude of a decimal mantissa [m0, m1) x 10^exp -> binary32 bits (sign handled by caller)
CERES_HD inline uint32_t decimal_to_bits(const DecDigits& dd) {
    uint64_t sig; int nsig; long e10; bool sticky;
    collect_u64(dd, sig, nsig, e10, sticky);
    if (sig == 0) return 0u;
    if (e10 + nsig <= -46) return 0u;                      // < 10^-46 < 2^-150: rounds to zero
    if (e10 + nsig - 1 >= 39) return 0x7f800000u;          // >= 10^39: overflow
    if (!sticky && sig < (uint64_t(1) << 24) && e10 >= -10 && e10 <= 10) {
        static constexpr float p10f[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
        const float m = float(sig);                        // exact
        const float r = e10 >= 0 ? m * p10f[e10] : m / p10f[-e10];   // one correctly rounded op
        return float_to_bits(r);
    }
    if (!sticky && sig < (uint64_t(1) << 53) && e10 >= -22 && e10 <= 22) {
        static constexpr double p10d[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                            1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        const double m = double(sig);
        const double r = e10 >= 0 ? m * p10d[e10] : m / p10d[-e10];
        const bool exact = e10 >= 0 && r < 9007199254740992.0 * 1.0;   // integer results below 2^53 are exact
        const uint64_t u = double_to_bits(r);
        const uint64_t low = u & ((uint64_t(1) << 29) - 1);
        // a correctly rounded double that sits exactly on a binary32 midpoint may hide the true
        // side of the midpoint: settle those exactly (the value is never subnormal here)
        if (exact || low != (uint64_t(1) << 28)) return float_to_bits(float(r));
        return round_decimal_slow(dd, r);
    }
    return round_decimal_slow(dd, double(sig) * pow10_approx(e10));
}

// hexadecimal mantissa (digits in [m0, m1), at most one '.') x 2^p2 -> binary32 bits
CERES_HD inline uint32_t hex_to_bits(const char* m0, const char* m1, long p2) {
    uint64_t m = 0;
    int nd = 0;
    bool sticky = false, frac = false, started = false;
    long adj = 0;
    for (const char* q = m0; q < m1; ++q) {
        if (*q == '.') { frac = true; continue; }
        const int h = hex_val(*q);
        if (!started && h == 0) { if (frac) adj -= 4; continue; }
        started = true;
        if (nd < 15) { m = (m << 4) | uint64_t(h); ++nd; if (frac) adj -= 4; }
        else { if (h) sticky = true; if (!frac) adj += 4; }
    }
    if (m == 0) return 0u;
    long e2 = p2 + adj;                                    // value = m * 2^e2 (+ sticky)
    // normalise m to [2^59, 2^60)
    int top = 63;
    while (!((m >> top) & 1)) --top;
    const int sh = 59 - top;
    m <<= sh;
    e2 -= sh;
    // value = m * 2^e2 with m in [2^59, 2^60): the leading bit has weight 2^(e2 + 59)
    const long lead = e2 + 59;
    if (lead > 127) return 0x7f800000u;                    // >= 2^128
    const long keep_lsb = lead >= -126 ? lead - 23 : -149; // weight of the last kept bit
    const long drop = keep_lsb - e2;                       // low bits of m rounded away (>= 36)
    if (drop >= 64) return 0u;                             // below half of 2^-149
    const uint64_t kept = m >> drop;
    const uint64_t rem = m & ((uint64_t(1) << drop) - 1);
    const uint64_t half = uint64_t(1) << (drop - 1);
    const bool round_up = rem > half || (rem == half && (sticky || (kept & 1)));
    Cand c{kept + (round_up ? 1 : 0), int(keep_lsb)};
    if (keep_lsb > -149 && c.k == (uint64_t(1) << 24)) { c.k = 1u << 23; c.q += 1; }
    return cand_bits(c);                                   // subnormal k == 2^23 is the smallest normal
}

CERES_HD inline bool match_ci(Cursor s, long off, const char* word) {
    for (long i = 0; word[i]; ++i)
        if (lower(s.at(off + i)) != word[i]) return false;
    return true;
}

// glibc strtof(nptr, &endptr) on the bounded string; returns the number of characters consumed
// (0 = no conversion, value 0).
CERES_HD inline long strtof_exact(Cursor s, float* out) {
    long i = 0;
    while (is_space(s.at(i))) ++i;
    bool neg = false;
    if (s.at(i) == '+' || s.at(i) == '-') { neg = s.at(i) == '-'; ++i; }
    uint32_t mag;
    long end;
    const char c0 = lower(s.at(i));
    if (c0 == 'i' && match_ci(s, i, "inf")) {
        end = i + 3;
        if (match_ci(s, end, "inity")) end += 5;
        mag = 0x7f800000u;
    } else if (c0 == 'n' && match_ci(s, i, "nan")) {
        end = i + 3;
        mag = 0x7fc00000u;
        if (s.at(end) == '(') {
            long j = end + 1;
            while (true) {
                const char c = s.at(j);
                if (is_digit(c) || (lower(c) >= 'a' && lower(c) <= 'z') || c == '_') { ++j; continue; }
                break;
            }
            if (s.at(j) == ')') {
                // glibc: payload = strtoull(chars, &ep, 0) when it consumes all of them
                uint64_t pay = 0;
                long k = end + 1;
                int base = 10;
                if (s.at(k) == '0' && lower(s.at(k + 1)) == 'x' && hex_val(s.at(k + 2)) >= 0) { base = 16; k += 2; }
                else if (s.at(k) == '0') base = 8;
                bool ok = k < j;
                for (long q = k; q < j; ++q) {
                    const int dv = base == 16 ? hex_val(s.at(q)) : (is_digit(s.at(q)) ? s.at(q) - '0' : -1);
                    if (dv < 0 || dv >= base) { ok = false; break; }
                    pay = pay * uint64_t(base) + uint64_t(dv);
                }
                if (ok) mag = 0x7fc00000u | uint32_t(pay & 0x3fffffu);
                end = j + 1;
            }
        }
    } else if (s.at(i) == '0' && lower(s.at(i + 1)) == 'x' &&
               (hex_val(s.at(i + 2)) >= 0 || (s.at(i + 2) == '.' && hex_val(s.at(i + 3)) >= 0))) {
        long j = i + 2;
        const char* m0 = s.p + j;
        bool dot = false;
        while (hex_val(s.at(j)) >= 0 || (!dot && s.at(j) == '.')) { if (s.at(j) == '.') dot = true; ++j; }
        const char* m1 = s.p + j;
        long p2 = 0;
        if (lower(s.at(j)) == 'p') {
            long k = j + 1;
            bool eneg = false;
            if (s.at(k) == '+' || s.at(k) == '-') { eneg = s.at(k) == '-'; ++k; }
            if (is_digit(s.at(k))) {
                long ev = 0;
                while (is_digit(s.at(k))) { if (ev < 100000000) ev = ev * 10 + (s.at(k) - '0'); ++k; }
                p2 = eneg ? -ev : ev;
                j = k;
            }
        }
        end = j;
        mag = hex_to_bits(m0, m1, p2);
    } else {
        long j = i;
        const char* m0 = s.p + j;
        bool dot = false, any = false;
        while (is_digit(s.at(j)) || (!dot && s.at(j) == '.')) {
            if (s.at(j) == '.') dot = true; else any = true;
            ++j;
        }
        if (!any) { *out = 0.0f; return 0; }                 // no conversion: endptr = nptr
        const char* m1 = s.p + j;
        long e10 = 0;
        if (lower(s.at(j)) == 'e') {
            long k = j + 1;
            bool eneg = false;
            if (s.at(k) == '+' || s.at(k) == '-') { eneg = s.at(k) == '-'; ++k; }
            if (is_digit(s.at(k))) {
                long ev = 0;
                while (is_digit(s.at(k))) { if (ev < 100000000) ev = ev * 10 + (s.at(k) - '0'); ++k; }
                e10 = eneg ? -ev : ev;
                j = k;
            }
        }
        end = j;
        mag = decimal_to_bits(DecDigits{m0, m1, e10});
    }
    *out = bits_to_float(mag | (neg ? 0x80000000u : 0u));
    return end;
}

// glibc strtol(nptr, &endptr, 10) narrowed to int the way obj_norms.hpp:36 stores it
// (`int index = std::strtol(...)`); returns characters consumed (0 = no conversion).
CERES_HD inline long strtol10(Cursor s, long* out) {
    long i = 0;
    while (is_space(s.at(i))) ++i;
    bool neg = false;
    if (s.at(i) == '+' || s.at(i) == '-') { neg = s.at(i) == '-'; ++i; }
    if (!is_digit(s.at(i))) { *out = 0; return 0; }
    uint64_t v = 0;
    bool ovf = false;
    while (is_digit(s.at(i))) {
        const uint64_t d = uint64_t(s.at(i) - '0');
        if (!ovf) {
            if (v > (uint64_t(1) << 63) / 10) ovf = true;
            else {
                v = v * 10 + d;
                if (v > (uint64_t(1) << 63)) ovf = true;
            }
        }
        ++i;
    }
    long r;
    if (neg) r = (ovf || v > (uint64_t(1) << 63)) ? (long)(uint64_t(1) << 63) : (long)(0 - v);
    else r = (ovf || v > uint64_t(0x7fffffffffffffffull)) ? 0x7fffffffffffffffl : long(v);
    *out = r;
    return i;
}

}  // namespace txt
}  // namespace ceres
