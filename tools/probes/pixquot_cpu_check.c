/* CPU proof for render_hip.hip's pix_quot (CERES_FAST_PIXQUOT): for every image size n in
 * [1, 65536] and every pixel index i < n, with a = 2 * (i + 0.5f) (exact) and ANY reciprocal
 * estimate r0 within one ulp of the correctly rounded 1/n (v_rcp_f32's documented accuracy),
 *     q = fma(fma(-n, q0, a), r0, q0),  q0 = a * r0
 * equals the correctly rounded a / n.  Checks r0 = RN(1/n) and its two float neighbours, i.e. every
 * value the hardware estimate can return, so the result holds whatever v_rcp_f32 returns.
 * Build: gcc -O2 -fopenmp -ffp-contract=off tools/probes/pixquot_cpu_check.c -o /tmp/pixquot_cpu -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

static float nextf(float x, int dir) { return nextafterf(x, dir > 0 ? INFINITY : -INFINITY); }

int main(void) {
    unsigned long long bad = 0, pairs = 0;
    long long first_n = -1, first_i = -1;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : bad, pairs)
    for (int n = 1; n <= 65536; ++n) {
        const float fn = (float)n;
        const float rn = 1.0f / fn;
        const float cand[3] = {nextf(rn, -1), rn, nextf(rn, +1)};
        for (int i = 0; i < n; ++i) {
            const float a = 2.0f * ((float)i + 0.5f);
            const float exact = a / fn;
            for (int c = 0; c < 3; ++c) {
                const float r0 = cand[c];
                const float q0 = a * r0;
                const float q = fmaf(fmaf(-fn, q0, a), r0, q0);
                ++pairs;
                if (q != exact) {
                    ++bad;
#pragma omp critical
                    if (first_n < 0) { first_n = n; first_i = i; }
                }
            }
        }
    }
    printf("pairs x estimates %llu mismatches %llu", pairs, bad);
    if (bad) printf(" first n=%lld i=%lld", first_n, first_i);
    printf("\n");
    return bad != 0;
}
