/* tools/libm_exhaustive.c — pins csrc/hip/rt_libm.h against this image's glibc libm.
 *
 * Every finite float (both signs) for sinf, asinf and atanf; for atan2f, N random (y, x)
 * pairs of random bit patterns and N pairs of unit-vector components (get_sphere_uv's
 * inputs, hitable.h:14-19).  Prints one line per function: inputs tested, results that
 * differ bitwise.  STRIDE > 1 tests every STRIDE-th float only (the CPU test suite's quick
 * form: tests/test_host_api.py).
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -I<pkg>/csrc/hip tools/libm_exhaustive.c -lm
 *   ./a.out [STRIDE] [ATAN2_PAIRS]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_libm.h"

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float flt(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* NaN results compare equal whatever their payload */
static int same(float a, float b) { return bits(a) == bits(b) || (a != a && b != b); }

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 0) : 1;
    const long pairs = argc > 2 ? atol(argv[2]) : 2000000000L;
    long n1 = 0, d_sin = 0, d_asin = 0, d_atan = 0;
#pragma omp parallel for schedule(dynamic, 1 << 20) reduction(+ : n1, d_sin, d_asin, d_atan)
    for (int64_t b = 0; b < 0x7f800000LL; b += (int64_t)stride) {
        for (int sg = 0; sg < 2; sg++) {
            const float f = flt((uint32_t)b | (sg ? 0x80000000u : 0u));
            n1++;
            d_sin += !same(sinf(f), rt_sinf(f));
            d_asin += !same(asinf(f), rt_asinf(f));
            d_atan += !same(atanf(f), rt_atanf(f));
        }
    }
    printf("sinf   %ld finite floats, %ld differ\n", n1, d_sin);
    printf("asinf  %ld finite floats, %ld differ\n", n1, d_asin);
    printf("atanf  %ld finite floats, %ld differ\n", n1, d_atan);
    long n2 = 0, d2 = 0;
#pragma omp parallel reduction(+ : n2, d2)
    {
        uint64_t s = 0x1234567ull;
#ifdef _OPENMP
        extern int omp_get_thread_num(void);
        s += (uint64_t)omp_get_thread_num() * 0x51ED270B7u;
#endif
#pragma omp for schedule(static)
        for (long i = 0; i < pairs; i++) {
            const uint64_t z = splitmix(&s);
            float y, x;
            if (i & 1) {   /* components of a random unit vector (get_sphere_uv's p.z, p.x) */
                const double a = (double)(z >> 11) * 0x1p-53 * 6.283185307179586, c = (double)(uint32_t)z * 0x1p-32 * 2 - 1;
                const double r = sqrt(1 - c * c);
                y = (float)(r * sin(a)); x = (float)(r * cos(a));
            } else {       /* any two bit patterns */
                y = flt((uint32_t)z); x = flt((uint32_t)(z >> 32));
            }
            n2++;
            d2 += !same(atan2f(y, x), rt_atan2f(y, x));
        }
    }
    printf("atan2f %ld pairs, %ld differ\n", n2, d2);
    return (d_sin || d_asin || d_atan || d2) ? 1 : 0;
}
