/* tests/native/div_rn_check.c — the megakernel's division by a shared reciprocal
 * (rt_device.h div_rn): with y = RN(1/b), q = RN(x*y), r = fma(-q, b, x) (exact) and
 * fma(r, y, q) must equal the IEEE quotient RN(x/b) (Markstein's theorem) for every
 * x, b whose reciprocal and quotient are normal floats.  Random pairs over a wide
 * exponent range plus the kernel's own shapes: image coordinates (px + u) / nx,
 * normals (p - c) / r, unit vectors d / |d|, ray distances / |d|^2, sphere roots.
 * Usage: div_rn_check [N]; prints the mismatch count, exit status 1 on any. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xs(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static float rf(int emin, int emax) {
    uint32_t m = (uint32_t)xs() & 0x7FFFFF;
    int e = emin + (int)(xs() % (uint64_t)(emax - emin + 1));
    uint32_t bits = ((uint32_t)(e + 127) << 23) | m | ((xs() & 1) ? 0x80000000u : 0);
    float f;
    memcpy(&f, &bits, 4);
    return f;
}
static float div_rn(float x, float b, float y) {
    volatile float q = x * y;   /* no contraction: the kernel's v_mul_f32 */
    return fmaf(fmaf(-q, b, x), y, q);
}
static long bad = 0;
static void check(float x, float b) {
    volatile float y = 1.0f / b;
    volatile float ref = x / b;
    if (!isnormal(y) || !isnormal(ref)) return;
    float got = div_rn(x, b, y);
    if (memcmp(&got, (const void *)&ref, 4) != 0) {
        if (bad < 10) printf("mismatch x=%a b=%a ieee=%a div_rn=%a\n", x, b, (double)ref, (double)got);
        bad++;
    }
}
int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 20000000L;
    for (long i = 0; i < n; i++) {
        check(rf(-60, 60), rf(-60, 60));                                       /* wide range */
        int nx = 1 + (int)(xs() % 4096);
        check((float)((double)(xs() % (uint64_t)nx) + (double)(xs() >> 16) * 0x1p-48), (float)nx); /* camera */
        float r = rf(-8, 12);
        check(r * (1.0f + rf(-24, -1)), r);                                     /* normal component */
        float a = rf(-4, 4), c = rf(-4, 4), d = rf(-4, 4);
        float len = sqrtf(a * a + c * c + d * d);
        check(a, len);                                                          /* unit vector */
        check(rf(-10, 14), a * a + c * c + d * d);                              /* distance / |d|^2 */
        {   /* a sphere's roots (-b -+ sqrt(disc)) / |d|^2, sphere.h:33-40 (prim_t_head, sphere_t) */
            float ox = rf(-2, 10), oy = rf(-2, 10), oz = rf(-2, 10), rad = rf(-4, 10);
            float aa = a * a + c * c + d * d, bb = ox * a + oy * c + oz * d;
            float cc = ox * ox + oy * oy + oz * oz - rad * rad, disc = bb * bb - aa * cc;
            if (disc > 0) {
                check(-bb - sqrtf(disc), aa);
                check(-bb + sqrtf(disc), aa);
            }
        }
    }
    printf("%ld mismatches in %ld x 5-7 divisions\n", bad, n);
    return bad != 0;
}
