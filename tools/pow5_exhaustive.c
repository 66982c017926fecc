/* tools/pow5_exhaustive.c — schlick's pow (material.h:19) on the device (rt_device.h pow5, the
 * correctly rounded x^5 as a double-double) against glibc's pow(x, 5.0), for every float
 * 1 - cosine in [0, 1] and three refractive indices: how many double results differ, and how
 * many of the float reflect_prob the kernel and the reference compute from them differ (the
 * only value the path reads).  Log: profiles/r05/pow5_exhaustive.log.
 *   gcc -O2 -ffp-contract=off tools/pow5_exhaustive.c -lm && ./a.out
 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static double pow5(double x) {
    const double x2 = x * x; const double x4h = x2 * x2; const double x4l = fma(x2, x2, -x4h);
    const double p = x4h * x; const double pe = fma(x4h, x, -p); return p + (pe + x4l * x);
}
int main(void) {
    const float idx[3] = {1.5f, 1.3f, 2.4f};
    for (int k = 0; k < 3; k++) {
        float r0 = (1 - idx[k]) / (1 + idx[k]); r0 = r0 * r0;
        long dd = 0, fd = 0;
        for (uint32_t b = 0; b <= 0x3f800000u; b++) {
            float c; memcpy(&c, &b, 4);            /* 1 - cosine as a float in [0, 1] */
            double a = pow((double)c, 5.0), m = pow5((double)c);
            if (a != m) {
                dd++;
                float fa = (float)(r0 + (double)(1 - r0) * a), fm = (float)(r0 + (double)(1 - r0) * m);
                if (fa != fm) fd++;
            }
        }
        printf("ref_idx %.1f: %ld double results differ, %ld reflect_prob floats differ\n", idx[k], dd, fd);
    }
    return 0;
}
