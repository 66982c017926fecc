// tests/native/log_check.cpp — host check of the device log (rt_device.h: log_f64)
// against glibc's log on u48 inputs (the counter stream's draws), run by
// tests/test_host_api.py.  Prints: samples, max ulp difference, count of samples
// whose float hit_distance (constant_medium.h:36) differs for several densities.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "rt_device.h"

int main(int argc, char **argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
    const float densities[] = {0.0001f, 0.01f, 0.2f, 1.0f, 7.5f};
    unsigned long long state = 0x9E3779B97F4A7C15ull;
    long maxulp = 0, fdiff = 0, tested = 0;
    auto check = [&](double u) {
        const double a = std::log(u), b = log_f64(u);
        long long ia, ib;
        __builtin_memcpy(&ia, &a, 8);
        __builtin_memcpy(&ib, &b, 8);
        const long d = (long)std::llabs(ia - ib);
        if (d > maxulp) maxulp = d;
        for (float den : densities) {
            const float fa = (float)((double)(-(1 / den)) * a), fb = (float)((double)(-(1 / den)) * b);
            if (fa != fb) fdiff++;
        }
        tested++;
    };
    for (long i = 0; i < n; i++) {
        state = state * 6364136223846793005ull + 1442695040888963407ull;
        check((double)(state >> 16) * 0x1p-48);
    }
    // edges: the smallest draws, values around the path switch and next to 1
    for (long m = 1; m < 4096; m++) check((double)m * 0x1p-48);
    for (long m = -2048; m < 2048; m++) check(0.9375 + (double)m * 0x1p-48);
    for (long m = 1; m < 4096; m++) check(1.0 - (double)m * 0x1p-48);
    std::printf("%ld %ld %ld\n", tested, maxulp, fdiff);
    return 0;
}
