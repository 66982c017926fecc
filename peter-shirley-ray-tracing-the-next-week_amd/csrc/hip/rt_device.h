// rt_device.h — device code of the path-tracing megakernel (rt_kernel.hip): vectors, the counter
// RNG, primitive tests and hit records (the reference's hitable classes), textures
// and Perlin noise, the BVH node step, and the wave-cooperative samplers.
// Arithmetic follows the reference's float/double promotions; compiled with
// -ffp-contract=off (only the BVH slab test uses explicit FMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "rt_layout.h"
#include "rt_libm.h"
#include "rt_log_table.h"
#include "rt_kernel.h"

#define RT_FLT_MAX 0x1.fffffep+127f
// Values the shading stage and the samplers leave unset where no lane reads them
// (default copies kept alive across branches cost register moves; some of them, left
// unset, made the allocator spill instead — those stay initialised):
// Such a value is FROZEN (unset_f: LLVM `freeze` of poison — an arbitrary but defined
// value, so the compiler may pick whatever saves a move), never an uninitialised read:
// reading an indeterminate value is undefined behaviour the compiler may exploit (round
// 4's build with bits 16-64 left uninitialised faulted in the empty-scene case).
#ifndef RT_SHADE_LEAN
#define RT_SHADE_LEAN 117   // bits: 1 scatter outputs, 2 hit record, 4 texture value, 8 jitter, 16 rejection
                            // points, 32 noise scale, 64 unit direction (2, 8: spills, off)
#endif
#define RT_INF __builtin_huge_valf()
// The float transcendentals of the path (texture sines, get_sphere_uv's atan2/asin) are
// glibc's (rt_libm.h, exhaustively pinned); ocml's forms, which differ from glibc's on
// 18-40 % of the call sites' inputs, remain only in rt_math_probe for the comparison.

namespace {

// Wave ballot of a bool: the lane mask itself (HIP's __ballot takes an int, and the
// int round trip can materialise the mask as 0/1 per lane and compare it again).
__device__ __forceinline__ uint64_t wballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

// ------------------------------------------------------------------ vec3
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float a, float b, float c) { V3 r; r.x = a; r.y = b; r.z = c; return r; }
// a value no lane reads (RT_SHADE_LEAN): whatever the VGPR the register allocator gives
// an empty asm's output holds — a defined value to the compiler (no undefined behaviour
// to exploit), materialised by no instruction, so a join of it with a computed value
// costs no move (LLVM's freeze, __builtin_nondeterministic_value, is folded to a
// constant instead: 55 more v_movs in c4's variant than uninitialised values)
__device__ __forceinline__ float unset_f() {
    float x;
    asm volatile("; unset %0" : "=v"(x));
    return x;
}
__device__ __forceinline__ V3 unset_v3() { return mk(unset_f(), unset_f(), unset_f()); }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 scale(float t, V3 v) { return mk(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ V3 divs(V3 v, float t) { return mk(v.x / t, v.y / t, v.z / t); }
__device__ __forceinline__ V3 neg(V3 v) { return mk(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(V3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ V3 unit(V3 v) { return divs(v, len(v)); }
__device__ __forceinline__ float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

struct Ray { V3 o, d; float time; };

// x / b, correctly rounded, from y = RN(1/b) (Markstein): q = RN(x*y); the remainder
// x - b*q is exact as one FMA, and RN(q + r*y) = RN(x / b) whenever y is a normal
// float and the quotient neither overflows nor underflows (tests/native/div_rn_check.c
// compares it with IEEE division on 4e8 random pairs).  3 VALU instead of the ~11 of
// an IEEE division; callers take it only when every lane's y is normal (a wave-uniform
// test) and their quotients are O(1) (unit vectors, normals, image coordinates) or
// ray distances, else the IEEE division.
__device__ __forceinline__ float div_rn(float x, float b, float y) {
    const float q = x * y;
    return __builtin_fmaf(__builtin_fmaf(-q, b, x), y, q);
}
__device__ __forceinline__ V3 divs_rn(V3 v, float t, float y) { return mk(div_rn(v.x, t, y), div_rn(v.y, t, y), div_rn(v.z, t, y)); }
__device__ __forceinline__ bool normal_recip(float y) {
    const float m = __builtin_fabsf(y);
    return m >= 0x1p-126f && m <= 0x1.fffffep+127f;
}
// A divisor shared by several divisions of a lane: a, y = RN(1/a) (one IEEE division),
// and whether the wave may divide by it with div_rn (every lane that uses it has a
// normal reciprocal).
struct Recip { float a, y; bool ok; };
__device__ __forceinline__ Recip recip_of(float a, bool use) {
    Recip r;
    r.a = a;
    r.y = 1.0f / a;
    r.ok = wballot(use && !normal_recip(r.y)) == 0ull;
    return r;
}
__device__ __forceinline__ float div_by(float x, const Recip &r) { return r.ok ? div_rn(x, r.a, r.y) : x / r.a; }
__device__ __forceinline__ V3 at(const Ray &r, float t) { return add(r.o, scale(t, r.d)); }

// ------------------------------------------------------------------- RNG
// Per-sample drand48 streams: sample (pixel, s) runs drand48's own
// generator (x = a x + c mod 2^48, draw = x / 2^48; the reference's drand48,
// main.cpp:305-306, camera.h:45-53, material.h:44-118) from x0 = key mod 2^48, key =
// mix64(seed_key ^ (pixel << 32 | s)); constant_medium draws come from a second
// drand48 stream of the sample, from mix64(key ^ 0xD1B5..) mod 2^48, stepped once per
// medium and segment whether or not the medium draws (media_hit), so the draw of
// medium k at segment d is its (d * nmedia + k + 1)-th value.  Random access for the cooperative samplers: x_{n+j} = A_j x_n + C_j, with
// (A_j, C_j) from a table (RT_LCG_JUMPS entries, LDS).
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kLcgA = 0x5DEECE66Dull, kLcgC = 0xBull, kLcgM = 0xFFFFFFFFFFFFull;
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// (z >> 16) * 2^-48, built as the double 1 + (z >> 16) * 2^-48 (the 48 bits as the
// top of the 52-bit mantissa) minus 1: both steps exact, so the same value as the
// integer conversion, for one f64 add instead of two conversions, a scale and an add.
__device__ __forceinline__ double u48(uint64_t z) {
    const uint64_t bits = 0x3FF0000000000000ull | ((z >> 12) & 0x000FFFFFFFFFFFF0ull);
    return __longlong_as_double((long long)bits) - 1.0;
}
// x * 2^-48 for a 48-bit state, the same way
__device__ __forceinline__ double u48x(uint64_t x) {
    return __longlong_as_double((long long)(0x3FF0000000000000ull | (x << 4))) - 1.0;
}
// One drand48 step, mod 2^48 with 32-bit operations: a = 5 * 2^32 + 0xDEECE66D, x =
// xh * 2^32 + xl (xh < 2^16), so a x = 0xDEECE66D xl + (5 xl + 0xDEECE66D xh) 2^32
// (mod 2^48): one v_mad_u64_u32 (+ c) and two multiply-adds into the high word, of
// which only 16 bits are kept — so 16 x 16-bit products suffice (v_mad_u32_u16).
// The four instructions are spelled out: from the C form, p = xl * 0xDEECE66D + c and
// hi = (p >> 32) + 5 xl + 0xDEECE66D xh, the compiler built the high word as a 64-bit sum
// (three v_mad_u64_u32, two of them by 0, a 64-bit add and two moves; round 4: c4 -0.3 %).
// The same values either way (the GPU parity tests are bitwise).
__device__ __forceinline__ uint64_t lcg_step(uint64_t x) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    static_assert(kLcgC == 11, "the drand48 increment is the inline constant of v_mad_u64_u32 below");
    uint64_t p, cy;   // cy: the carry-out SGPR pair gfx9 requires (unused)
    uint32_t hi;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 11" : "=v"(p), "=s"(cy) : "v"(xl), "s"(0xDEECE66Du));
    asm("v_mad_u32_u16 %0, %1, 5, %2" : "=v"(hi) : "v"(xl), "v"((uint32_t)(p >> 32)));
    asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(hi) : "v"(xh), "s"(0xE66Du), "v"(hi));
    return ((uint64_t)(hi & 0xFFFFu) << 32) | (uint32_t)p;
}
// j steps at once: x_{n+j} = A_j x_n + C_j (mod 2^48); jt = (A_j lo, A_j hi, C_j lo, C_j hi)
typedef unsigned U4j __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint64_t lcg_jump(uint64_t x, U4j jt) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint64_t c = ((uint64_t)jt.w << 32) | jt.z;
    uint64_t p, cy;
    uint32_t hi;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(p), "=s"(cy) : "v"(xl), "v"(jt.x), "v"(c));   // wraps mod 2^64: 48 bits kept
    asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(hi) : "v"(xl), "v"(jt.y), "v"((uint32_t)(p >> 32)));
    asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(hi) : "v"(xh), "v"(jt.x), "v"(hi));
    return ((uint64_t)(hi & 0xFFFFu) << 32) | (uint32_t)p;
}
// Jumps of 0 .. RT_LCG_JUMPS - 1 steps: a cooperative round's candidate t of an owner
// drawing K per candidate starts K t <= 3 * 63 steps on, and an owner advances by K
// tried <= 3 * 64 (coop_reject).
#define RT_LCG_JUMPS 193
struct LcgJumpTable {
    U4j e[RT_LCG_JUMPS];
    constexpr LcgJumpTable() : e() {
        uint64_t A = 1, C = 0;
        for (int j = 0; j < RT_LCG_JUMPS; ++j) {
            e[j] = U4j{(uint32_t)A, (uint32_t)(A >> 32), (uint32_t)C, (uint32_t)(C >> 32)};
            A = (A * kLcgA) & kLcgM;
            C = (C * kLcgA + kLcgC) & kLcgM;
        }
    }
};
__constant__ const LcgJumpTable kLcgJump = LcgJumpTable();
typedef __attribute__((address_space(3))) const U4j LdsJump;   // the table's LDS copy (ds_read_b128)

// key of sample (pixel, sample): mix64(seed_key ^ (pixel << 32 | sample)) with
// seed_key = mix64(seed ^ 0x5851F42D4C957F2D), computed once per launch
__device__ __forceinline__ uint64_t seed_key(uint64_t seed) { return mix64(seed ^ 0x5851F42D4C957F2Dull); }
__device__ __forceinline__ uint64_t sample_key(uint64_t skey, uint32_t pixel, uint32_t sample) {
    return mix64(skey ^ (((uint64_t)pixel << 32) | sample));
}
struct Rng {
    uint64_t x;      // the sample's drand48 state
    uint64_t xm;     // its medium stream's state (media_hit steps it once per medium and segment)
    // media = false: the scene has no constant_medium, so the medium stream is never read
    __device__ __forceinline__ void start(uint64_t k, bool media = true) {
        x = k & kLcgM;
        xm = media ? mix64(k ^ 0xD1B54A32D192ED03ull) & kLcgM : 0;
    }
    __device__ __forceinline__ double next() { x = lcg_step(x); return u48x(x); }
    __device__ __forceinline__ void skip() { x = lcg_step(x); }   // a draw whose value is not used
    __device__ __forceinline__ void skip2() { x = lcg_step(lcg_step(x)); }   // two of them (a constant jump's
                                                                            // 64-bit addend got hoisted and spilled)
};

// Natural log in double for x in [0, 1) — constant_medium's log(drand48())
// (constant_medium.h:36).  glibc's log is within ~0.52 ulp; so is this, and its
// result only feeds a float rounding of (double)(-1/density) * log(u), which a
// last-bit difference changes with probability ~2^-29.  Table path (glibc's
// scheme): x = 2^k z, z in [0.6875, 1.375), log x = k ln2 + log(1/invc) + log1p(r),
// r = fma(z, invc, -1), |r| < 0.004, log(1/invc) a double-double from
// tools/gen_log_table.py.  The row for [1 - 2^-8, 1) has invc = 1 and log(1/invc) = 0,
// so next to 1 the result is r + r^2 p(r) with r = x - 1 exact: relatively accurate
// without glibc's separate near-1 path (a branch nearly every wave took for some lane).
// About 25 double operations instead of ocml's ~100.
// The polynomial's coefficients (none of them an inline constant) come in `pc`: the
// megakernel passes them from LDS (read at the call), since as immediates the compiler
// kept them in VGPRs across the whole persistent loop and spilled them.
struct LogConsts { double c07, c06, c02, c025, c03; };   // the polynomial's coefficients
__host__ __device__ __forceinline__ double log_f64(double x, LogConsts pc = LogConsts{1.0 / 7, -1.0 / 6, 0.2, -0.25, 1.0 / 3}) {
    if (!(x > 0.0)) return -__builtin_huge_val();
    uint64_t ix;
    __builtin_memcpy(&ix, &x, 8);
    const uint64_t tmp = ix - RT_LOG_OFF;
    const int i = (int)((tmp >> 45) & (RT_LOG_N - 1));
    const int64_t k = (int64_t)tmp >> 52;
    const uint64_t iz = ix - (tmp & (0xFFFull << 52));
    double z;
    __builtin_memcpy(&z, &iz, 8);
    const double *T = rt_log_table[i];
    const double r = __builtin_fma(z, T[0], -1.0);
    const double kd = (double)k;
    const double ln2_hi = 0x1.62e42fefa3800p-1, ln2_lo = 0x1.ef35793c76730p-45;   // kd * ln2_hi exact
    const double w = __builtin_fma(kd, ln2_hi, T[1]);   // kd * ln2_hi is exact: same as mul + add
    const double hi = w + r;
    const double lo = (w - hi) + r + __builtin_fma(kd, ln2_lo, T[2]);
    const double r2 = r * r;
    double q = __builtin_fma(r, pc.c07, pc.c06);
    q = __builtin_fma(q, r, pc.c02);
    q = __builtin_fma(q, r, pc.c025);
    q = __builtin_fma(q, r, pc.c03);
    q = __builtin_fma(q, r, -0.5);
    const double p = r2 * q;
    return (lo + p) + hi;
}

// pow(x, 5.0) for the x = (double)(float) of schlick (material.h:19).  x has 24
// significant bits, so x*x is exact; x^4 and x^5 are carried as double-double and
// rounded once: the double result is the correctly rounded x^5 except in
// vanishingly rare near-ties, i.e. what glibc's pow returns, at a fraction of
// ocml's general pow cost (and register pressure).
__device__ __forceinline__ double pow5(double x) {
    const double x2 = x * x;
    const double x4h = x2 * x2;
    const double x4l = __builtin_fma(x2, x2, -x4h);
    const double p = x4h * x;
    const double pe = __builtin_fma(x4h, x, -p);
    return p + (pe + x4l * x);
}

// ----------------------------------------------------------- scene access
__device__ __forceinline__ float4 ld4(const float4 *p, uint32_t i) { return p[i]; }
__device__ __forceinline__ int fbits(float f) { return __float_as_int(f); }

// BVH slab test primitives: packed FP32 FMA for the lo/hi plane pairs, IEEE
// min/max (minnum: a NaN plane distance from an axis-parallel ray leaves that axis
// unconstrained, i.e. conservative).  Plain builtins, not inline asm: the
// compiler forms v_min3/v_max3 itself, and inline asm would make its hazard
// recognizer pad the sequence with s_nop (an issue slot each).
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ F2 pk_fma(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float vmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float vmin3(float a, float b, float c) { return vmin(vmin(a, b), c); }
__device__ __forceinline__ float vmax3(float a, float b, float c) { return vmax(vmax(a, b), c); }

// Ray into the object space of an instance chain (hitable.h:66-67, 129-135).
__device__ __forceinline__ Ray to_object(const float4 *insts, int inst, Ray r) {
    const float4 *I = insts + inst * 7;
    int nops = fbits(I[0].x);
    for (int k = 0; k < nops; ++k) {
        float4 op = I[1 + k];
        int code = fbits(op.x);
        if (code == RT_OP_TRANSLATE) {
            r.o = sub(r.o, mk(op.y, op.z, op.w));
        } else if (code == RT_OP_ROTATE_Y) {
            float s = op.y, c = op.z;
            V3 o = r.o, d = r.d;
            o.x = c * r.o.x - s * r.o.z;
            o.z = s * r.o.x + c * r.o.z;
            d.x = c * r.d.x - s * r.d.z;
            d.z = s * r.d.x + c * r.d.z;
            r.o = o; r.d = d;
        }
    }
    return r;
}
// The same for a wave-uniform chain (flat-scan groups, pre-scanned primitives): the
// records through the scalar cache (constant address space, uniform index), the op
// codes in SGPRs and scalar branches, instead of a chain of dependent vector loads.
typedef float F4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const F4v ConstInst;
__device__ __forceinline__ Ray to_object_uniform(const float4 *insts, int inst, Ray r) {
    const ConstInst *I = (const ConstInst *)insts + inst * 7;
    const int nops = fbits(I[0].x);
    for (int k = 0; k < nops; ++k) {
        const F4v op = I[1 + k];
        const int code = fbits(op.x);
        if (code == RT_OP_TRANSLATE) {
            r.o = sub(r.o, mk(op.y, op.z, op.w));
        } else if (code == RT_OP_ROTATE_Y) {
            const float s = op.y, c = op.z;
            V3 o = r.o, d = r.d;
            o.x = c * r.o.x - s * r.o.z;
            o.z = s * r.o.x + c * r.o.z;
            d.x = c * r.d.x - s * r.d.z;
            d.z = s * r.d.x + c * r.d.z;
            r.o = o; r.d = d;
        }
    }
    return r;
}

// Hit point / normal back to world space, innermost wrapper first (hitable.h:43-45, 69, 137-145).
__device__ __forceinline__ void to_world(const float4 *insts, int inst, V3 &p, V3 &n) {
    const float4 *I = insts + inst * 7;
    int nops = fbits(I[0].x);
    for (int k = nops - 1; k >= 0; --k) {
        float4 op = I[1 + k];
        int code = fbits(op.x);
        if (code == RT_OP_TRANSLATE) {
            p = add(p, mk(op.y, op.z, op.w));
        } else if (code == RT_OP_ROTATE_Y) {
            float s = op.y, c = op.z;
            V3 q = p, m = n;
            q.x = c * p.x + s * p.z;
            q.z = -s * p.x + c * p.z;
            m.x = c * n.x + s * n.z;
            m.z = -s * n.x + c * n.z;
            p = q; n = m;
        } else if (code == RT_OP_FLIP) {
            n = neg(n);
        }
    }
}

// Candidate hit distance of one primitive for a search starting at t_min with no
// upper bound (RT_INF = miss).  The caller keeps the closest (t, key) pair, which
// reproduces hitable_list's sequential `t < closest` / `t <= closest` acceptance.
__device__ __forceinline__ float sphere_t(V3 c, float rad, const Ray &r, float tmin) {   // sphere.h:25-52
    V3 oc = sub(r.o, c);
    float a = dot(r.d, r.d);
    float b = dot(oc, r.d);
    float cc = dot(oc, oc) - rad * rad;
    float disc = b * b - a * cc;
    if (disc > 0) {
        float t = (-b - sqrtf(disc)) / a;
        if (t < RT_FLT_MAX && t > tmin) return t;
        t = (-b + sqrtf(disc)) / a;
        if (t < RT_FLT_MAX && t > tmin) return t;
    }
    return RT_INF;
}

__device__ __forceinline__ V3 msphere_center(float4 g0, float4 g1, float4 g2, float time) {   // sphere.h:81-83
    return add(mk(g0.x, g0.y, g0.z), scale((time - g1.w) / g2.x, mk(g1.x, g1.y, g1.z)));
}

// One rect test for a plane axis (aarect.h:50-100); oa/da: ray along the plane
// normal, (oi, di) and (oj, dj): the two in-plane axes.  Written once per kind
// with direct field reads so the compiler never indexes the ray through memory.
__device__ __forceinline__ float plane_t(float oa, float da, float oi, float di, float oj, float dj, float4 g0, float k,
                                         float tmin) {
    float t = (k - oa) / da;
    if (t < tmin || t > RT_FLT_MAX) return RT_INF;
    float a = oi + t * di;
    float b = oj + t * dj;
    if (a < g0.x || a > g0.y || b < g0.z || b > g0.w) return RT_INF;
    return t;
}
__device__ __forceinline__ float rect_t(int kind, float4 g0, float k, const Ray &r, float tmin) {
    if (kind == RT_PRIM_XY_RECT) return plane_t(r.o.z, r.d.z, r.o.x, r.d.x, r.o.y, r.d.y, g0, k, tmin);
    if (kind == RT_PRIM_XZ_RECT) return plane_t(r.o.y, r.d.y, r.o.x, r.d.x, r.o.z, r.d.z, g0, k, tmin);
    return plane_t(r.o.x, r.d.x, r.o.y, r.d.y, r.o.z, r.d.z, g0, k, tmin);
}

// prim kinds: 0 sphere, 1 moving sphere, 2 xy, 3 xz, 4 yz  (rect axis = 2, 1, 0)
__device__ __forceinline__ int rect_axis(int kind) { return 4 - kind; }

// Test of one primitive whose 32-B head (g0, mm) is already loaded.  Written
// for a wave whose lanes test different kinds: the sphere terms and the rect's
// plane terms are computed with selects rather than per-kind branches, and the
// first quotient — (-b - sqrt(disc)) / a for a sphere (sphere.h:33), (k - o_a) / d_a
// for a rect (aarect.h:51) — is ONE IEEE division either way.  Every value is the
// same float the per-kind code computes (same operands, same operations); only
// the moving-sphere centre and a sphere's second root stay behind branches.
// kInst = false: the scene has no instance chains (the host knows), so the kernel
// carries no instance code at all (fewer registers live across the leaf tests).
// kKinds: what the WAVE tests in this call — 1 spheres only, 2 rects only, 3 both
// (the caller ballots the kinds): a uniform wave skips the other kind's terms
// (sphere-only: no plane selects; rect-only: no quadratic and no square root).
template <bool kInst = true, int kKinds = 3>
__device__ __forceinline__ float prim_t_head(float4 g0, float4 mm, const float4 *P, const float4 *insts, uint32_t idx,
                                             const Ray &r0, float tmin, int &key, int &kind_out) {
    const int kind = fbits(mm.x) & 0xff;
    const int inst = fbits(mm.z);
    const int order = fbits(mm.w);
    kind_out = kind | (kInst && inst >= 0 ? 0x100 : 0);
    Ray r = r0;
    if (kInst && inst >= 0) r = to_object(insts, inst, r0);
    const bool sph = kKinds == 1 ? true : (kKinds == 2 ? false : kind <= RT_PRIM_MOVING_SPHERE);
    key = sph ? order : -1 - order;   // a later rect wins a tie (aarect.h:52 accepts t == t_max)
    // sphere.h:25-52 (moving: the centre at r.time, sphere.h:81-83)
    V3 c = mk(g0.x, g0.y, g0.z);
    if (kKinds != 2 && kind == RT_PRIM_MOVING_SPHERE) c = msphere_center(g0, P[idx * 4 + 2], P[idx * 4 + 3], r.time);
    const V3 oc = sub(r.o, c);
    const float a = dot(r.d, r.d);
    const float b = dot(oc, r.d);
    const float cc = dot(oc, oc) - g0.w * g0.w;
    const float disc = b * b - a * cc;
    const float sq = sqrtf(disc);
    // aarect.h:50-100: ray along the plane normal (oa, da) and the two in-plane axes
    const bool xy = kind == RT_PRIM_XY_RECT, xz = kind == RT_PRIM_XZ_RECT;
    const float oa = xy ? r.o.z : (xz ? r.o.y : r.o.x), da = xy ? r.d.z : (xz ? r.d.y : r.d.x);
    const float oi = xy || xz ? r.o.x : r.o.y, di = xy || xz ? r.d.x : r.d.y;
    const float oj = xy ? r.o.y : r.o.z, dj = xy ? r.d.y : r.d.z;
    const float t = (sph ? -b - sq : mm.y - oa) / (sph ? a : da);
    if (sph) {
        if (!(disc > 0)) return RT_INF;
        if (t < RT_FLT_MAX && t > tmin) return t;
        const float t2 = (-b + sq) / a;
        return (t2 < RT_FLT_MAX && t2 > tmin) ? t2 : RT_INF;
    }
    if (t < tmin || t > RT_FLT_MAX) return RT_INF;
    const float ai = oi + t * di, bj = oj + t * dj;
    return (ai < g0.x || ai > g0.y || bj < g0.z || bj > g0.w) ? RT_INF : t;
}

template <bool kInst = true>
__device__ __forceinline__ float prim_t(const float4 *P, const float4 *insts, uint32_t idx, const Ray &r0, float tmin,
                                        int &key, int &kind_out) {
    return prim_t_head<kInst>(P[idx * 4 + 0], P[idx * 4 + 1], P, insts, idx, r0, tmin, key, kind_out);
}

struct Hit { V3 p, n; float u, v; int mat; };

// get_sphere_uv (hitable.h:14-19): float atan2/asin, then the double M_PI arithmetic.
__device__ __forceinline__ void sphere_uv(V3 p, float &u, float &v) {
    const float phi = rt_atan2f(p.z, p.x);
    const float theta = rt_asinf(p.y);
    u = (float)(1 - ((double)phi + 3.14159265358979323846) / (2 * 3.14159265358979323846));
    v = (float)(((double)theta + 3.14159265358979323846 / 2) / 3.14159265358979323846);
}

// Rebuilds the reference's hit_record for the winning primitive (sphere.h:34-38,
// 103-106; aarect.h:58-63; hitable.h:43-45, 69, 137-145).
// (u, v) is computed only for materials whose texture reads it (an image texture):
// every other texture ignores it (texture.h:22-56).
// kUV = false: no material of the scene reads (u, v) (no image texture), so the
// uv code (sphere: atan2/asin + double divisions) is not compiled in.
template <bool kInst = true, bool kUV = true>
__device__ __forceinline__ Hit prim_record(const float4 *P, const float4 *insts, const float4 *mats, uint32_t idx,
                                           const Ray &r0, float t) {
    const float4 g0 = P[idx * 4 + 0];
    const float4 mm = P[idx * 4 + 1];
    int kind = fbits(mm.x) & 0xff;
    int flip = (fbits(mm.x) >> 8) & 1;
    int inst = fbits(mm.z);
    Ray r = r0;
    if (kInst && inst >= 0) r = to_object(insts, inst, r0);
    Hit h;
    h.p = at(r, t);
    // sphere normals (p - c) / radius (sphere.h:37, 105): mm.y = RN(1/radius) from the
    // host (0 when not a normal float: then every lane of the wave divides exactly)
    const bool rn = wballot(kind <= RT_PRIM_MOVING_SPHERE && mm.y == 0.f) == 0ull;
    if (kind == RT_PRIM_SPHERE) {
        const V3 v = sub(h.p, mk(g0.x, g0.y, g0.z));
        h.n = rn ? divs_rn(v, g0.w, mm.y) : divs(v, g0.w);
    } else if (kind == RT_PRIM_MOVING_SPHERE) {
        const V3 v = sub(h.p, msphere_center(g0, P[idx * 4 + 2], P[idx * 4 + 3], r.time));
        h.n = rn ? divs_rn(v, g0.w, mm.y) : divs(v, g0.w);
    } else {
        int axis = rect_axis(kind);
        h.n = mk(axis == 0 ? 1.f : 0.f, axis == 1 ? 1.f : 0.f, axis == 2 ? 1.f : 0.f);
    }
    h.u = 0.f;
    h.v = 0.f;
    h.mat = fbits(mm.x) >> 9;
    if (kUV && (fbits(mats[h.mat * 2 + 1].w) & 1)) {
        if (kind == RT_PRIM_SPHERE) {
            sphere_uv(h.n, h.u, h.v);   // sphere.h:36: the same (p - center) / radius, before any flip
        } else if (kind != RT_PRIM_MOVING_SPHERE) {                          // aarect.h:54-59
            float oi, di, oj, dj;
            if (kind == RT_PRIM_XY_RECT) { oi = r.o.x; di = r.d.x; oj = r.o.y; dj = r.d.y; }
            else if (kind == RT_PRIM_XZ_RECT) { oi = r.o.x; di = r.d.x; oj = r.o.z; dj = r.d.z; }
            else { oi = r.o.y; di = r.d.y; oj = r.o.z; dj = r.d.z; }
            const float a = oi + t * di, b = oj + t * dj;
            h.u = (a - g0.x) / (g0.y - g0.x);
            h.v = (b - g0.z) / (g0.w - g0.z);
        }
    }
    if (flip) h.n = neg(h.n);
    if (kInst && inst >= 0) to_world(insts, inst, h.p, h.n);
    return h;
}

// Closest boundary hit of a constant_medium (its own small list), t > / >= tmin.
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask);
// true on exactly one active lane: counts a wave-level event once per wave
__device__ __forceinline__ bool first_active() { return lanes_below(wballot(1)) == 0; }

struct Counters {
    uint64_t samples = 0, segments = 0, nodes = 0, spheres = 0, mspheres = 0, rects = 0, instanced = 0, media = 0,
             shades = 0, noise = 0;
    // wave-level trip counts (SIMD efficiency = lane-level count / (64 x wave-level count))
    uint64_t w_iters = 0, w_nodes = 0, w_prims = 0, w_rius = 0, l_rius = 0;
    // material divergence of the shading stage: wave passes through the scatter
    // branches, the distinct materials each pass ran, and the lanes that scattered
    uint64_t w_shade = 0, w_kinds = 0, l_scatter = 0;
    uint64_t ball[RT_BALL_N] = {0, 0, 0, 0, 0, 0, 0, 0};   // the ball waves (rt_layout.h RT_BALL_*), wave-level
    __device__ __forceinline__ void prim(int kind) {
        const int k = kind & 0xff;
        if (k == RT_PRIM_SPHERE) spheres++;
        else if (k == RT_PRIM_MOVING_SPHERE) mspheres++;
        else rects++;
        if (kind & 0x100) instanced++;
    }
};

template <bool kCount, bool kInst = true>
__device__ __forceinline__ float boundary_t(const float4 *B, const float4 *insts, int first, int count, const Ray &r,
                                            float tmin, Counters &cnt) {
    float best = RT_INF;
    for (int q = 0; q < count; ++q) {
        int key, kind;
        float t = prim_t<kInst>(B, insts, (uint32_t)(first + q), r, tmin, key, kind);
        if (kCount) cnt.prim(kind);
        if (t < best) best = t;
    }
    return best;
}

// ----------------------------------------------------------------- Perlin
// One noise() (perlin.h:43-61, 25-39).  The six permutation reads are issued
// together, then the eight gradient reads: two memory round trips per call.
// (RV / PM: the tables' pointer types — global memory, or final()'s variant's LDS copies)
template <class RV, class PM>
__device__ __forceinline__ float perlin_noise(RV ranvec, PM perm, V3 p) {
    float u = p.x - floorf(p.x);
    float v = p.y - floorf(p.y);
    float w = p.z - floorf(p.z);
    u = u * u * (3 - 2 * u);
    v = v * v * (3 - 2 * v);
    w = w * w * (3 - 2 * w);
    const int i = (int)floorf(p.x);
    const int j = (int)floorf(p.y);
    const int k = (int)floorf(p.z);
    const float uu = u * u * (3 - 2 * u);
    const float vv = v * v * (3 - 2 * v);
    const float ww = w * w * (3 - 2 * w);
    const int px[2] = {perm[i & 255], perm[(i + 1) & 255]};
    const int py[2] = {perm[256 + (j & 255)], perm[256 + ((j + 1) & 255)]};
    const int pz[2] = {perm[512 + (k & 255)], perm[512 + ((k + 1) & 255)]};
    float accum = 0;   // corner order i, j, k as perlin_interp sums them
#pragma unroll 1
    for (int a = 0; a < 2; ++a) {
        V3 g[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const auto t = ranvec[px[a] ^ py[c >> 1] ^ pz[c & 1]];
            g[c] = mk(t.x, t.y, t.z);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int b = c >> 1, d = c & 1;
            V3 weight_v = mk(u - a, v - b, w - d);
            accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) * (d * ww + (1 - d) * (1 - ww)) *
                     dot(g[c], weight_v);
        }
    }
    return accum;
}

// Texture chain of one lane down to its leaf: checker_texture picks a child by
// the sign of the sines (texture.h:35-44).  Returns the leaf kind (-1: chain too deep).
// kChecker = false: the scene has no checker_texture, the leaf is the material's own.
template <bool kChecker = true>
__device__ __forceinline__ int tex_leaf(const RtKernelArgs &A, int ti, V3 p, float4 &t0, float4 &t1) {
    if (!kChecker) {
        t0 = A.texs[ti * 2 + 0];
        t1 = A.texs[ti * 2 + 1];
        return fbits(t0.x);
    }
    for (int guard = 0; guard < RT_MAX_CHECKER_DEPTH; ++guard) {
        t0 = A.texs[ti * 2 + 0];
        t1 = A.texs[ti * 2 + 1];
        const int kind = fbits(t0.x);
        if (kind != RT_TEX_CHECKER) return kind;
        float sines = rt_sinf(10 * p.x) * rt_sinf(10 * p.y) * rt_sinf(10 * p.z);
        ti = (sines < 0) ? fbits(t0.z) : fbits(t0.y);
    }
    return -1;
}

// texture::value of a constant or image leaf (texture.h:16-27; surface_texture.h:19-30);
// the noise leaf is finished after coop_turb.
template <bool kUV = true>
__device__ __forceinline__ V3 tex_value_leaf(const RtKernelArgs &A, int kind, float4 t0, float4 t1, float u, float v) {
    if (kind == RT_TEX_CONSTANT) return mk(t1.x, t1.y, t1.z);
    if (kUV && kind == RT_TEX_IMAGE) {   // stride 3 as the reference addresses it
        const int nx = fbits(t0.y), ny = fbits(t0.z);
        const uint8_t *data = A.texels + fbits(t0.w);
        int i = (int)((1 - u) * nx);
        int j = (int)((double)((1 - v) * ny) - 0.001);
        if (i < 0) i = 0;
        if (j < 0) j = 0;
        if (i > nx - 1) i = nx - 1;
        if (j > ny - 1) j = ny - 1;
        const float r = (float)((int)data[3 * i + 3 * nx * j] / 255.0);
        const float gg = (float)((int)data[3 * i + 3 * nx * j + 1] / 255.0);
        const float b = (float)((int)data[3 * i + 3 * nx * j + 2] / 255.0);
        return mk(r, gg, b);
    }
    return mk(0, 0, 0);
}

// ------------------------------------------------------------ BVH node step
// Per-ray slab-test constants: 1/d (padded boxes need no exact division) and
// -o/d, duplicated into packed pairs for v_pk_fma_f32.
// LDS nodes (LdsNodes::load_signed): lx/ly/lz are the byte offsets of the ray's
// near planes in the axis' plane (+4 when the direction is negative: hi before lo).
// kSplit = 1: every value of a node in a plane of its own, one dword
// per node — 14 planes of RT_LDS_NODE_CAP dwords: the child references c0, c1, then x-lo,
// x-hi, y-lo, y-hi, z-lo, z-hi of child 0 and child 1 in turn (RtSplit) — so the values of
// both children for one axis and side are one plane (4 KiB) apart and load as one
// ds_read2st64_b32; 56 KiB instead of 64.  The media variants (final()) use it: final() c4
// 51.52 -> 51.33 ms, its c5 rank share of 8 26.77 -> 26.63, c5 199.5 -> 198.6, while the
// random scenes' variant measured slower with it (c3 44.06 -> 44.28) and keeps the float4
// planes (profiles/r05/ab_lds_split_layouts.log).  The gain is not fewer bank conflicts —
// it has more: the LDS has 32 banks and both values of a pair fall in one (0.26 -> 0.33 of
// the LDS-active cycles); blocks of 32 nodes conflict the same, an odd 15-dword node stride
// conflicts least (0.20) and was slower on final() (+0.45 %): profiles/r05/lds_layouts/.
enum RtSplit { RS_C0 = 0, RS_C1 = 1, RS_XLO = 2, RS_XHI = 4, RS_YLO = 6, RS_YHI = 8, RS_ZLO = 10, RS_ZHI = 12, RS_PLANES = 14 };
// The LDS node layout of a kernel variant: dword planes for the media variants' BVH2 in
// LDS (final()), float4 planes otherwise (the layout each measured fastest)
__host__ __device__ constexpr int rt_lds_split(int mode, int feat, int width) {
    return (mode == 1 && (feat & RT_FEAT_MEDIA) != 0 && width == 2) ? 1 : 0;
}
#define RT_SPLIT_PB (RT_LDS_NODE_CAP * 4)   // bytes per dword plane
// node bytes of the LDS layout (the host asks rt_lds_need_bytes for its scene's variant)
template <int kSplit>
constexpr uint32_t lds_node_bytes() { return kSplit ? RS_PLANES * RT_SPLIT_PB : RT_LDS_NODE_BYTES; }
// an interior node's reference: its byte offset in a plane
template <int kSplit>
__host__ __device__ __forceinline__ uint32_t lds_node_ref(uint32_t n) { return kSplit ? n * 4 : n * 16; }
struct Slab { F2 ix, iy, iz, nox, noy, noz; float tmin; uint32_t lx, ly, lz, fx, fy, fz; };
template <int kSplit = 0>
__device__ __forceinline__ Slab make_slab(const Ray &r, float tmin) {
    const float ix = __builtin_amdgcn_rcpf(r.d.x), iy = __builtin_amdgcn_rcpf(r.d.y), iz = __builtin_amdgcn_rcpf(r.d.z);
    Slab s;
    s.ix = F2{ix, ix}; s.iy = F2{iy, iy}; s.iz = F2{iz, iz};
    s.nox = F2{-r.o.x * ix, -r.o.x * ix}; s.noy = F2{-r.o.y * iy, -r.o.y * iy}; s.noz = F2{-r.o.z * iz, -r.o.z * iz};
    s.tmin = tmin;
    if (kSplit) {
        const uint32_t sx = __float_as_uint(ix) >> 31, sy = __float_as_uint(iy) >> 31, sz = __float_as_uint(iz) >> 31;
        s.lx = (RS_XLO + 2 * sx) * RT_SPLIT_PB; s.fx = (RS_XHI - 2 * sx) * RT_SPLIT_PB;
        s.ly = (RS_YLO + 2 * sy) * RT_SPLIT_PB; s.fy = (RS_YHI - 2 * sy) * RT_SPLIT_PB;
        s.lz = (RS_ZLO + 2 * sz) * RT_SPLIT_PB; s.fz = (RS_ZHI - 2 * sz) * RT_SPLIT_PB;
    } else {
        s.lx = ((__float_as_uint(ix) >> 31) << 2) + RT_LDS_NODE_CAP * 16;
        s.ly = ((__float_as_uint(iy) >> 31) << 2) + 2 * RT_LDS_NODE_CAP * 16;
        s.lz = ((__float_as_uint(iz) >> 31) << 2) + 3 * RT_LDS_NODE_CAP * 16;
        s.fx = s.lx ^ 4u; s.fy = s.ly ^ 4u; s.fz = s.lz ^ 4u;
    }
    return s;
}
// entry distance of one child box, +inf if the ray misses it (or, kSlots, the slot
// is empty: BVH4 nodes may have unused slots; BVH2 interior nodes never do)
// [tn, tf] of one child box (a hit iff tn <= tf; NaN slabs are ignored by min/max)
// The clamps to [tmin, best_t] are signed-integer max/min on the float bits: exact
// when either operand is >= 0, and when both are negative they pick the value
// further out (tn lower, tf higher), i.e. conservative; a NaN from all three axes
// (zero direction) culls the box, where the primitives could not be hit either.
// Float min/max would need tmin and best_t canonicalised in every step (3 VALU).
__device__ __forceinline__ float imax(float a, float b) { return __int_as_float(max(__float_as_int(a), __float_as_int(b))); }
__device__ __forceinline__ float imin(float a, float b) { return __int_as_float(min(__float_as_int(a), __float_as_int(b))); }
__device__ __forceinline__ void box_span(const Slab &s, F2 x, F2 y, F2 z, float best_t, float &tn, float &tf) {
    const F2 a = pk_fma(x, s.ix, s.nox), b = pk_fma(y, s.iy, s.noy), e = pk_fma(z, s.iz, s.noz);
    tn = imax(vmax3(vmin(a.x, a.y), vmin(b.x, b.y), vmin(e.x, e.y)), s.tmin);
    tf = imin(vmin3(vmax(a.x, a.y), vmax(b.x, b.y), vmax(e.x, e.y)), best_t);
}
template <bool kSlots>
__device__ __forceinline__ float box_entry(const Slab &s, F2 x, F2 y, F2 z, float best_t, uint32_t c) {
    float tn, tf;
    box_span(s, x, y, z, best_t, tn, tf);
    return (tn <= tf && (!kSlots || c != RT_EMPTY_CHILD)) ? tn : RT_INF;
}
__device__ __forceinline__ void cas(float &ka, uint32_t &ca, float &kb, uint32_t &cb) {
    const bool sw = kb < ka;
    const float tk = sw ? kb : ka;
    kb = sw ? ka : kb;
    ka = tk;
    const uint32_t tc = sw ? cb : ca;
    cb = sw ? ca : cb;
    ca = tc;
}
// One interior node: test the children, push the hit ones but the nearest far to
// near (branch-free: a slot is written, then kept only if the child was hit; the
// builder bounds sp by RT_STACK_DEPTH - 1), return the nearest (or empty).
// Where a node step reads its node.  BVH2 nodes are 4 float4 (rt_layout.h); the
// global reader fetches them from HBM (L1/L2), the LDS reader from the workgroup's
// copy, stored as 4 planes of RT_LDS_NODE_CAP float4 so that lanes reading different
// nodes spread over 16 bank windows instead of 4 (the plane contents: load_signed).
typedef __attribute__((address_space(3))) const F4v LdsF4;
__device__ __forceinline__ float4 f4(F4v v) { return make_float4(v.x, v.y, v.z, v.w); }
struct GlobalNodes {
    const float4 *p;
    __device__ __forceinline__ void load2(uint32_t n, float4 &b0, float4 &b1, float4 &b2, float4 &cf) const {
        const float4 *N = p + n * 4;
        b0 = N[0]; b1 = N[1]; b2 = N[2]; cf = N[3];
    }
    __device__ __forceinline__ const float4 *ptr4(uint32_t n) const { return p + n * 8; }
    __device__ __forceinline__ const float4 *ptr8(uint32_t n) const { return p + n * 16; }
    __device__ __forceinline__ const float4 *ptr8q(uint32_t n) const { return p + n * 8; }
};
// LDS planes, per axis: plane 0 holds the child references (first,
// so that their read needs no address add: the LDS base fits the immediate offset),
// plane 1 + a (lo0, hi0, lo1, hi1) of axis a for both children.  A lane reads its near planes at
// +0 or +4 by the sign of its direction (Slab::lx..lz) and its far planes at the
// other word: near/far come out of the load, not out of a min and a max per axis
// and child (12 VALU per node step for 6 address adds; the node's 4 float4 read by
// four ds_read_b128, round 2: c4 56.95 -> 55.68 ms).
template <int kSplit = 0>
struct LdsNodes {   // node references are byte offsets (n * 16, kSplit: n * 4) into the planes
    const LdsF4 *p;
    // the six plane offsets become LDS addresses once per round, opaque to the
    // compiler, which would otherwise re-split base + plane + sign per node step
    // (11 address adds per node instead of 6)
    static __device__ __forceinline__ uint32_t opaque(uint32_t x) { asm("" : "+v"(x)); return x; }
    __device__ __forceinline__ void prepare(Slab &s) const {
        const uint32_t b = (uint32_t)(size_t)p;
        s.lx = opaque(b + s.lx); s.ly = opaque(b + s.ly); s.lz = opaque(b + s.lz);
        s.fx = opaque(b + s.fx); s.fy = opaque(b + s.fy); s.fz = opaque(b + s.fz);
    }
    // after prepare()
    __device__ __forceinline__ void load_signed(uint32_t n, const Slab &s, F2 &nx, F2 &ny, F2 &nz, F2 &fx, F2 &fy, F2 &fz,
                                                uint32_t &c0, uint32_t &c1) const {
        typedef __attribute__((address_space(3))) const float LdsF;
        typedef __attribute__((address_space(3))) const char LdsC;
        if constexpr (kSplit) {
            auto pair = [&](uint32_t a) {   // (child 0, child 1): one plane apart, one ds_read2st64_b32
                const LdsF *q = (const LdsF *)(size_t)(n + a);
                return F2{q[0], q[RT_LDS_NODE_CAP]};
            };
            nx = pair(s.lx); fx = pair(s.fx);
            ny = pair(s.ly); fy = pair(s.fy);
            nz = pair(s.lz); fz = pair(s.fz);
            typedef __attribute__((address_space(3))) const uint32_t LdsU;
            const LdsU *C = (const LdsU *)((LdsC *)p + n);
            c0 = C[0]; c1 = C[RT_LDS_NODE_CAP];
        } else {
            auto pair = [&](uint32_t a) {   // (child 0, child 1) at one address: one ds_read2_b32
                const LdsF *q = (const LdsF *)(size_t)(n + a);
                return F2{q[0], q[2]};
            };
            nx = pair(s.lx); fx = pair(s.fx);
            ny = pair(s.ly); fy = pair(s.fy);
            nz = pair(s.lz); fz = pair(s.fz);
            typedef unsigned U2v __attribute__((ext_vector_type(2)));
            const __attribute__((address_space(3))) U2v *C =
                (const __attribute__((address_space(3))) U2v *)((LdsC *)p + n);
            const U2v c = *C;
            c0 = c.x; c1 = c.y;
        }
    }
    __device__ __forceinline__ const float4 *ptr4(uint32_t) const { return nullptr; }   // wide BVHs stay in HBM
    __device__ __forceinline__ const float4 *ptr8(uint32_t) const { return nullptr; }
    __device__ __forceinline__ const float4 *ptr8q(uint32_t) const { return nullptr; }
};

// The traversal stack: one column per lane, [depth][lane] (a wave's push or pop is one
// conflict-free ds_write_b32 / ds_read_b32), addressed by the depth `sp` with one shift-add.
// (sp as a byte offset, depth x 256, makes the address one add but turns the conditional
// +-1 steps, carry-in adds, into selects: c4 51.54 -> 51.68 ms with 8 B spilled, round 5.)
#define RT_SP_UNIT 1
__device__ __forceinline__ uint32_t &stk_at(uint32_t *stk, int sp) {   // one shift-add per address
    return *reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(stk) + ((uint32_t)sp << 8));
}
// The BVH2-in-LDS stacks hold 16-bit entries (round 6): [depth][lane] of
// int16, 128 B per depth level, half the LDS of 32-bit entries (final(): 56 -> 28 KiB per CU,
// the room of the ball waves' path pools).  An interior reference there is a byte offset into
// the node planes (< 16 KiB) and a leaf is encoded by the LDS copy as
// 0xFFFF8000 | (count - 1) << 12 | first (first < 4096: rt_scene_create keeps scenes of more
// primitives out of LDS), so an entry is the reference's low 16 bits and the sign-extending
// read (ds_read_i16) restores it — no encode or decode instruction on a push or a pop.
#define RT_LDS_LEAF16(ref) (0xFFFF8000u | ((RT_LEAF_COUNT(ref) - 1u) << 12) | RT_LEAF_FIRST(ref))
#define RT_LDS_LEAF16_FIRST(ref) ((ref) & 0xFFFu)
#define RT_LDS_LEAF16_COUNT(ref) ((((ref) >> 12) & 0x7u) + 1u)
__device__ __forceinline__ void stk16_put(uint32_t *stk, int sp, uint32_t v) {
    *reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(stk) + ((uint32_t)sp << 7)) = (uint16_t)v;
}
__device__ __forceinline__ uint32_t stk16_get(uint32_t *stk, int sp) {
    return (uint32_t)(int32_t) * reinterpret_cast<int16_t *>(reinterpret_cast<char *>(stk) + ((uint32_t)sp << 7));
}

// 8-wide node step's tail: the nearest hit child (the first one in slot order on
// ties) is the next node, the other hit children are pushed in reverse slot order.
// The builder puts the children in slots by direction from the node's centre (slot
// bit a set = the child lies on the + side of axis a), so rays going + on all axes
// pop the nearer siblings first; siblings are not sorted per ray: an 8-key sort
// costs more VALU than the box tests themselves.
__device__ __forceinline__ uint32_t wide8_tail(const float k[8], const uint32_t ch[8], uint32_t *stk, int &sp) {
    const float kmin = vmin(vmin3(vmin3(k[0], k[1], k[2]), vmin3(k[3], k[4], k[5]), k[6]), k[7]);
    int sel = 8;   // the first slot holding the nearest hit (8: no hit)
#pragma unroll
    for (int c = 7; c >= 0; --c) sel = (k[c] != RT_INF && k[c] == kmin) ? c : sel;
    uint32_t next = RT_EMPTY_CHILD;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        next = c == sel ? ch[c] : next;
    }
#pragma unroll
    for (int c = 7; c >= 0; --c) {   // slot written, then kept only if pushed
        stk_at(stk, sp) = ch[c];
        sp += (k[c] != RT_INF && c != sel) ? RT_SP_UNIT : 0;
    }
    return next;
}

// One interior node: test the children, push the hit ones but the nearest far to
// near (branch-free: a slot is written, then kept only if the child was hit; the
// builder bounds sp by the BVH depth), return the nearest (or empty).
template <int kWidth, class Nodes>
__device__ __forceinline__ uint32_t node_step(const Nodes &src, uint32_t node, const Slab &s, float best_t, uint32_t *stk,
                                              int &sp) {
    if constexpr (kWidth == 2 && !std::is_same<Nodes, GlobalNodes>::value) {
        F2 nx, ny, nz, fx, fy, fz;
        uint32_t c0, c1;
        src.load_signed(node, s, nx, ny, nz, fx, fy, fz, c0, c1);
        // both children per packed FMA: .x child 0, .y child 1
        const F2 an = pk_fma(nx, s.ix, s.nox), bn = pk_fma(ny, s.iy, s.noy), en = pk_fma(nz, s.iz, s.noz);
        const F2 af = pk_fma(fx, s.ix, s.nox), bf = pk_fma(fy, s.iy, s.noy), ef = pk_fma(fz, s.iz, s.noz);
        const float tn0 = imax(vmax3(an.x, bn.x, en.x), s.tmin), tf0 = imin(vmin3(af.x, bf.x, ef.x), best_t);
        const float tn1 = imax(vmax3(an.y, bn.y, en.y), s.tmin), tf1 = imin(vmin3(af.y, bf.y, ef.y), best_t);
        const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
        const bool lt = tn1 < tn0;
        const bool second = h1 & (!h0 | lt);
        const uint32_t nearc = second ? c1 : (h0 ? c0 : RT_EMPTY_CHILD), farc = second ? c0 : c1;
        stk16_put(stk, sp, farc);
        const int sp0 = h0 ? sp + RT_SP_UNIT : sp;
        sp = h1 ? sp0 : sp;
        return nearc;
    } else if (kWidth == 2) {   // rt_dnode2
        float4 b0, b1, b2, cf;
        src.load2(node, b0, b1, b2, cf);
        const uint32_t c0 = (uint32_t)fbits(cf.x), c1 = (uint32_t)fbits(cf.y);
        // hit flags and the order as lane masks (SALU), not +inf entry keys compared
        // and selected per lane: 3 compares instead of 5 compares and 7 selects, and
        // no compare -> select hazard waits (s_nop) between them
        float tn0, tf0, tn1, tf1;
        box_span(s, F2{b0.x, b0.y}, F2{b0.z, b0.w}, F2{b1.x, b1.y}, best_t, tn0, tf0);
        box_span(s, F2{b1.z, b1.w}, F2{b2.x, b2.y}, F2{b2.z, b2.w}, best_t, tn1, tf1);
        const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;   // a hit's entry is finite (tf <= best_t)
        const bool lt = tn1 < tn0;
        const bool second = h1 & (!h0 | lt);           // ties: child 0 first (no short circuit: no branch)
        const uint32_t nearc = second ? c1 : (h0 ? c0 : RT_EMPTY_CHILD), farc = second ? c0 : c1;
        stk_at(stk, sp) = farc;                        // kept only if both children were hit
        const int sp0 = h0 ? sp + RT_SP_UNIT : sp;
        sp = h1 ? sp0 : sp;
        return nearc;
    } else if (kWidth == 8) {   // rt_dnode8
        const float4 *N = src.ptr8(node);
        float4 q[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) q[i] = N[i];
        const float4 c0 = N[12], c1 = N[13];
        const uint32_t ch[8] = {(uint32_t)fbits(c0.x), (uint32_t)fbits(c0.y), (uint32_t)fbits(c0.z), (uint32_t)fbits(c0.w),
                                (uint32_t)fbits(c1.x), (uint32_t)fbits(c1.y), (uint32_t)fbits(c1.z), (uint32_t)fbits(c1.w)};
        float k[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int p = c >> 1;
            const float4 x = q[p], y = q[4 + p], z = q[8 + p];
            k[c] = (c & 1) ? box_entry<true>(s, F2{x.z, x.w}, F2{y.z, y.w}, F2{z.z, z.w}, best_t, ch[c])
                           : box_entry<true>(s, F2{x.x, x.y}, F2{y.x, y.y}, F2{z.x, z.y}, best_t, ch[c]);
        }
        return wide8_tail(k, ch, stk, sp);
    } else if (kWidth == RT_BVH_CW8) {   // rt_dnode8q: planes origin + q * 2^e, in ray space
        const float4 *N = src.ptr8q(node);
        const float4 h = N[0], qx = N[1], qy = N[2], qz = N[3], c0 = N[4], c1 = N[5];
        const uint32_t ch[8] = {(uint32_t)fbits(c0.x), (uint32_t)fbits(c0.y), (uint32_t)fbits(c0.z), (uint32_t)fbits(c0.w),
                                (uint32_t)fbits(c1.x), (uint32_t)fbits(c1.y), (uint32_t)fbits(c1.z), (uint32_t)fbits(c1.w)};
        const uint32_t eb = (uint32_t)fbits(h.w);
        // t(plane q) = (origin + q * step - o) / d = q * (step / d) + (origin - o) / d
        const float ax = __uint_as_float((eb & 0xFFu) << 23) * s.ix.x, bx = __builtin_fmaf(h.x, s.ix.x, s.nox.x);
        const float ay = __uint_as_float(((eb >> 8) & 0xFFu) << 23) * s.iy.x, by = __builtin_fmaf(h.y, s.iy.x, s.noy.x);
        const float az = __uint_as_float(((eb >> 16) & 0xFFu) << 23) * s.iz.x, bz = __builtin_fmaf(h.z, s.iz.x, s.noz.x);
        const uint32_t wx[4] = {(uint32_t)fbits(qx.x), (uint32_t)fbits(qx.y), (uint32_t)fbits(qx.z), (uint32_t)fbits(qx.w)};
        const uint32_t wy[4] = {(uint32_t)fbits(qy.x), (uint32_t)fbits(qy.y), (uint32_t)fbits(qy.z), (uint32_t)fbits(qy.w)};
        const uint32_t wz[4] = {(uint32_t)fbits(qz.x), (uint32_t)fbits(qz.y), (uint32_t)fbits(qz.z), (uint32_t)fbits(qz.w)};
        float k[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int w = c >> 2, sh = 8 * (c & 3);
            const F2 px = F2{(float)((wx[w] >> sh) & 0xFFu), (float)((wx[2 + w] >> sh) & 0xFFu)};
            const F2 py = F2{(float)((wy[w] >> sh) & 0xFFu), (float)((wy[2 + w] >> sh) & 0xFFu)};
            const F2 pz = F2{(float)((wz[w] >> sh) & 0xFFu), (float)((wz[2 + w] >> sh) & 0xFFu)};
            const F2 a = pk_fma(px, F2{ax, ax}, F2{bx, bx}), b = pk_fma(py, F2{ay, ay}, F2{by, by}),
                     e = pk_fma(pz, F2{az, az}, F2{bz, bz});
            const float tn = imax(vmax3(vmin(a.x, a.y), vmin(b.x, b.y), vmin(e.x, e.y)), s.tmin);
            const float tf = imin(vmin3(vmax(a.x, a.y), vmax(b.x, b.y), vmax(e.x, e.y)), best_t);
            k[c] = (tn <= tf && ch[c] != RT_EMPTY_CHILD) ? tn : RT_INF;
        }
        return wide8_tail(k, ch, stk, sp);
    } else {             // rt_dnode4
        const float4 *N = src.ptr4(node);
        const float4 qx01 = N[0], qx23 = N[1], qy01 = N[2], qy23 = N[3], qz01 = N[4], qz23 = N[5], cf = N[6];
        uint32_t c0 = (uint32_t)fbits(cf.x), c1 = (uint32_t)fbits(cf.y), c2 = (uint32_t)fbits(cf.z),
                 c3 = (uint32_t)fbits(cf.w);
        float k0 = box_entry<true>(s, F2{qx01.x, qx01.y}, F2{qy01.x, qy01.y}, F2{qz01.x, qz01.y}, best_t, c0);
        float k1 = box_entry<true>(s, F2{qx01.z, qx01.w}, F2{qy01.z, qy01.w}, F2{qz01.z, qz01.w}, best_t, c1);
        float k2 = box_entry<true>(s, F2{qx23.x, qx23.y}, F2{qy23.x, qy23.y}, F2{qz23.x, qz23.y}, best_t, c2);
        float k3 = box_entry<true>(s, F2{qx23.z, qx23.w}, F2{qy23.z, qy23.w}, F2{qz23.z, qz23.w}, best_t, c3);
        cas(k0, c0, k1, c1);   // sorting network, nearest first
        cas(k2, c2, k3, c3);
        cas(k0, c0, k2, c2);
        cas(k1, c1, k3, c3);
        cas(k1, c1, k2, c2);
        stk_at(stk, sp) = c3;
        sp += k3 != RT_INF ? RT_SP_UNIT : 0;
        stk_at(stk, sp) = c2;
        sp += k2 != RT_INF ? RT_SP_UNIT : 0;
        stk_at(stk, sp) = c1;
        sp += k1 != RT_INF ? RT_SP_UNIT : 0;
        return k0 != RT_INF ? c0 : RT_EMPTY_CHILD;
    }
}

// One traversal round's descent (both engines).  A lane that reaches a leaf
// postpones it (pleaf) and keeps descending speculatively until the lanes hold a
// leaf or have nothing left (Aila & Laine 2009), so node steps and leaf tests both
// run with most lanes busy; culling against a not-yet-updated best_t is merely
// conservative.  One branch per step (the node fetch): parking a leaf and popping
// the stack are selects, the pop's LDS read unconditional (the exec-mask
// bookkeeping of two more branches per step cost more: 76.2 -> 74.9 ms on c4).
// The descent ends once at most RT_DESCEND_TAIL lanes still look for their first
// leaf: those few carry their node and stack into the next round instead of
// holding the other lanes in node steps at a few percent lane occupancy
// (tail 0 / 2 / 4 / 6 / 8 / 12 on c4: 71.45 / 66.92 / 65.41 / 64.96 / 65.04 /
// 66.14 ms).  The closest hit is independent of the order its leaves are tested
// in (list-order tie-break), so the images are unchanged.
// kSteps = 2 takes two node steps between exit checks (one ballot, popcount and
// loop branch per two steps; the extra step is speculative for lanes already
// done): c4 65.08 -> 64.32 ms with the cut-off at 8 (2 steps and tail 6 / 10 / 12:
// 64.52 / 64.05 / 64.29; 3 steps 64.99), c3 -1.0 %, but c2 (instance chains,
// longer node steps) +0.8 %, so the instance variant keeps single steps.
#ifndef RT_DESCEND_TAIL
#define RT_DESCEND_TAIL 6
#endif
#ifndef RT_DESCEND_TAIL2
#define RT_DESCEND_TAIL2 8
#endif
#ifndef RT_DESCEND_TAIL_DRY
#define RT_DESCEND_TAIL_DRY 0
#endif
// dry = true (a wave draining the launch's last paths, few lanes live): no tail cut —
// the cut trades a few lanes' node steps for the others', and with a handful of lanes
// every round's fixed cost (slab set-up, leaf pass, exit checks) is on the path's
// latency, which is what the launch's end waits for.
template <int kWidth, bool kCount, int kSteps = 1, class Nodes>
__device__ __forceinline__ uint32_t descend(const Nodes &nodes, uint32_t &node, const Slab &sl, float best_t,
                                            uint32_t *stk, int &sp, Counters &cnt, bool dry = false) {
    const int kTail = dry ? RT_DESCEND_TAIL_DRY : (kSteps == 1 ? RT_DESCEND_TAIL : RT_DESCEND_TAIL2);
    uint32_t pleaf = RT_EMPTY_CHILD;
    for (;;) {
#pragma unroll
        for (int u = 0; u < kSteps; ++u) {
            if (!(node & RT_LEAF_BIT)) {
                if (kCount) { cnt.nodes++; if (first_active()) cnt.w_nodes++; }
                node = node_step<kWidth>(nodes, node, sl, best_t, stk, sp);
            }
            const bool leaf = node != RT_EMPTY_CHILD && (node & RT_LEAF_BIT);
            const bool park = leaf && pleaf == RT_EMPTY_CHILD;
            pleaf = park ? node : pleaf;
            node = park ? RT_EMPTY_CHILD : node;
            const bool pop = node == RT_EMPTY_CHILD && sp > 0;
            sp -= pop ? RT_SP_UNIT : 0;
            // sp >= 0: pops only from a non-empty stack (LDS nodes: 16-bit entries)
            const uint32_t top = std::is_same<Nodes, GlobalNodes>::value ? stk_at(stk, sp) : stk16_get(stk, sp);
            node = pop ? top : node;
        }
        if (__popcll(wballot(pleaf == RT_EMPTY_CHILD && node != RT_EMPTY_CHILD)) <= kTail) {
            return pleaf;
        }
    }
}

// --------------------------------------------------------------- scatter
// Candidates of the two rejection loops: `base` is the stream counter before the
// candidate's first draw.
struct SphereCand {   // material.h:41-47 random_in_unit_sphere
    __device__ __forceinline__ bool operator()(uint64_t base, V3 &p) const {
        const uint64_t x1 = lcg_step(base), x2 = lcg_step(x1), x3 = lcg_step(x2);
        p = sub(scale(2.0f, mk((float)u48x(x1), (float)u48x(x2), (float)u48x(x3))), mk(1, 1, 1));
        return (double)dot(p, p) < 1.0;
    }
};
struct DiskCand {     // camera.h:6-12 random_in_unit_disk
    __device__ __forceinline__ bool operator()(uint64_t base, V3 &p) const {
        const uint64_t x1 = lcg_step(base), x2 = lcg_step(x1);
        p = sub(scale(2.0f, mk((float)u48x(x1), (float)u48x(x2), 0)), mk(1, 1, 0));
        return (double)dot(p, p) < 1.0;
    }
};
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(2 * dot(v, n), n)); }   // material.h:36-38

// ------------------------------------------------------------ work claim
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Work items a wave claims per atomic: RtKernelArgs.claim (host: up to 512, fewer
// for small jobs so that every wave gets work).

// ------------------------------------------- cooperative rejection sampling
// The rejection loops of the reference (camera.h:6-12 random_in_unit_disk,
// material.h:41-47 random_in_unit_sphere) accept the first candidate inside the
// unit ball; candidate c of a loop entered after draw n uses draws n+K*c+1 ..
// n+K*c+K.  Counter streams are random access, so the wave evaluates the
// candidates of all lanes that need a point at once: the m requesting lanes
// publish (stream position) in LDS slots 0..m-1 and all 64 lanes take candidates
// round-robin (lane L evaluates candidate c0 + L/m of slot L%m).  Each owner keeps
// its lowest accepted candidate, so the point and the draws consumed are exactly
// those of its own sequential loop; rounds repeat for owners whose candidates all
// failed.  A lane loop that ran ~6 wave trips at ~16% SIMD efficiency (the
// slowest lane of 48 decides) takes ~2-3 fully used trips.
// Must be called with all 64 lanes of the wave active.
struct CoopSlot {
    uint64_t ctr;
    uint64_t pad;
};

// Per requester count m (1..64): the lanes congruent to 0 mod m, and ceil(2^16 / m)
// (lane / m == (lane * inv) >> 16 exactly for lane < 64).  A wave-uniform index, so
// a scalar load replaces a scalar loop and an integer division per round.
struct CoopTable {
    uint64_t stride_mask[65];
    uint32_t inv[65];
    constexpr CoopTable() : stride_mask(), inv() {
        for (int m = 1; m <= 64; ++m) {
            uint64_t p = 0;
            for (int b = 0; b < 64; b += m) p |= 1ull << b;
            stride_mask[m] = p;
            inv[m] = (0xFFFFu + (uint32_t)m) / (uint32_t)m;
        }
    }
};
__constant__ const CoopTable kCoop = CoopTable();

// One candidate per lane and round (two per lane measured slower: the extra
// candidate costs every lane more than the saved rounds).  Candidate position
// c = lane belongs to slot c mod m as that owner's candidate c / m.
template <int K, bool kCount, class Cand>
__device__ __forceinline__ V3 coop_reject(bool want, Rng &g, CoopSlot *slots, const LdsJump *jt, uint32_t lane,
                                          Counters &cnt, Cand cand) {
    // read by the requesting lanes only, and each of them wins a point
    V3 res = (RT_SHADE_LEAN & 16) ? unset_v3() : mk(0, 0, 0);
    bool pending = want;
    uint64_t U = wballot(pending);
    while (U != 0ull) {
        const uint32_t m = (uint32_t)__popcll(U);            // wave-uniform
        const uint32_t inv = kCoop.inv[m];
        const uint64_t P = kCoop.stride_mask[m];               // lanes congruent to 0 mod m
        const uint32_t r = lanes_below(U);
        if (pending) slots[r].ctr = g.x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t t = (lane * inv) >> 16;                 // lane / m
        const uint32_t slot = lane - t * m;
        const uint64_t base = lcg_jump(slots[slot].ctr, jt[K * t]);   // the owner's state before candidate t
        V3 p;
        const uint64_t okm = wballot(cand(base, p));
        if (kCount && first_active()) cnt.w_rius++;
        uint32_t src = lane;
        bool won = false;
        if (pending) {
            const uint64_t win = okm & (P << r);
            won = win != 0ull;
            src = won ? (uint32_t)__builtin_ctzll(win) : lane;
            // candidates consumed: up to the winner, or all of the owner's this round
            const uint32_t tried = ((won ? src : 63u - r) * inv >> 16) + 1u;
            g.x = lcg_jump(g.x, jt[K * tried]);
            if (kCount) cnt.l_rius += tried;
            pending = !won;
        }
        // every lane takes part in the exchange (bpermute reads the source lane's register)
        const float px = __shfl(p.x, (int)src), py = __shfl(p.y, (int)src), pz = __shfl(p.z, (int)src);
        if (won) res = mk(px, py, pz);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        U = wballot(pending);
    }
    return res;
}

// coop_reject for a wave whose requesting lanes need different samplers: lanes
// with `disk` true want random_in_unit_disk (2 draws per candidate, camera.h:6-12),
// the others random_in_unit_sphere (3 draws, material.h:41-47).  The owner
// publishes its draw count per candidate beside its stream position, every lane
// evaluates three draws and tests the candidate the way its owner's loop would (a
// disk candidate's third draw is never used, and its z is 0 as in the reference),
// and each owner advances its stream by its own count: the points and draws are
// exactly those of coop_reject<2> / coop_reject<3>.  Lets the megakernel run the
// lens-disk candidates of new camera samples in the shading stage's rounds.
template <bool kCount>
__device__ __forceinline__ V3 coop_reject_mixed(bool want, bool disk, Rng &g, CoopSlot *slots, const LdsJump *jt,
                                                uint32_t lane, Counters &cnt) {
    V3 res = (RT_SHADE_LEAN & 16) ? unset_v3() : mk(0, 0, 0);   // read by the requesting lanes only
    bool pending = want;
    const uint32_t K = disk ? 2u : 3u;
    uint64_t U = wballot(pending);
    while (U != 0ull) {
        const uint32_t m = (uint32_t)__popcll(U);            // wave-uniform
        const uint32_t inv = kCoop.inv[m];
        const uint64_t P = kCoop.stride_mask[m];               // lanes congruent to 0 mod m
        const uint32_t r = lanes_below(U);
        if (pending) { slots[r].ctr = g.x; slots[r].pad = K; }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t t = (lane * inv) >> 16;                 // lane / m
        const uint32_t slot = lane - t * m;
        const uint32_t kk = (uint32_t)slots[slot].pad;
        const uint64_t x1 = lcg_step(lcg_jump(slots[slot].ctr, jt[kk * t])), x2 = lcg_step(x1), x3 = lcg_step(x2);
        const float pz = kk == 3u ? 2.0f * (float)u48x(x3) - 1.0f : 0.0f;
        const V3 p = mk(2.0f * (float)u48x(x1) - 1.0f, 2.0f * (float)u48x(x2) - 1.0f, pz);
        const uint64_t okm = wballot((double)dot(p, p) < 1.0);
        if (kCount && first_active()) cnt.w_rius++;
        uint32_t src = lane;
        bool won = false;
        if (pending) {
            const uint64_t win = okm & (P << r);
            won = win != 0ull;
            src = won ? (uint32_t)__builtin_ctzll(win) : lane;
            const uint32_t tried = ((won ? src : 63u - r) * inv >> 16) + 1u;
            g.x = lcg_jump(g.x, jt[K * tried]);
            if (kCount) cnt.l_rius += tried;
            pending = !won;
        }
        const float qx = __shfl(p.x, (int)src), qy = __shfl(p.y, (int)src), qz = __shfl(p.z, (int)src);
        if (won) res = mk(qx, qy, qz);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        U = wballot(pending);
    }
    return res;
}

// Cooperative turbulence (perlin.h:64-74).  Octave k of turb(q) is
// noise(q * 2^k) weighted 2^-k: `temp_p *= 2` and `weight *= 0.5` are exact, so
// the octaves are independent.  The lanes that need turb publish q in LDS and the
// wave evaluates the 7 octaves of up to 9 of them at once, one noise() per lane;
// each owner gathers its 7 values and sums them in octave order, exactly as the
// reference's loop does.  A wave with one noisy lane used to run all 7 octaves as
// a chain of 28 dependent gathers; now it runs one noise() per round.
// Must be called with all 64 lanes of the wave active.
template <class RV, class PM>
__device__ __forceinline__ float coop_turb(bool want, V3 q, RV ranvec, PM perm, CoopSlot *slots,
                                           uint32_t lane) {
    const uint64_t U = wballot(want);
    if (U == 0ull) return 0.f;
    float res = 0.f;
    const uint32_t m = (uint32_t)__popcll(U);
    const uint32_t r = lanes_below(U);
    float4 *pts = reinterpret_cast<float4 *>(slots);
    if (want) pts[r] = make_float4(q.x, q.y, q.z, 0.f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t lo = lane / 7, oct = lane - lo * 7;
    for (uint32_t base = 0; base < m; base += 9) {
        const uint32_t o = base + lo;
        float val = 0.f;
        if (lane < 63 && o < m) {
            const float4 pt = pts[o];
            const float s = (float)(1u << oct);
            val = perlin_noise(ranvec, perm, mk(pt.x * s, pt.y * s, pt.z * s));
        }
        const bool mine = want && r >= base && r < base + 9;
        const uint32_t src0 = ((r - base) * 7u) & 63u;
        float acc = 0.f, weight = 1.0f;
#pragma unroll
        for (int kk = 0; kk < 7; ++kk) {
            const float nk = __shfl(val, (int)((src0 + kk) & 63u));
            acc += weight * nk;
            weight = (float)((double)weight * 0.5);
        }
        if (mine) res = fabsf(acc);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return res;
}

// ----------------------------------------------------------------- camera
// camera.h:41-56's state, kept in LDS and read (volatile: once per use, not hoisted)
// by the camera stage: held in SGPRs across the persistent loop, its 24 floats
// pushed the kernel past the SGPR limit and came back as per-iteration v_readlanes.
typedef float CamV4 __attribute__((ext_vector_type(4)));
struct CamView { V3 llc, hor, ver, org, cu, cv; float t0, t1, lens; };
// Written float by float: whole-vector initialisers from the kernel-argument arrays
// made the compiler assemble them in scratch memory.
__device__ __forceinline__ void store_camera(const RtKernelArgs &A, CamV4 *lds) {
    float *f = reinterpret_cast<float *>(lds);
    const float v[24] = {A.llc[0], A.llc[1], A.llc[2], A.ct0,  A.hor[0], A.hor[1], A.hor[2], A.ct1,
                         A.ver[0], A.ver[1], A.ver[2], A.lens, A.org[0], A.org[1], A.org[2], 0.f,
                         A.cu[0],  A.cu[1],  A.cu[2],  0.f,    A.cv[0],  A.cv[1],  A.cv[2],  0.f};
#pragma unroll
    for (int k = 0; k < 24; ++k) f[k] = v[k];
}
typedef __attribute__((address_space(3))) const volatile CamV4 LdsCamV4;   // keeps ds_read (not flat)
__device__ __forceinline__ CamView load_camera(const CamV4 *lds) {
    const LdsCamV4 *v = (const LdsCamV4 *)lds;
    const CamV4 a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], f = v[5];
    CamView C;
    C.llc = mk(a.x, a.y, a.z); C.t0 = a.w;
    C.hor = mk(b.x, b.y, b.z); C.t1 = b.w;
    C.ver = mk(c.x, c.y, c.z); C.lens = c.w;
    C.org = mk(d.x, d.y, d.z);
    C.cu = mk(e.x, e.y, e.z);
    C.cv = mk(f.x, f.y, f.z);
    return C;
}

// ------------------------------------------------------- lockstep primitives
// hitable_list's acceptance (hitable_list.h:20-32: `t < closest`, ties to the earlier
// list entry, the key) as selects: bitwise operators, so no short-circuit branches and
// no exec-mask juggling around three moves per tested primitive.
__device__ __forceinline__ void keep_closest(bool in, float t, int key, uint32_t idx, float &best_t, int &best_key,
                                             uint32_t &best_prim) {
    const bool take = in & ((t < best_t) | ((t == best_t) & (key < best_key)));
    best_t = take ? t : best_t;
    best_key = take ? key : best_key;
    best_prim = take ? idx : best_prim;
}

// Tests primitives [first, first + count) (4 float4 each, read through the scalar
// cache: P is a constant-address-space pointer and q is uniform, so the records land
// in SGPRs) against every lane's ray in lockstep: the primitive, its kind and its
// instance are the same in all lanes (scalar loads and branches), so only
// the kind's own test runs and no lane idles behind another's traversal.  Lanes
// with `in` false compute but keep nothing.  kPerPrimInst: each primitive's own
// instance chain; otherwise the caller transformed `r`.  Used by the BVH modes'
// pre-scan; the flat scan, whose groups are ordered by kind, runs scan_group below.
typedef __attribute__((address_space(4))) const F4v ConstF4;   // uniform index: scalar (SMEM) loads
template <bool kCount, bool kInst, bool kPerPrimInst, class PT>
__device__ __forceinline__ void lockstep_prims(PT P, int first, int count, const float4 *insts,
                                               const Ray &r, float tmin, bool in, int group_inst, float &best_t,
                                               int &best_key, uint32_t &best_prim, Counters &cnt) {
    for (int q = first; q < first + count; ++q) {
        const F4v g0v = P[4 * q], mmv = P[4 * q + 1];
        const float4 g0 = f4(g0v);
        const int kind = __builtin_amdgcn_readfirstlane(fbits(mmv.x)) & 0xff;
        const int inst = kPerPrimInst ? __builtin_amdgcn_readfirstlane(fbits(mmv.z)) : group_inst;
        Ray ro = r;
        if (kInst && kPerPrimInst && inst >= 0) ro = to_object_uniform(insts, inst, r);
        float t;
        if (kind == RT_PRIM_SPHERE) {
            t = sphere_t(mk(g0.x, g0.y, g0.z), g0.w, ro, tmin);
        } else if (kind == RT_PRIM_MOVING_SPHERE) {
            t = sphere_t(msphere_center(g0, f4(P[4 * q + 2]), f4(P[4 * q + 3]), ro.time), g0.w, ro, tmin);
        } else {
            t = rect_t(kind, g0, mmv.y, ro, tmin);
        }
        const int order = fbits(mmv.w);
        const int key = kind <= RT_PRIM_MOVING_SPHERE ? order : -1 - order;
        if (kCount && in) cnt.prim(kind | (kInst && inst >= 0 ? 0x100 : 0));
        if (kCount && first_active()) cnt.w_prims++;
        keep_closest(in, t, key, (uint32_t)q, best_t, best_key, best_prim);
    }
}

// The flat scan's primitives of one group (rt_dgroup), one run per kind: no kind
// branches or kind selects per primitive (c2: 49.6 -> 45.8 ms).  A rect run's
// quotients (k - o_a) / d_a (aarect.h:51) share the lane's divisor, but a div_rn by
// a per-run reciprocal (one IEEE division + the wave's range check per run) measured
// slower than the IEEE division per rect (45.2 vs 45.8 ms): runs hold 1-3 rects.
// The scan's closest hit: t and key << 8 | primitive (keys are unique and |key| <=
// RT_SCAN_MAX, primitives < 256), so one compare and one select carry both.
struct ScanBest { float t; int kp; };
static_assert(RT_SCAN_MAX < 256, "ScanBest packs the primitive index in 8 bits");
template <bool kCount>
__device__ __forceinline__ void scan_keep(float t, int key, int q, bool in, int ck, ScanBest &b, Counters &cnt) {
    if (kCount && in) cnt.prim(ck);
    if (kCount && first_active()) cnt.w_prims++;
    const int kp = key * 256 + q;   // wave-uniform
    const bool take = in & ((t < b.t) | ((t == b.t) & (kp < b.kp)));
    b.t = take ? t : b.t;
    b.kp = take ? kp : b.kp;
}
// plane_t without branches: the in-plane coordinates are computed for every t (an
// out-of-range t is replaced by RT_INF either way), so one select decides the hit
template <bool kCount>
__device__ __forceinline__ int scan_rects(const ConstF4 *P, int q, int n, float oa, float da, float oi, float di,
                                          float oj, float dj, float tmin, bool in, int ck, ScanBest &b, Counters &cnt) {
    const int e = q + n;
    auto test = [&](F4v g0, F4v mm, int i) {
        const float t = (mm.y - oa) / da;
        const float a = oi + t * di, c = oj + t * dj;
        const bool miss = (t < tmin) | (t > RT_FLT_MAX) | (a < g0.x) | (a > g0.y) | (c < g0.z) | (c > g0.w);
        scan_keep<kCount>(miss ? RT_INF : t, -1 - fbits(mm.w), i, in, ck, b, cnt);
    };
    const ConstF4 *p = P + 4 * q;   // a running record pointer: no per-primitive address arithmetic
    // two records per scalar-load wait (scalar loads return out of order, so
    // every use waits for all of them: a pair halves the waits)
    for (; q + 1 < e; q += 2, p += 8) {
        const F4v g0a = p[0], mma = p[1], g0b = p[4], mmb = p[5];
        test(g0a, mma, q);
        test(g0b, mmb, q + 1);
    }
    if (q < e) test(p[0], p[1], q);
    return e;
}
// ro: the lanes' rays in the group's object space; kinds / nyz: rt_dgroup's counts
template <bool kCount, bool kInst>
__device__ __forceinline__ void scan_group(const ConstF4 *P, int q, int kinds, int nyz, int inst, const Ray &ro,
                                           float tmin, bool in, ScanBest &b, Counters &cnt) {
    const int ik = kInst && inst >= 0 ? 0x100 : 0;
    for (const int e = q + (kinds & 0xff); q < e; ++q) {
        const F4v g0 = P[4 * q], mm = P[4 * q + 1];
        const float t = sphere_t(mk(g0.x, g0.y, g0.z), g0.w, ro, tmin);
        scan_keep<kCount>(t, fbits(mm.w), q, in, RT_PRIM_SPHERE | ik, b, cnt);
    }
    for (const int e = q + ((kinds >> 8) & 0xff); q < e; ++q) {
        const F4v g0v = P[4 * q], mm = P[4 * q + 1];
        const float4 g0 = f4(g0v);
        const float t = sphere_t(msphere_center(g0, f4(P[4 * q + 2]), f4(P[4 * q + 3]), ro.time), g0.w, ro, tmin);
        scan_keep<kCount>(t, fbits(mm.w), q, in, RT_PRIM_MOVING_SPHERE | ik, b, cnt);
    }
    q = scan_rects<kCount>(P, q, (kinds >> 16) & 0xff, ro.o.z, ro.d.z, ro.o.x, ro.d.x, ro.o.y, ro.d.y, tmin, in,
                           RT_PRIM_XY_RECT | ik, b, cnt);
    q = scan_rects<kCount>(P, q, (kinds >> 24) & 0xff, ro.o.y, ro.d.y, ro.o.x, ro.d.x, ro.o.z, ro.d.z, tmin, in,
                           RT_PRIM_XZ_RECT | ik, b, cnt);
    scan_rects<kCount>(P, q, nyz, ro.o.x, ro.d.x, ro.o.y, ro.d.y, ro.o.z, ro.d.z, tmin, in, RT_PRIM_YZ_RECT | ik,
                       b, cnt);
}

// ------------------------------------------------------------------ media
// Constants the media stage reads from LDS (rt_megakernel fills them at launch): a
// volatile read at each use, so the compiler neither hoists them into registers held
// across the persistent loop (where they were spilled to scratch) nor folds them back.
typedef LogConsts MediaConsts;   // log_f64's coefficients
// The media stage reads them as one record copy at the use (five volatile reads measure
// alike; only 0.2 from LDS, the round-4 way, spilled with the glibc sine inlined, c4 +1.4 %:
// profiles/r05/ab_log_consts_ocml_r04.log).
typedef __attribute__((address_space(3))) const volatile MediaConsts LdsMediaConsts;
// constant_medium::hit for every medium after the surface search
// (constant_medium.h:26-50): the boundary's entry/exit, clipped to [t_min, best]
// (best = the surface hit, if any), and the free-flight distance from the
// medium stream.  Returns the material of the medium that scatters (best_t and
// `have` updated) or -1.
// A medium's record and its first boundary primitive's 32-B head, preloaded into
// LDS once per workgroup (load_media): every lane reads the same address, so the
// media loop costs no dependent global round trips.
struct MediumRec {
    int4 md;      // first boundary prim, count, -(1/density) bits, material
    float4 g0;    // first boundary prim: geometry
    float4 mm;    // first boundary prim: kind | flags, -, instance, order
};
#ifndef RT_LDS_MEDIA
#define RT_LDS_MEDIA 8
#endif
template <int kBlock>
__device__ __forceinline__ void load_media(const RtKernelArgs &A, MediumRec *lds) {
    const int n = min(A.nmedia, RT_LDS_MEDIA);
    for (int i = threadIdx.x; i < n; i += kBlock) {   // field by field: a whole-struct copy went through scratch
        const int4 md = A.media[i];
        lds[i].md = md;
        lds[i].g0 = A.bprims[md.x * 4 + 0];
        lds[i].mm = A.bprims[md.x * 4 + 1];
    }
}

// One medium's test (constant_medium.h:26-50) against the surface result.
template <bool kCount, bool kInst = true>
__device__ __forceinline__ void medium_one(const RtKernelArgs &A, const MediumRec &M, int k, const Ray &r, const Recip &rd,
                                           const Recip &ra, uint64_t xk, bool &have, float &best_t,
                                           int &med_mat, LdsMediaConsts *mc, Counters &cnt) {
    const float dlen = rd.a;
    if (kCount) cnt.media++;
    const int4 md = M.md;
    float r1, r2;
    bool ok;
    const float4 bm = M.mm;
    if (md.y == 1 && (fbits(bm.x) & 0xff) == RT_PRIM_SPHERE && fbits(bm.z) < 0) {   // wave-uniform
        // one sphere: both boundary calls (constant_medium.h:28-29) share the roots
        if (kCount) cnt.spheres++;
        const float4 sg = M.g0;
        V3 oc = sub(r.o, mk(sg.x, sg.y, sg.z));
        const float a = ra.a;
        float b = dot(oc, r.d);
        float cc = dot(oc, oc) - sg.w * sg.w;
        float disc = b * b - a * cc;
        const bool valid = disc > 0;
        if (wballot(valid) == 0ull) return;   // the whole wave misses the boundary
        const float sq = sqrtf(disc);
        const float ta = div_by(-b - sq, ra);
        const float tb = div_by(-b + sq, ra);
        // selects, not branches: sphere.h:33-44 for t_min = -FLT_MAX, then t_min = r1 + 0.0001
        const bool fa = ta < RT_FLT_MAX && ta > -RT_FLT_MAX, fb = tb < RT_FLT_MAX && tb > -RT_FLT_MAX;
        r1 = fa ? ta : tb;
        const float tmin2 = (float)((double)r1 + 0.0001);
        const bool ga = ta < RT_FLT_MAX && ta > tmin2, gb = tb < RT_FLT_MAX && tb > tmin2;
        r2 = ga ? ta : tb;
        ok = valid && (fa || fb) && (ga || gb);
    } else {
        r1 = boundary_t<kCount, kInst>(A.bprims, A.insts, md.x, md.y, r, -RT_FLT_MAX, cnt);
        ok = r1 != RT_INF;
        if (wballot(ok) == 0ull) return;
        r2 = boundary_t<kCount, kInst>(A.bprims, A.insts, md.x, md.y, r, (float)((double)r1 + 0.0001), cnt);
        ok = ok && r2 != RT_INF;
    }
    const float tmax = have ? best_t : RT_FLT_MAX;
    r1 = r1 < A.tmin ? A.tmin : r1;
    r2 = r2 > tmax ? tmax : r2;
    ok = ok && !(r1 >= r2);
    if (wballot(ok) == 0ull) return;   // no lane inside the medium: no free-flight draw
    r1 = r1 < 0 ? 0.f : r1;
    const float distance_inside_boundary = (r2 - r1) * dlen;
    const float neg_inv_density = __int_as_float(md.z);   // -(1/density), host-side
#if !defined(__HIP_DEVICE_COMPILE__)   // (the host pass never runs device code)
    const LogConsts lc{mc->c07, mc->c06, mc->c02, mc->c025, mc->c03};
#else                                   // one copy of the record through an opaque LDS address: read at the use
    uint32_t mca = (uint32_t)(size_t)mc;
    asm volatile("" : "+v"(mca));
    const LogConsts lc = *(__attribute__((address_space(3))) const LogConsts *)(size_t)mca;
#endif
    // (An exp pre-test that skipped the double log for a wave of sure misses — u below
    // 2^(-density D log2 e) (1 - 2^-12) — measured slower, round 6: in every wave c4 48.95 ->
    // 49.45 ms, the share of 8 25.32 -> 25.63 (a wave seldom holds only sure misses of both
    // media); in the ball waves only, where final()'s fog after the dense medium's scatter
    // almost never scatters, 48.88 -> 49.17 and 25.19 -> 25.45: profiles/r06/pretest*_ab.log.)
    const float hit_distance = (float)((double)neg_inv_density * log_f64(u48x(xk), lc));
    const bool hit = ok && hit_distance < distance_inside_boundary;
    const float tm = r1 + div_by(hit_distance, rd);
    best_t = hit ? tm : best_t;
    have = have || hit;
    med_mat = hit ? md.w : med_mat;
}

// All media in list order.  The first RT_LDS_MEDIA come from the workgroup's LDS
// copy through an explicit LDS pointer, the rest from HBM, in two loops: one loop
// choosing per medium between the two made the compiler select the address and
// issue generic (flat) loads, which wait on both memory counters.
template <bool kCount, bool kInst = true>
__device__ __forceinline__ int media_hit(const RtKernelArgs &A, const MediumRec *lds_media, LdsMediaConsts *mc, const Ray &r,
                                         const Recip &rd, Rng &g, bool &have, float &best_t, Counters &cnt) {
    // a = |d|^2 of the boundary spheres' quadratics (sphere.h:28), its reciprocal once for all media
    const Recip ra = recip_of(dot(r.d, r.d), true);
    typedef unsigned U4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const U4v LdsU4;
    int med_mat = -1;
    const int nl = min(A.nmedia, RT_LDS_MEDIA);
    for (int k = 0; k < nl; ++k) {
        const LdsU4 *p = (const LdsU4 *)lds_media + 3 * k;
        const U4v x = p[0], y = p[1], z = p[2];
        MediumRec M;
        M.md = make_int4((int)x.x, (int)x.y, (int)x.z, (int)x.w);
        M.g0 = make_float4(__uint_as_float(y.x), __uint_as_float(y.y), __uint_as_float(y.z), __uint_as_float(y.w));
        M.mm = make_float4(__uint_as_float(z.x), __uint_as_float(z.y), __uint_as_float(z.z), __uint_as_float(z.w));
        g.xm = lcg_step(g.xm);   // this medium's draw, taken or not
        medium_one<kCount, kInst>(A, M, k, r, rd, ra, g.xm, have, best_t, med_mat, mc, cnt);
    }
    for (int k = RT_LDS_MEDIA; k < A.nmedia; ++k) {
        MediumRec M;
        M.md = A.media[k];
        M.g0 = A.bprims[M.md.x * 4 + 0];
        M.mm = A.bprims[M.md.x * 4 + 1];
        g.xm = lcg_step(g.xm);
        medium_one<kCount, kInst>(A, M, k, r, rd, ra, g.xm, have, best_t, med_mat, mc, cnt);
    }
    return med_mat;
}

// ------------------------------------------------------------------ shade
struct ShadeOut {
    bool scattered;
    V3 att, emitted;
    Ray ray;
};

// shade() in three parts, so that the megakernel can run other lanes' rejection
// candidates in the same cooperative rounds (shade_begin -> coop -> shade_finish).
struct ShadeState {
    int kind;           // material kind (-1: no shading)
    bool live;          // depth < max_depth (main.cpp:34)
    bool wants_sphere;  // needs random_in_unit_sphere
    V3 tv;              // texture value (lambertian / isotropic / light)
};

// Material, depth test, texture value incl. cooperative turbulence (textures
// texture.h / perlin.h).  Must be called with all 64 lanes of the wave active.
template <bool kCount, bool kUV = true, bool kChecker = true, class RV = const float4 *, class PM = const int *>
__device__ __forceinline__ ShadeState shade_begin(const RtKernelArgs &A, bool ready, bool have, const Hit &hr, int depth,
                                                  CoopSlot *slots, uint32_t lane, Counters &cnt, RV ranvec, PM perm) {
    const bool shading = ready && have;
    ShadeState st;
    st.kind = -1;
    st.live = false;
    st.tv = (RT_SHADE_LEAN & 4) ? unset_v3() : mk(0, 0, 0);   // read for the textured and noisy lanes only
    bool noisy = false;
    float nscale = (RT_SHADE_LEAN & 32) ? unset_f() : 0.f;     // read for the noisy lanes only
    if (shading) {
        if (kCount) cnt.shades++;
        const float4 m0 = A.mats[hr.mat * 2 + 0], m1 = A.mats[hr.mat * 2 + 1];
        st.kind = fbits(m0.x);
        st.live = depth < A.max_depth;
        const bool textured = st.kind == RT_MAT_DIFFUSE_LIGHT ||
                              (st.live && (st.kind == RT_MAT_LAMBERTIAN || st.kind == RT_MAT_ISOTROPIC));
        if (textured && (fbits(m1.w) & 2)) {   // a constant texture, resolved by the host (capi.cpp)
            st.tv = mk(m1.x, m1.y, m1.z);
        } else if (textured) {
            float4 t0, t1;
            const int tkind = tex_leaf<kChecker>(A, fbits(m0.y), hr.p, t0, t1);   // texture.h:35-44
            noisy = tkind == RT_TEX_NOISE;
            nscale = t0.w;
            if (!noisy) st.tv = tex_value_leaf<kUV>(A, tkind, t0, t1, hr.u, hr.v);
        }
    }
    if (kCount && noisy) cnt.noise++;
    const float turb = coop_turb(noisy, scale(nscale, hr.p), ranvec, perm, slots, lane);   // perlin.h:64-74
    if (noisy) {                                                                               // texture.h:52-56
        const float sv = 1 + rt_sinf(nscale * hr.p.x + 5 * turb);
        const float h = 0.5f * 1;
        st.tv = mk(sv * h, sv * h, sv * h);
    }
    st.wants_sphere = shading && st.live && (st.kind == RT_MAT_LAMBERTIAN || st.kind == RT_MAT_METAL ||
                                             st.kind == RT_MAT_ISOTROPIC);
    return st;
}

// The path ends at this segment whatever the scatter draws: a miss, a light, or
// the depth limit (only metal can still end after its rius, material.h:81).
__device__ __forceinline__ bool shade_ends(bool ready, bool have, const ShadeState &st) {
    return ready && (!have || !st.live || st.kind == RT_MAT_DIFFUSE_LIGHT);
}

// emitted() of the segment: the background on a miss (TNW/Chapter03:29-31 for the
// sky), the light's texture, else black.
__device__ __forceinline__ V3 shade_emitted(const RtKernelArgs &A, bool have, const Ray &r, const Recip &rd,
                                            const ShadeState &st) {
    if (!have) {
        if (A.background != RT_BG_SKY) return mk(0, 0, 0);
        const V3 ud = mk(div_by(r.d.x, rd), div_by(r.d.y, rd), div_by(r.d.z, rd));   // unit(r.d), vec3.h:146
        const float t = (float)(0.5 * ((double)ud.y + 1.0));
        return add(scale((float)(1.0 - (double)t), mk(1.0f, 1.0f, 1.0f)), scale(t, mk(0.5f, 0.7f, 1.0f)));
    }
    return st.kind == RT_MAT_DIFFUSE_LIGHT ? st.tv : mk(0, 0, 0);
}

// material::scatter (material.h) given the lane's random_in_unit_sphere point.
// dlen = |r.d|, computed once per segment and shared with the media (RtKernelArgs.need_dlen).
__device__ __forceinline__ ShadeOut shade_finish(const RtKernelArgs &A, bool ready, bool have, const Ray &r, const Recip &rd,
                                                 const Hit &hr, const ShadeState &st, V3 rius, Rng &g) {
    ShadeOut o;
    o.scattered = false;
    // (lean: o.emitted is set below for every ready lane, the only callers; o.att and o.ray
    // by the scattering branches)
    if (RT_SHADE_LEAN & 1) {
        o.emitted = unset_v3();
        o.att = unset_v3();
        o.ray.o = unset_v3(); o.ray.d = unset_v3(); o.ray.time = unset_f();
    } else {
        o.emitted = mk(0, 0, 0);
        o.att = mk(0, 0, 0);
        o.ray = r;
    }
    // RT_SHADE_LEAN: o.att and o.ray are set by the scattering branches only (the caller
    // reads them only when o.scattered): default copies of the ray, kept alive down every
    // early return, were ~30 register moves per wave iteration
    const int kind = st.kind;
    // unit(r.d) (vec3.h:146) once, for the lanes whose scatter needs it (metal,
    // dielectric) instead of once in each of their branches
    const bool wants_unit = ready && have && st.live && (kind == RT_MAT_METAL || kind == RT_MAT_DIELECTRIC);
    V3 ud = (RT_SHADE_LEAN & 64) ? unset_v3() : mk(0, 0, 0);   // read by the metal and dielectric lanes only
    if (wants_unit) ud = mk(div_by(r.d.x, rd), div_by(r.d.y, rd), div_by(r.d.z, rd));
    if (!ready) return o;
    o.emitted = shade_emitted(A, have, r, rd, st);
    if (!have || !st.live) return o;
    const float4 m0 = A.mats[hr.mat * 2 + 0];
    const float4 m1 = A.mats[hr.mat * 2 + 1];
    Ray ns = r;
    if (RT_SHADE_LEAN & 1) { ns.o = unset_v3(); ns.d = unset_v3(); ns.time = unset_f(); }
    if (kind == RT_MAT_LAMBERTIAN) {                              // material.h:64-69
        V3 target = add(add(hr.p, hr.n), rius);
        ns.o = hr.p; ns.d = sub(target, hr.p); ns.time = r.time;
        o.att = st.tv;
        o.scattered = true;
    } else if (kind == RT_MAT_METAL) {                            // material.h:77-82
        V3 reflected = reflect(ud, hr.n);
        ns.o = hr.p; ns.d = add(reflected, scale(m0.z, rius)); ns.time = 0.0f;
        o.att = mk(m1.x, m1.y, m1.z);
        o.scattered = dot(ns.d, hr.n) > 0;
    } else if (kind == RT_MAT_DIELECTRIC) {                       // material.h:90-120
        const float ref_idx = m0.w;
        V3 outward_normal;
        V3 reflected = reflect(r.d, hr.n);
        float ni_over_nt, cosine;
        o.att = mk(1.0f, 1.0f, 1.0f);
        float dn = dot(r.d, hr.n);
        if (dn > 0) {
            outward_normal = neg(hr.n);
            ni_over_nt = ref_idx;
            cosine = div_by(dot(r.d, hr.n), rd);
            cosine = sqrtf(1 - m1.z * (1 - cosine * cosine));   // m1.z = ref_idx * ref_idx
        } else {
            outward_normal = hr.n;
            ni_over_nt = m1.x;                                   // (float)(1.0 / (double)ref_idx)
            cosine = div_by(-dot(r.d, hr.n), rd);
        }
        // refract, material.h:23-33
        const V3 uv = ud;
        float dt = dot(uv, outward_normal);
        float disc = (float)(1.0 - (double)(ni_over_nt * ni_over_nt * (1 - dt * dt)));
        float reflect_prob;
        V3 refracted = mk(0, 0, 0);
        if (disc > 0) {
            refracted = sub(scale(ni_over_nt, sub(uv, scale(dt, outward_normal))), scale(sqrtf(disc), outward_normal));
            // schlick, material.h:16-20
            const float r0 = m1.y;   // ((1 - ref_idx) / (1 + ref_idx))^2, host-side
            reflect_prob = (float)(r0 + (double)(1 - r0) * pow5((double)(1 - cosine)));
        } else {
            reflect_prob = 1.0f;
        }
        ns.o = hr.p; ns.time = 0.0f;
        ns.d = (g.next() < (double)reflect_prob) ? reflected : refracted;
        o.scattered = true;
    } else if (kind == RT_MAT_ISOTROPIC) {                        // material.h:145-149
        ns.o = hr.p; ns.d = rius; ns.time = 0.0f;
        o.att = st.tv;
        o.scattered = true;
    }
    o.ray = ns;
    return o;
}

}  // namespace
