// tools/microbench/valu_rates.hip — issue cost of the integer / f64 VALU instructions the
// megakernel's RNG and media code use, on gfx950: 8 independent chains per wave, 8 waves
// per SIMD on every CU, cycles per wave-instruction per SIMD from the kernel time.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>

#define N_ITER 4096
// shader clock of the run: block 0's first wave stamps s_memtime (shader cycles) and
// s_memrealtime (100 MHz) at its start and end (MI355X_MICROARCH.md, in-kernel clock);
// the stores are plain vector stores of lane 0
__device__ unsigned long long g_stamps[4];
#define STAMP(k)                                                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                              \
        g_stamps[k] = __builtin_amdgcn_s_memtime();                                         \
        g_stamps[k + 1] = __builtin_amdgcn_s_memrealtime();                                 \
    }
#define BODY8(S) S(x0) S(x1) S(x2) S(x3) S(x4) S(x5) S(x6) S(x7)

#define K32(name, asmtxt)                                                                   \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t c) {                \
        STAMP(0)                                                                            \
        uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,      \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                     \
        for (int i = 0; i < N_ITER; ++i) {                                                  \
            _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                 \
                BODY8(STEP)                                                                 \
            }                                                                               \
        }                                                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;        \
        STAMP(2)                                                                            \
    }
// K32D: the instruction reads two more VGPRs, distinct (c and d): the VOP3 forms' issue cost
// without a source register read twice
#define K32D(name, asmtxt)                                                                  \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t c) {                \
        STAMP(0)                                                                            \
        uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,      \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                     \
        const uint32_t d = c ^ threadIdx.x;                                                 \
        for (int i = 0; i < N_ITER; ++i) {                                                  \
            _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                 \
                BODY8(STEPD)                                                                \
            }                                                                               \
        }                                                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;        \
        STAMP(2)                                                                            \
    }
#define STEPD(x) asm volatile(ASM : "+v"(x) : "v"(c), "v"(d));
#define ASM "v_fma_f32 %0, %0, %1, %2"
K32D(k_fma_f32_d, ASM)
#undef ASM
#define ASM "v_min3_f32 %0, %0, %1, %2"
K32D(k_min3_f32_d, ASM)
#undef ASM
#define ASM "v_med3_f32 %0, %0, %1, %2"
K32D(k_med3_f32_d, ASM)
#undef ASM
#define ASM "v_fma_mix_f32 %0, %2, %1, %0 op_sel_hi:[1,0,0]"
K32D(k_fma_mix_lo_d, ASM)
#undef ASM
#define ASM "v_fma_mix_f32 %0, %2, %1, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
K32D(k_fma_mix_hi_d, ASM)
#undef ASM
#define ASM "v_cvt_f32_f16 %0, %1"
K32D(k_cvt_f32_f16_d, ASM)
#undef ASM
#define ASM "v_add3_u32 %0, %0, %1, %2"
K32D(k_add3_u32_d, ASM)
#undef ASM
#define ASM "v_cndmask_b32_e64 %0, %1, %2, s[40:41]"
K32D(k_cndmask_s_d, ASM)
#undef ASM
#define ASM "v_mad_u32_u24 %0, %0, %1, %2"
K32D(k_mad_u32_u24_d, ASM)
#undef ASM
#undef STEPD

#define STEP(x) asm volatile(ASM : "+v"(x) : "v"(c));
#define ASM "v_add_u32 %0, %0, %1"
K32(k_add_u32, ASM)
#undef ASM
#define ASM "v_mul_lo_u32 %0, %0, %1"
K32(k_mul_lo_u32, ASM)
#undef ASM
#define ASM "v_mul_hi_u32 %0, %0, %1"
K32(k_mul_hi_u32, ASM)
#undef ASM
#define ASM "v_mul_u32_u24 %0, %0, %1"
K32(k_mul_u32_u24, ASM)
#undef ASM
#define ASM "v_mul_hi_u32_u24 %0, %0, %1"
K32(k_mul_hi_u32_u24, ASM)
#undef ASM
#define ASM "v_xor_b32 %0, %0, %1"
K32(k_xor_b32, ASM)
#undef ASM
#define ASM "v_alignbit_b32 %0, %0, %1, 13"
K32(k_alignbit, ASM)
#undef ASM
#define ASM "v_fma_f32 %0, %0, %1, %1"
K32(k_fma_f32, ASM)
#undef ASM
#define ASM "v_add_f32 %0, %0, %1"
K32(k_add_f32, ASM)
#undef ASM
#define ASM "v_mul_f32 %0, %0, %1"
K32(k_mul_f32, ASM)
#undef ASM
#define ASM "v_max_f32 %0, %0, %1"
K32(k_max_f32, ASM)
#undef ASM
#define ASM "v_min3_f32 %0, %0, %1, %0"
K32(k_min3_f32, ASM)
#undef ASM
// (the VCC-mask form: k_cndmask_vcc below, with VCC bound as an operand; written as a
// plain K32 kernel it read a VCC the compiler also used, and measured 23 cycles)
#define ASM "v_mov_b32 %0, %1"
K32(k_mov_b32, ASM)
#undef ASM
// (v_cmp_lt_f32 writing VCC: k_cmp_f32 below, with VCC declared clobbered; as a plain K32
// kernel it overwrote the clock stamp the compiler kept in VCC: "measured clock 100 MHz")
#define ASM "v_sqrt_f32 %0, %0"
K32(k_sqrt_f32, ASM)
#undef ASM
#define ASM "v_rcp_f32 %0, %0"
K32(k_rcp_f32, ASM)
#undef ASM
#define ASM "v_cvt_f32_ubyte1 %0, %0"
K32(k_cvt_ubyte, ASM)
#undef ASM
#define ASM "v_fmac_f32 %0, %1, %1"
K32(k_fmac_f32, ASM)
#undef ASM
#define ASM "v_sub_f32 %0, %0, %1"
K32(k_sub_f32, ASM)
#undef ASM
#define ASM "v_min_f32 %0, %0, %1"
K32(k_min_f32, ASM)
#undef ASM
#define ASM "v_max_i32 %0, %0, %1"
K32(k_max_i32, ASM)
#undef ASM
#define ASM "v_med3_f32 %0, %0, %1, %1"
K32(k_med3_f32, ASM)
#undef ASM
#define ASM "v_and_b32 %0, %0, %1"
K32(k_and_b32, ASM)
#undef ASM
#define ASM "v_lshlrev_b32 %0, 3, %0"
K32(k_lshl_b32, ASM)
#undef ASM
#define ASM "v_bfe_u32 %0, %0, 3, 7"
K32(k_bfe_u32, ASM)
#undef ASM
#define ASM "v_cndmask_b32_e64 %0, %0, %1, s[40:41]"
K32(k_cndmask_s, ASM)
#undef ASM
#define ASM "v_perm_b32 %0, %0, %1, %1"
K32(k_perm_b32, ASM)
#undef ASM
#define ASM "v_max_f32_e64 %0, %0, %1"
K32(k_max_f32_e64, ASM)
#undef ASM
#define ASM "v_mul_f32_e64 %0, %0, %1"
K32(k_mul_f32_e64, ASM)
#undef ASM
#define ASM "v_add3_u32 %0, %0, %1, %1"
K32(k_add3_u32, ASM)
#undef ASM
#define ASM "v_cvt_f32_f64 %0, %1"
#undef ASM
#undef STEP

#define K64(name, asmtxt)                                                                   \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t c) {                \
        STAMP(0)                                                                            \
        uint64_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,      \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                     \
        uint64_t cc = c;                                                                    \
        for (int i = 0; i < N_ITER; ++i) {                                                  \
            _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                 \
                BODY8(STEP)                                                                 \
            }                                                                               \
        }                                                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7); \
        STAMP(2)                                                                            \
    }
#define STEP(x) asm volatile(ASM : "+v"(x) : "v"(cc));
#define ASM "v_mad_u64_u32 %0, vcc, %0, %1, %0"
#undef ASM
#define ASM "v_lshrrev_b64 %0, 27, %0"
K64(k_lshr_b64, ASM)
#undef ASM
#define ASM "v_add_f64 %0, %0, %1"
K64(k_add_f64, ASM)
#undef ASM
#define ASM "v_fma_f64 %0, %0, %1, %1"
K64(k_fma_f64, ASM)
#undef ASM
#define ASM "v_lshl_add_u64 %0, %0, 0, %1"
K64(k_lshl_add_u64, ASM)
#undef ASM
#define ASM "v_pk_fma_f32 %0, %0, %1, %1"
K64(k_pk_fma_f32, ASM)
#undef ASM
#define ASM "v_pk_add_f32 %0, %0, %1"
K64(k_pk_add_f32, ASM)
#undef ASM
#define ASM "v_pk_mul_f32 %0, %0, %1"
K64(k_pk_mul_f32, ASM)
#undef ASM
#define ASM "v_mov_b64 %0, %1"
K64(k_mov_b64, ASM)
#undef ASM
#undef STEP

// compares write VCC (declared clobbered): 8 independent compares of the chains' values
__global__ __launch_bounds__(256) void k_cmp_f32(uint32_t *out, uint32_t c) {
    STAMP(0)
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = (float)(threadIdx.x + j);
    const float cf = (float)c;
    for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(x[j]), "v"(cf) : "vcc");
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)x[threadIdx.x & 7];
    STAMP(2)
}
// the VCC-mask select: VCC set by one SALU move per 8 selects, inside the same asm block
__global__ __launch_bounds__(256) void k_cndmask_vcc(uint32_t *out, uint32_t c) {
    STAMP(0)
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    const uint64_t m = 0xAAAAAAAAAAAAAAAAull ^ c;
    for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            asm volatile("s_mov_b64 vcc, %8\n\t"
                         "v_cndmask_b32 %0, %0, %9, vcc\n\tv_cndmask_b32 %1, %1, %9, vcc\n\t"
                         "v_cndmask_b32 %2, %2, %9, vcc\n\tv_cndmask_b32 %3, %3, %9, vcc\n\t"
                         "v_cndmask_b32 %4, %4, %9, vcc\n\tv_cndmask_b32 %5, %5, %9, vcc\n\t"
                         "v_cndmask_b32 %6, %6, %9, vcc\n\tv_cndmask_b32 %7, %7, %9, vcc"
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                         : "s"(m), "v"(c)
                         : "vcc");
        }
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= x[j];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    STAMP(2)
}

// v_mad_u64_u32 writes a 64-bit result from two 32-bit sources
__global__ __launch_bounds__(256) void k_mad_u64_u32(uint32_t *out, uint32_t c) {
    STAMP(0)
    uint64_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
    for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint32_t lo = (uint32_t)x[j];
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[j]) : "v"(lo), "v"(c) : "vcc");
            }
        }
    }
    uint64_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= x[j];
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)r;
    STAMP(2)
}

int main() {
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    const int waves_per_simd = 8, blocks = cus * waves_per_simd;      // 4 waves per block -> 1 per SIMD
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    struct { const char *name; void (*k)(uint32_t *, uint32_t); } ks[] = {
        {"v_add_u32", k_add_u32}, {"v_xor_b32", k_xor_b32}, {"v_fma_f32", k_fma_f32},
        {"v_alignbit_b32", k_alignbit}, {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
        {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mad_u64_u32", k_mad_u64_u32},
        {"v_lshrrev_b64", k_lshr_b64}, {"v_lshl_add_u64", k_lshl_add_u64}, {"v_add_f64", k_add_f64},
        {"v_fma_f64", k_fma_f64}, {"v_add_f32", k_add_f32}, {"v_mul_f32", k_mul_f32}, {"v_max_f32", k_max_f32},
        {"v_min3_f32", k_min3_f32}, {"v_cndmask_b32", k_cndmask_vcc}, {"v_mov_b32", k_mov_b32}, {"v_cmp_lt_f32", k_cmp_f32},
        {"v_sqrt_f32", k_sqrt_f32}, {"v_rcp_f32", k_rcp_f32}, {"v_cvt_f32_ubyte1", k_cvt_ubyte},
        {"v_pk_fma_f32", k_pk_fma_f32}, {"v_pk_add_f32", k_pk_add_f32}, {"v_pk_mul_f32", k_pk_mul_f32},
        {"v_mov_b64", k_mov_b64}, {"v_fmac_f32", k_fmac_f32}, {"v_sub_f32", k_sub_f32}, {"v_min_f32", k_min_f32},
        {"v_max_i32", k_max_i32}, {"v_med3_f32", k_med3_f32}, {"v_and_b32", k_and_b32}, {"v_lshlrev_b32", k_lshl_b32},
        {"v_bfe_u32", k_bfe_u32}, {"v_cndmask_b32 (sgpr mask)", k_cndmask_s}, {"v_perm_b32", k_perm_b32},
        {"v_max_f32_e64", k_max_f32_e64}, {"v_mul_f32_e64", k_mul_f32_e64}, {"v_add3_u32", k_add3_u32},
        {"v_fma_f32 (distinct)", k_fma_f32_d}, {"v_min3_f32 (distinct)", k_min3_f32_d},
        {"v_med3_f32 (distinct)", k_med3_f32_d}, {"v_add3_u32 (distinct)", k_add3_u32_d},
        {"v_cndmask_b32 (sgpr mask, distinct)", k_cndmask_s_d}, {"v_mad_u32_u24 (distinct)", k_mad_u32_u24_d},
        {"v_fma_mix_f32 lo (distinct)", k_fma_mix_lo_d}, {"v_fma_mix_f32 hi (distinct)", k_fma_mix_hi_d},
        {"v_cvt_f32_f16 (distinct)", k_cvt_f32_f16_d}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B9u);   // warm-up
        double mss[5], mhzs[5];
        for (int rep = 0; rep < 5; ++rep) {   // median of 5 launches
            hipEventRecord(a);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B9u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            unsigned long long st[4];
            hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st);
            mss[rep] = ms;
            mhzs[rep] = (double)(st[2] - st[0]) / (double)(st[3] - st[1]) * 100.0;   // shader cycles per 10 ns
        }
        std::sort(mss, mss + 5);
        std::sort(mhzs, mhzs + 5);
        const double ms = mss[2], mhz = mhzs[2];
        const double insts_per_simd = (double)waves_per_simd * N_ITER * 32;
        const double cyc = ms * 1e-3 * clk * 1e3 / insts_per_simd;
        printf("%-18s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (clock %d MHz)  measured clock %.0f MHz: %.2f cycles\n",
               k.name, ms, cyc, clk / 1000, mhz, ms * 1e-3 * mhz * 1e6 / insts_per_simd);
    }
    return 0;
}
