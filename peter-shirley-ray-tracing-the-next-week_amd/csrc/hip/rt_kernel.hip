// rt_kernel.hip — persistent path-tracing megakernel for gfx950 (MI355X).
//
// Device restatement of the reference's hot path:
//   sample loop        main.cpp:299-313   (jitter, get_ray, color, de_nan, col += temp)
//   camera::get_ray    camera.h:41-56
//   color()            main.cpp:25-46     (iterative: throughput * emitted)
//   closest hit        hitable_list.h:20-32 via a BVH2 with exact list-order tie-breaking
//   sphere / moving_sphere / xy|xz|yz_rect / box / flip_normals / translate / rotate_y
//   constant_medium    constant_medium.h:26-50 (evaluated after the surface search)
//   material::scatter  material.h:16-151 ; texture::value texture.h:16-59 ; perlin.h:25-74
//
// Execution model (wave64, CDNA4):
//   * persistent workgroups (16 waves, one per CU, with the BVH2 in LDS; 4 waves with
//     it in HBM; 4 for the flat scan); each LANE owns one camera path at a time and
//     regenerates a new camera sample as soon as its path terminates, so lanes stay
//     busy across bounces (path regeneration) instead of idling until the longest
//     path of the wave finishes;
//   * work = (chunk of `chunk` samples) x (pixel), one sample by default (short items
//     keep a wave's lanes on neighbouring pixels); a wave claims A.claim (<= 512)
//     work items per atomic (one global atomic per claim) and hands them
//     to the lanes that need work with a ballot + mbcnt prefix count;
//   * each item's radiance is summed in registers and stored once into a partial-sum
//     slab [chunk][pixel]; rt_resolve sums the chunks in order (deterministic, no
//     float atomics, independent of the number of GPUs; with one sample per item
//     it is the reference's own `col += temp` order);
//   * the BVH traversal stack lives in LDS, laid out [wave][depth][lane] so every
//     push/pop of a wave is one conflict-free LDS access (16-bit entries with the BVH2
//     in LDS, rt_device.h stk16_*);
//   * ball waves (stage 6, final()'s variant): the workgroup's last A.ball_waves waves
//     gather, through two LDS path pools, the paths whose segments start inside the
//     dense medium's ball, whose closest-hit searches end at the medium cell's few
//     primitives without a BVH descent, so those waves skip the traversal stage;
//   * nodes, primitives and materials are 16-B records read with dwordx4 loads.
//
// Arithmetic follows the reference's float/double promotions; the file is compiled
// with -ffp-contract=off so no FMA is introduced where the reference has none (the
// BVH slab test, which decides nothing about the result, uses explicit fmaf).
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "rt_device.h"

namespace {

// Minimum waves per SIMD the register allocation must allow (launch_bounds second
// argument; 4 -> <= 128 VGPRs -> 16 waves per CU).  5 waves (96 VGPRs) spill 63
// VGPRs and run 24% slower.

// partial sums in the slab: rgb, 12 B per work item (16-B float4 records until round 3)
#define RT_SLAB_FLOATS 3
// Shade once this many lanes of a wave have their closest hit (see stage 3).
#ifndef RT_READY_BATCH
#define RT_READY_BATCH 48
#endif

// Node steps per descent exit check outside the instance variant (rt_device.h descend).
#ifndef RT_DESCEND_STEPS
#define RT_DESCEND_STEPS 2
#endif


// A wave whose claims found the pool dry and that holds at most this many live paths
// runs latency-first (descend's tail cut off)
#ifndef RT_DRY_LANES
#define RT_DRY_LANES 16
#endif


// Pre-made sample starts per wave (refill): one per lane.
#define RT_PRE 64

// Path pools of the ball waves (stage 6): paths whose segment starts inside the medium
// cell's ball, and paths that left it, waiting in LDS for a wave of their kind (80 B each)
#ifndef RT_BALL_POOL
#define RT_BALL_POOL 80
#endif
#ifndef RT_NORM_POOL
#define RT_NORM_POOL 64
#endif
typedef unsigned U4p __attribute__((ext_vector_type(4)));

#ifndef RT_WAVES_PER_SIMD
#define RT_WAVES_PER_SIMD 4
#endif

// kCount: visit counters (RT_FLAG_COUNT).  kProf: wave-level s_memtime stamps per
// stage (RT_FLAG_PROFILE, a diagnostic build whose timing is never quoted).
// Lane phases of the batched state machine below.
// PH_PARK (ball waves): a new segment the medium cell did not decide, waiting for stage 6 to
// move it to a normal wave instead of traversing here
enum : int { PH_IDLE = 0, PH_TRAV = 1, PH_READY = 2, PH_PARK = 3 };

// kFeat (RT_FEAT_*): the scene features the variant carries code for — instance
// chains (cornell scenes), (u, v)-reading materials (earth()), checker textures
// (the random scenes).  The host launches the smallest compiled variant covering
// the scene (final(): media only); RT_FEAT_ALL runs anything.
// kMode, the closest-hit search:
//   0  BVH in HBM (nodes through L1/L2), 4-wave workgroups, 24-entry LDS stacks;
//   1  BVH2 nodes in LDS (one workgroup of RT_LDS_BLOCK threads per CU copies them
//      at launch; node steps read them with ds_read_b128), stacks of the scene's depth;
//   2  flat scan of the primitive groups (rt_layout.h rt_dgroup), primitives in LDS,
//      no BVH and no stack: scenes of at most RT_SCAN_MAX primitives.
// Kernel arguments re-read each loop iteration: the persistent
// loop reads ~40 uniform arguments; held in SGPRs across it they overflowed the 102
// addressable SGPRs, which the compiler spilled into the lanes of a VGPR (v_writelane
// at entry, a v_readlane — a VALU issue — per use).  Through a kernarg pointer that is
// made opaque at the top of every iteration they are scalar loads (SMEM, scalar
// cache) at their first use in the iteration instead (c4 53.01 -> 52.24 ms, c3
// 45.55 -> 45.44 ms; SGPR spills 36 -> 0).
typedef __attribute__((address_space(4))) const RtKernelArgs KArgs;
__device__ __forceinline__ KArgs *opaque_kargs(KArgs *p) {
    asm volatile("" : "+s"(p));
    return p;
}

template <bool kCount, bool kProf, int kWidth, int kFeat, int kMode>
__global__ __launch_bounds__(kMode == 1 ? RT_LDS_BLOCK : RT_BLOCK, RT_WAVES_PER_SIMD) void rt_megakernel(RtKernelArgs A_param) {
    (void)A_param;   // read through ka (the same bytes: the kernarg segment holds A_param at offset 0)
    KArgs *ka = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#define A (*(const RtKernelArgs *)ka)
    constexpr bool kInst = (kFeat & RT_FEAT_INST) != 0, kUV = (kFeat & RT_FEAT_UV) != 0,
                   kChecker = (kFeat & RT_FEAT_CHECKER) != 0, kPrescan = (kFeat & RT_FEAT_PRESCAN) != 0,
                   kMedia = (kFeat & RT_FEAT_MEDIA) != 0;
    constexpr bool kLds = kMode == 1, kScan = kMode == 2;
    // the ball waves (stage 6) and the medium cell that ends their paths' closest-hit searches
    // (stage 3): the media variant without instance chains (final(); a cell needs a medium
    // bounded by one plain sphere, and the instance variants have no registers to spare) with
    // the BVH2 in LDS.  The cell is tested in ball waves only: in the others, whose lanes
    // mostly start outside the ball, its lockstep tests cost every lane (c4 +3.8 %)
    constexpr bool kBall = kMedia && !kInst && kFeat != RT_FEAT_ALL && kLds && kWidth == 2;
    constexpr bool kCell = kBall;
    // the LDS node layout (rt_device.h RtSplit): dword planes in the media variants (final()),
    // float4 planes otherwise, as each measured fastest
    constexpr int kSplit = rt_lds_split(kMode, kFeat, kWidth);
    constexpr int kBlock = kLds ? RT_LDS_BLOCK : RT_BLOCK;
    __shared__ uint32_t lds_stack[kMode ? 1 : RT_BLOCK / 64][kMode ? 1 : (kWidth >= 8 ? RT_STACK_DEPTH_W8 : RT_STACK_DEPTH)][64];
    __shared__ CoopSlot lds_slots[kBlock / 64][64];
    __shared__ MediumRec lds_media[RT_LDS_MEDIA];
    __shared__ CamV4 lds_cam[6];
    __shared__ MediaConsts lds_mconst;
    __shared__ U4j lds_jump[RT_LCG_JUMPS];   // drand48 jump-ahead table (coop_reject)
    // per wave: the next RT_PRE work items' sample starts, made 64 at a time (refill)
    __shared__ uint64_t lds_pre_key[kBlock / 64][RT_PRE];
    __shared__ float2 lds_pre_uv[kBlock / 64][RT_PRE];
    __shared__ uint2 lds_pre_cp[kBlock / 64][RT_PRE];   // each entry's (sample chunk, job pixel)
    // stage 6's path pools (kBall): [0] paths inside the ball, [1] paths outside; a lock, the
    // two counts and the number of ball waves still running
    __shared__ U4p lds_pool_in[kBall ? RT_BALL_POOL : 1][5];
    __shared__ U4p lds_pool_out[kBall ? RT_NORM_POOL : 1][5];
    __shared__ uint32_t lds_pool_ctl[4];
    // (kBall) Perlin's tables (perlin.h:76-79: 256 gradients, 3 x 256 permutations), 7 KiB of
    // the LDS the 16-bit stacks left: the noise texture's dependent gathers from LDS
    __shared__ F4v lds_ranvec[kBall ? 256 : 1];
    __shared__ int lds_perm[kBall ? 768 : 1];
    extern __shared__ float4 lds_dyn[];   // kLds: node planes, then the stacks
    const uint32_t lane = lane_id();
    // the wave's index in the workgroup is wave-uniform: its LDS bases live in SGPRs
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // (LDS variant: 16-bit entries, [wave][depth][lane], rt_device.h stk16_*)
    uint32_t *stk = kLds ? reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(lds_dyn) + lds_node_bytes<kSplit>() +
                                                        (wave * (uint32_t)A.stack_depth * 64u + lane) * 2u)
                         : &lds_stack[kMode ? 0 : wave][0][lane];
    CoopSlot *slots = lds_slots[wave];
    uint64_t *pre_key = lds_pre_key[wave];
    float2 *pre_uv = lds_pre_uv[wave];
    uint2 *pre_cp = lds_pre_cp[wave];
    // the media records are read from LDS (one broadcast read per medium)
    if (kMedia) load_media<kBlock>(A, lds_media);
    if (threadIdx.x == 0) {
        lds_pool_ctl[0] = lds_pool_ctl[1] = lds_pool_ctl[2] = 0;
        lds_pool_ctl[3] = kBall ? (uint32_t)min(max(A.ball_waves, 0), kBlock / 64) : 0u;
        store_camera(A, lds_cam);
        lds_mconst = LogConsts{1.0 / 7, -1.0 / 6, 0.2, -0.25, 1.0 / 3};
    }
    for (uint32_t i = threadIdx.x; i < RT_LCG_JUMPS; i += kBlock) lds_jump[i] = kLcgJump.e[i];
    if (kBall) {
        for (uint32_t i = threadIdx.x; i < 256; i += kBlock) {
            const float4 v = A.ranvec[i];
            lds_ranvec[i] = F4v{v.x, v.y, v.z, v.w};
        }
        for (uint32_t i = threadIdx.x; i < 768; i += kBlock) lds_perm[i] = A.perm[i];
    }
    rtl_lds_init(threadIdx.x);   // rt_libm.h's sine constants
    const LdsJump *jt = (const LdsJump *)lds_jump;
    if (kLds) {
        // interior child references become byte offsets into the planes (n * 16): a
        // node step's LDS address is then the reference itself (LdsNodes)
        for (uint32_t i = threadIdx.x; i < A.nnodes; i += kBlock) {
            const float4 *N = A.nodes + i * 4;
            const float4 b0 = N[0], b1 = N[1], b2 = N[2];
            float4 cf = N[3];
            const uint32_t c0 = (uint32_t)fbits(cf.x), c1 = (uint32_t)fbits(cf.y);
            // leaves in the 16-bit stack form (rt_device.h RT_LDS_LEAF16)
            cf.x = __uint_as_float((c0 & RT_LEAF_BIT) ? RT_LDS_LEAF16(c0) : lds_node_ref<kSplit>(c0));
            cf.y = __uint_as_float((c1 & RT_LEAF_BIT) ? RT_LDS_LEAF16(c1) : lds_node_ref<kSplit>(c1));
            if constexpr (kSplit) {   // one dword per node and plane (rt_device.h RtSplit)
                float *P = reinterpret_cast<float *>(lds_dyn) + i;
                constexpr uint32_t C = RT_LDS_NODE_CAP;
                P[RS_C0 * C] = cf.x; P[RS_C1 * C] = cf.y;
                P[RS_XLO * C] = b0.x; P[(RS_XLO + 1) * C] = b1.z; P[RS_XHI * C] = b0.y; P[(RS_XHI + 1) * C] = b1.w;
                P[RS_YLO * C] = b0.z; P[(RS_YLO + 1) * C] = b2.x; P[RS_YHI * C] = b0.w; P[(RS_YHI + 1) * C] = b2.y;
                P[RS_ZLO * C] = b1.x; P[(RS_ZLO + 1) * C] = b2.z; P[RS_ZHI * C] = b1.y; P[(RS_ZHI + 1) * C] = b2.w;
                continue;
            }
            // the references, then per-axis planes (LdsNodes::load_signed): (lo0, hi0, lo1, hi1) of x, y, z
            lds_dyn[i] = cf;
            lds_dyn[i + RT_LDS_NODE_CAP] = make_float4(b0.x, b0.y, b1.z, b1.w);
            lds_dyn[i + 2 * RT_LDS_NODE_CAP] = make_float4(b0.z, b0.w, b2.x, b2.y);
            lds_dyn[i + 3 * RT_LDS_NODE_CAP] = make_float4(b1.x, b1.y, b2.z, b2.w);
        }
    }
    __syncthreads();
    const GlobalNodes gnodes{A.nodes};
    const LdsNodes<kSplit> lnodes{(const LdsF4 *)lds_dyn};

    const uint64_t skey = seed_key(A.seed);   // per-launch part of the sample keys
    // wave-uniform claim pool, and the pre-made sample starts [pre_head, pre_head + pre_count)
    uint32_t pool_next = 0, pool_end = 0;
    bool exhausted = false;
    // entries [pre_head, pre_head + pre_count) of the wave's pre-made sample starts
    uint32_t pre_head = 0, pre_count = 0;

    // lane state: work item, path, traversal
    uint32_t item = 0xFFFFFFFFu;
    int s_cur = 0, s_end = 0;
    V3 part = mk(0, 0, 0);
    int phase = PH_IDLE;
    bool finished = false;
    Ray r;
    r.o = mk(0, 0, 0); r.d = mk(0, 0, 0); r.time = 0;
    V3 beta = mk(1, 1, 1);
    int depth = 0;
    Rng g; g.x = 0; g.xm = 0;
    // this lane's pre-made sample start, taken by retire_and_claim for camera_begin
    // (read out at once: a refill later in the same claim reuses the slots)
    bool pre_have = false;
    uint64_t pre_k = 0;
    float2 pre_cuv = make_float2(0.f, 0.f);
    uint32_t node = 0;
    int sp = 0;
    float best_t = RT_FLT_MAX;
    int best_key = 0x7FFFFFFF;
    uint32_t best_prim = 0xFFFFFFFFu;

    Counters cnt;
    uint64_t prof[5] = {0, 0, 0, 0, 0};   // claim, traverse, media, shade, of which scatter branches
    uint64_t prof_iters = 0;              // (kProf) this wave's loop iterations
    uint64_t stamp = kProf ? __builtin_amdgcn_s_memtime() : 0;
    // wave timeline (kProf): start, first sight of the empty pool, end (s_memrealtime: one clock for all CUs)
    const uint64_t rt_start = kProf ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t rt_exhaust = 0;
    uint32_t rt_items = 0;   // work items this wave claimed (kProf)
    uint64_t dr_iters = 0, dr_live = 0, dr_taken = 0;   // (kProf) after the dry point: iterations, live lanes, pooled paths taken
    uint64_t dr_prof[4] = {0, 0, 0, 0};                 // (kProf) ... and the stage cycles (claim, traverse, media, shade)
    auto mark = [&](int k) {
        if (kProf) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            prof[k] += now - stamp;
            if (exhausted) dr_prof[k < 4 ? k : 3] += now - stamp;
            stamp = now;
        }
    };
    // a new ray segment: closest-hit search from the root (hitable_list.h:20-32)
    bool fresh = false;   // a new segment the pre-scan has not seen yet
    auto begin_segment = [&](bool counted = true) {
        if (kPrescan || kCell) fresh = true;
        // LDS mode: byte offsets (the root is interior there)
        node = kLds ? lds_node_ref<kSplit>(A.root) : A.root;
        sp = 0;
        best_t = RT_FLT_MAX;
        best_key = 0x7FFFFFFF;
        best_prim = 0xFFFFFFFFu;
        phase = A.has_bvh ? PH_TRAV : PH_READY;
        if (kCount && counted) cnt.segments++;
    };

    // Sample starts are made for 64 work items at once, by all lanes of the wave
    // (refill): each item's pixel, sample key, medium-stream key and the two jitter
    // draws (main.cpp:305-306) — four of a new sample's five hashes, which a lane
    // starting a sample alone would run at the few-lane occupancy of path
    // regeneration.  They wait in the wave's LDS slots until a lane takes one.
    auto refill = [&]() {   // all 64 lanes; wave-uniform outcome
        if (pool_next == pool_end) {
            // claims are counted, not items: claim k < nbig covers A.claim items, later
            // ones A.claim_tail (the launch's last items go out in small claims, so that
            // no wave is left with a large claim while the others have run dry)
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(A.counter, 1u);
            k = __shfl(k, 0);
            const uint32_t big = min(k, A.nbig);
            const uint64_t b64 = (uint64_t)big * A.claim + (uint64_t)(k - big) * A.claim_tail;
            const uint32_t base = (uint32_t)min(b64, (uint64_t)A.nitems);
            const uint32_t size = k < A.nbig ? A.claim : A.claim_tail;
            if (base >= A.nitems) {
                exhausted = true;
                if (kProf) rt_exhaust = __builtin_amdgcn_s_memrealtime();
                return;
            }
            pool_next = base;
            pool_end = min(base + size, A.nitems);
        }
        const uint32_t n = min(64u, pool_end - pool_next);
        if (kProf) rt_items += n;
        if (lane < n) {
            // item -> (sample chunk c, job pixel p): the job's first ndeep pixels (capi.cpp:
            // those whose primary rays enter a dense medium) have all their chunks first,
            // sample-major, then the other pixels' (RtKernelArgs.ndeep)
            const uint32_t it = pool_next + lane;
            uint32_t c, pj;
            if (it < A.ndeep_items) {
                c = it / A.ndeep;
                pj = it - c * A.ndeep;
            } else {
                const uint32_t i2 = it - A.ndeep_items, nb = A.npix - A.ndeep;
                c = i2 / nb;
                pj = A.ndeep + (i2 - c * nb);
            }
            pre_cp[lane] = make_uint2(c, pj);
            const uint32_t xy = A.job_xy[pj];
            const int x = (int)(xy & 0xFFFFu), j = A.ny - 1 - (int)(xy >> 16);
            const uint64_t K = sample_key(skey, (uint32_t)(j * A.nx + x), c * (uint32_t)A.chunk + A.sample_offset);
            // main.cpp:305-306; A.rnx = RN(1/float(nx)) from the host (div_rn)
            const uint64_t x1 = lcg_step(K & kLcgM), x2 = lcg_step(x1);   // the sample's first two draws
            const float cu = div_rn((float)((double)x + u48x(x1)), (float)A.nx, A.rnx);
            const float cv = div_rn((float)((double)j + u48x(x2)), (float)A.ny, A.rny);
            pre_key[lane] = K;
            pre_uv[lane] = make_float2(cu, cv);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pre_head = 0;
        pre_count = n;
        pool_next += n;
    };
    // ---- stage 6's path pools (kBall; DESIGN.md §5c "ball waves") ----------------------
    // The workgroup's last A.ball_waves waves gather the paths whose segment starts inside
    // the medium cell's ball: their closest-hit searches end at the cell's few primitives
    // with no BVH descent, so a wave made of them skips the traversal stage.  Paths move
    // between waves through two LDS pools at segment starts (the whole path state, 80 B:
    // ray, throughput, depth, both drand48 states, the work item and its partial sum), so
    // every sample's draws, adds and slab slot are its own wherever it runs: images are
    // bitwise unchanged.  One spin lock guards both pools; a wave leaves the kernel only
    // after seeing both pools empty, so no path is stranded.
    const bool ballrole = kBall && (int)wave >= kBlock / 64 - A.ball_waves;   // wave-uniform
    typedef __attribute__((address_space(3))) volatile uint32_t LdsVU;
    auto pool_peek = [&](int k) -> uint32_t {   // a racy hint; decisions are made under the lock
        return __builtin_amdgcn_readfirstlane(((LdsVU *)lds_pool_ctl)[1 + k]);
    };
    // (A.ball_drain) with the claims exhausted a normal wave leaves the ball's paths to the ball
    // waves while one runs: there the medium cell ends their searches (in a normal wave a ball
    // path's segment took a full descent, in iterations that wait for the slowest lane: 17 us
    // against 11 in the drain, profiles/r06/wave_drain*.json).  A ball wave leaves under the lock
    // and lowers the count there, so a path pushed to the ball's pool after the last one left
    // is seen by its pusher, which takes it back or stays until the pool is empty.
    auto ball_pool_mine = [&]() -> bool {
        return ballrole || !A.ball_drain || __builtin_amdgcn_readfirstlane(((LdsVU *)lds_pool_ctl)[3]) == 0u;
    };
    auto pool_lock = [&]() {
        if (lane == 0)
            while (atomicCAS(&lds_pool_ctl[0], 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    };
    auto pool_unlock = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) atomicExch(&lds_pool_ctl[0], 0u);
    };
    auto pool_entry = [&](int k, uint32_t e) -> U4p * { return k == 0 ? lds_pool_in[e] : lds_pool_out[e]; };
    // lanes with `want` (a fresh segment) leave for pool k while it has room; returns who left
    auto pool_push = [&](int k, bool want) -> bool {
        const uint64_t M = wballot(want);
        if (M == 0ull) return false;
        const uint32_t cap = k == 0 ? RT_BALL_POOL : RT_NORM_POOL;
        if (pool_peek(k) >= cap) {
            if (kCount && k == 0 && lane == 0) cnt.ball[RT_BALL_DENIED] += (uint64_t)__popcll(M);
            return false;
        }
        pool_lock();
        const uint32_t n = __builtin_amdgcn_readfirstlane(((LdsVU *)lds_pool_ctl)[1 + k]);
        const uint32_t take = min((uint32_t)__popcll(M), cap - min(n, cap));
        const uint32_t rank = lanes_below(M);
        const bool go = want && rank < take;
        if (go) {
            U4p *E = pool_entry(k, n + rank);
            E[0] = U4p{__float_as_uint(r.o.x), __float_as_uint(r.o.y), __float_as_uint(r.o.z), __float_as_uint(r.time)};
            E[1] = U4p{__float_as_uint(r.d.x), __float_as_uint(r.d.y), __float_as_uint(r.d.z), __float_as_uint(beta.x)};
            E[2] = U4p{__float_as_uint(beta.y), __float_as_uint(beta.z), __float_as_uint(part.x), __float_as_uint(part.y)};
            E[3] = U4p{__float_as_uint(part.z), item, (uint32_t)s_cur, (uint32_t)s_end};
            E[4] = U4p{(uint32_t)g.x, (uint32_t)(g.x >> 32) | ((uint32_t)depth << 16), (uint32_t)g.xm, (uint32_t)(g.xm >> 32)};
        }
        if (lane == 0) ((LdsVU *)lds_pool_ctl)[1 + k] = n + take;
        pool_unlock();
        if (kCount && lane == 0) {
            cnt.ball[k == 0 ? RT_BALL_PUSH_IN : RT_BALL_PUSH_OUT] += take;
            if (k == 0) cnt.ball[RT_BALL_DENIED] += (uint64_t)__popcll(M) - take;
        }
        return go;
    };
    // lanes with `need` take paths from pool k (a fresh segment each); returns who took one
    auto pool_take = [&](int k, bool need) -> bool {
        const uint64_t M = wballot(need);
        if (M == 0ull || pool_peek(k) == 0u) return false;
        pool_lock();
        const uint32_t n = __builtin_amdgcn_readfirstlane(((LdsVU *)lds_pool_ctl)[1 + k]);
        const uint32_t take = min((uint32_t)__popcll(M), n);
        const uint32_t rank = lanes_below(M);
        const bool got = need && rank < take;
        if (got) {
            const U4p *E = pool_entry(k, n - take + rank);
            const U4p e0 = E[0], e1 = E[1], e2 = E[2], e3 = E[3], e4 = E[4];
            r.o = mk(__uint_as_float(e0.x), __uint_as_float(e0.y), __uint_as_float(e0.z));
            r.time = __uint_as_float(e0.w);
            r.d = mk(__uint_as_float(e1.x), __uint_as_float(e1.y), __uint_as_float(e1.z));
            beta = mk(__uint_as_float(e1.w), __uint_as_float(e2.x), __uint_as_float(e2.y));
            part = mk(__uint_as_float(e2.z), __uint_as_float(e2.w), __uint_as_float(e3.x));
            item = e3.y;
            s_cur = (int)e3.z;
            s_end = (int)e3.w;
            g.x = ((uint64_t)(e4.y & 0xFFFFu) << 32) | e4.x;
            depth = (int)(e4.y >> 16);
            g.xm = ((uint64_t)e4.w << 32) | e4.z;
        }
        if (lane == 0) ((LdsVU *)lds_pool_ctl)[1 + k] = n - take;
        pool_unlock();
        if (kCount && lane == 0) cnt.ball[RT_BALL_TAKEN] += take;
        if (kProf && exhausted) dr_taken += take;
        if (got) {
            finished = false;
            pre_have = false;
            begin_segment(false);   // (the segment was counted where it began)
        }
        return got;
    };

    // retire a finished work item (its sum to the slab), hand the lanes without work
    // the next pre-made sample starts (one global atomic per A.claim items).  top: the call
    // at the top of the iteration, the only one that takes pooled paths (kBall; one inlined
    // copy of the path-state load, where two spilled); in the other, a ball wave whose pool
    // holds paths leaves its idle lanes for the next top
    auto retire_and_claim = [&](bool top) {
        if (phase == PH_IDLE && !finished && item != 0xFFFFFFFFu && s_cur == s_end) {
            float *sl = A.slab + (size_t)item * RT_SLAB_FLOATS;   // 12 B per item
            sl[0] = part.x;
            sl[1] = part.y;
            sl[2] = part.z;
            item = 0xFFFFFFFFu;
        }
        bool need = phase == PH_IDLE && !finished && item == 0xFFFFFFFFu;
        if constexpr (kBall) {
            if (top) {
                // a ball wave takes the ball's paths first, the others the paths that left
                // it; lanes that found no work before (finished) look again: the pools refill
                need = phase == PH_IDLE && item == 0xFFFFFFFFu;
                // pool 0 holds the ball's paths, 1 the others'; with the claims exhausted a
                // wave whose own pool is empty takes from the other
                const bool other = exhausted && pool_peek(ballrole ? 0 : 1) == 0u && ball_pool_mine();
                const int k = (other == ballrole) ? 1 : 0;
                if (pool_take(k, need)) need = false;
            }
            if (ballrole && !exhausted) {
                // a ball wave claims new samples only while fewer than A.ball_claim of its lanes
                // hold a path, and outside the top only with its pool empty (its idle lanes wait
                // for the pool's paths at the next top); lanes left idle have no item.  A wave
                // with no path at all always claims at the top: only a claim finds the pool
                // exhausted, and a wave that never did would never leave the kernel.
                const uint32_t busy = (uint32_t)__popcll(wballot(!(phase == PH_IDLE && item == 0xFFFFFFFFu)));
                if ((!top && pool_peek(0) != 0u) || (busy >= (uint32_t)A.ball_claim && !(top && busy == 0u))) return;
            }
        }
        uint64_t need_mask = wballot(need);
        while (need_mask != 0ull) {
            if (pre_count == 0) {
                if (!exhausted) refill();
                if (pre_count == 0) break;
            }
            const uint32_t rank = lanes_below(need_mask);
            if (need && rank < pre_count) {
                const uint32_t e = pre_head + rank;
                pre_k = pre_key[e];
                pre_cuv = pre_uv[e];
                const uint2 cp = pre_cp[e];
                const uint32_t c = cp.x;
                item = c * A.npix + cp.y;   // the slab slot: [chunk][job pixel]
                pre_have = true;
                need = false;
                s_cur = (int)(c * (uint32_t)A.chunk);
                s_end = min(s_cur + A.chunk, A.ns);
                part = mk(0, 0, 0);
            }
            const uint32_t took = min((uint32_t)__popcll(need_mask), pre_count);
            pre_head += took;
            pre_count -= took;
            need_mask = wballot(need);
        }
        if (need) finished = true;
    };
    // a camera sample (main.cpp:305-308, camera.h:41-56): the sample's stream and
    // jitter, then (after the lens-disk point) the ray
    auto camera_begin = [&](bool starting, float &cu_, float &cv_) {
        if (starting) {
            if (pre_have) {   // a work item's first sample: made by refill
                g.start(pre_k, kMedia);
                g.skip2();   // the two jitter draws
                cu_ = pre_cuv.x;
                cv_ = pre_cuv.y;
                pre_have = false;
            } else {            // a further sample of a multi-sample work item (chunk > 1)
                const uint32_t c = item / A.npix;
                const uint32_t xy = A.job_xy[item - c * A.npix];
                const int px = (int)(xy & 0xFFFFu), j = A.ny - 1 - (int)(xy >> 16);
                g.start(sample_key(skey, (uint32_t)(j * A.nx + px), (uint32_t)s_cur + A.sample_offset), kMedia);
                cu_ = div_rn((float)((double)px + g.next()), (float)A.nx, A.rnx);
                cv_ = div_rn((float)((double)j + g.next()), (float)A.ny, A.rny);
            }
        }
    };
    // seg: begin the segment here (else the caller does)
    auto camera_finish = [&](bool starting, float cu_, float cv_, V3 disk, bool seg = true) {
        if (starting) {
            const CamView C = load_camera(lds_cam);
            V3 rd = scale(C.lens, disk);
            V3 offset = add(scale(rd.x, C.cu), scale(rd.y, C.cv));
            // camera.h:54: a closed shutter (t1 - t0 == 0, final() and the Cornell scenes)
            // gives time0 + u*0 = time0 for every draw u, so the draw is consumed unhashed
            const float span = C.t1 - C.t0;
            double u = 0.0;
            if (span != 0.0f) u = g.next(); else g.skip();
            float time = (float)((double)C.t0 + u * (double)span);
            V3 org = C.org;
            V3 dir = sub(sub(add(add(C.llc, scale(cu_, C.hor)), scale(cv_, C.ver)), org), offset);
            r.o = add(org, offset);
            r.d = dir;
            r.time = time;
            beta = mk(1, 1, 1);
            depth = 0;
            if (kCount) cnt.samples++;
            if (seg) begin_segment();
        }
    };
    // a path's radiance into its work item (de_nan, main.cpp:232-242; col += temp)
    auto end_path = [&](V3 L) {
        if (!(L.x == L.x)) L.x = 0;
        if (!(L.y == L.y)) L.y = 0;
        if (!(L.z == L.z)) L.z = 0;
        part = add(part, L);
        ++s_cur;
        phase = PH_IDLE;
    };

    for (;;) {
        // (not in the flat-scan variant: its scan reads the group records right at the
        // iteration's start, and the reload measured slower there, c2 37.63 -> 37.88 ms)
        if (!kScan) ka = opaque_kargs(ka);
        // ---- 1. claims and camera samples for lanes without a path --------------
        // (the first iteration, and paths that ended after the shading stage's
        // cooperative rounds: a metal's absorbed reflection; the others start their
        // next sample inside stage 5)
        retire_and_claim(true);
        const uint64_t live = wballot(!finished);
        // (kBall) a wave leaves only with the pools it serves empty: paths another wave left there
        // are taken by the next iteration's retire_and_claim (this one runs with no lane active).
        // A ball wave serves both and decides under the lock (ball_pool_mine)
        if (live == 0ull) {
            if (!kBall) break;
            if ((pool_peek(1) | (ball_pool_mine() ? pool_peek(0) : 0u)) == 0u) {
                if (!ballrole) break;
                pool_lock();
                const bool leave = (pool_peek(0) | pool_peek(1)) == 0u;
                if (leave && lane == 0) ((LdsVU *)lds_pool_ctl)[3] = ((LdsVU *)lds_pool_ctl)[3] - 1u;
                pool_unlock();
                if (leave) break;
            }
        }
        // the pool is dry and few paths are left: the launch's end waits on their latency
        const bool dry = exhausted && __popcll(live) <= RT_DRY_LANES;
        {
            const bool starting = phase == PH_IDLE && !finished && (!kBall || item != 0xFFFFFFFFu);
            float cu_ = (RT_SHADE_LEAN & 8) ? unset_f() : 0.f, cv_ = (RT_SHADE_LEAN & 8) ? unset_f() : 0.f;   // starting lanes only
            camera_begin(starting, cu_, cv_);
            const V3 disk = coop_reject<2, kCount>(starting, g, slots, jt, lane, cnt, DiskCand());
            camera_finish(starting, cu_, cv_, disk);
        }
        mark(0);
        if (kCount && first_active()) cnt.w_iters++;

        // ---- 3. closest surface hit: BVH traversal rounds --------------------
        // A round = descend until all but RT_DESCEND_TAIL searching lanes hold a
        // leaf, test the leaves.  The
        // wave keeps running rounds for the lanes still searching until
        // RT_READY_BATCH lanes have their hit, then shades that batch: a lane that
        // finished early no longer holds the wave in traversal, and a lane still
        // searching keeps its LDS stack and carries on in the next iteration.
        if constexpr (kScan) {
            // ---- 3'. closest surface hit, flat scan: every lane with a new segment,
            // group by group (box test for all lanes, skipped when none hits; one
            // object-space transform per group), primitive by primitive in lockstep.
            const bool act = phase == PH_TRAV;
            if (wballot(act) != 0ull) {
                // the records through the scalar cache (every lane reads the same one): SGPR
                // operands, no LDS round trip per primitive (an LDS copy: c2 52.58 -> 51.93 ms)
                const ConstF4 *P = (const ConstF4 *)A.prims;
                const ConstF4 *G = (const ConstF4 *)A.groups;
                const Slab sl = make_slab<kSplit>(r, A.tmin);
                ScanBest b{best_t, 0x7FFFFFFF};   // a new segment: nothing found yet
                for (int gi = 0; gi < A.ngroups; ++gi) {
                    const F4v gh = G[3 * gi], bx = G[3 * gi + 1], bz = G[3 * gi + 2];
                    float tn, tf;
                    box_span(sl, F2{bx.x, bx.y}, F2{bx.z, bx.w}, F2{bz.x, bz.y}, b.t, tn, tf);
                    const bool in = act && tn <= tf;
                    if (kCount && act) { cnt.nodes++; if (first_active()) cnt.w_nodes++; }
                    if (wballot(in) == 0ull) continue;
                    const int first = __builtin_amdgcn_readfirstlane(fbits(gh.x));
                    const int kinds = __builtin_amdgcn_readfirstlane(fbits(gh.w));
                    const int nyz = __builtin_amdgcn_readfirstlane(fbits(bz.z));
                    const int inst = __builtin_amdgcn_readfirstlane(fbits(gh.z));
                    Ray ro = r;
                    if (kInst && inst >= 0) ro = to_object_uniform(A.insts, inst, r);
                    scan_group<kCount, kInst>(P, first, kinds, nyz, inst, ro, A.tmin, in, b, cnt);
                }
                best_t = b.t;
                if (b.kp != 0x7FFFFFFF) { best_key = b.kp >> 8; best_prim = (uint32_t)(b.kp & 0xff); }
                if (act) phase = PH_READY;
            }
        } else {
            // the medium cell (capi.cpp): a new segment starting inside the ball tests the
            // primitives near it; a hit before the ray leaves the ball is the closest of
            // all (every other primitive lies outside), and the search ends without a descent
            if (kCell && ballrole && A.cell_n > 0) {
                bool in = false;
                float tsafe = 0.f;
                const bool fr = fresh && phase == PH_TRAV;
                if (fr) {
                    const V3 oc = sub(r.o, mk(A.cell_c[0], A.cell_c[1], A.cell_c[2]));
                    const float a = dot(r.d, r.d), b = dot(oc, r.d), cc = dot(oc, oc) - A.cell_r2;
                    if (cc < 0.f && a > 0.f) {
                        // where the ray leaves the ball: the larger root, without cancellation
                        // (approximate square root and reciprocals, ~1 ulp each: a bound, not a result)
                        const float q = __builtin_amdgcn_sqrtf(b * b - a * cc);
                        const float te = b >= 0.f ? -cc * __builtin_amdgcn_rcpf(b + q) : (q - b) * __builtin_amdgcn_rcpf(a);
                        tsafe = te * (1.f - 1.f / 4096);   // below it by far more than its rounding
                        in = true;
                    }
                }
                if (wballot(in) != 0ull) {
                    lockstep_prims<kCount, kInst, true>((const ConstF4 *)A.prims, A.cell_first, A.cell_n, A.insts, r, A.tmin,
                                                        in, -1, best_t, best_key, best_prim, cnt);
                    if (in && best_t < tsafe) phase = PH_READY;
                    if (kCount) {
                        const uint64_t decided = wballot(in && phase == PH_READY);
                        if (lane == 0) cnt.ball[RT_BALL_CELL_BALL] += (uint64_t)__popcll(decided);
                    }
                }
                // a new segment the cell did not decide waits for stage 6 to leave for a normal
                // wave (A.ball_park): a ball wave's few traversing lanes ran its traversal rounds
                // at a few lanes each.  Not once the claims are exhausted: a ball wave then takes
                // the other pool's paths too, and parking them again could pass a path between
                // the pool and a ball wave forever when no normal wave is left
                if (A.ball_park && !exhausted && fr && phase == PH_TRAV) phase = PH_PARK;
            }
            // pre-scan: the scene's largest primitives (capi.cpp), kept out of the BVH,
            // tested in lockstep by every lane with a new segment before its descent;
            // their hits also shorten best_t, which culls more of the BVH
            if (kPrescan && A.nprescan > 0) {
                const bool fr = fresh && phase == PH_TRAV;
                if (wballot(fr) != 0ull)
                    lockstep_prims<kCount, kInst, true>((const ConstF4 *)A.prims, 0, A.nprescan, A.insts, r, A.tmin, fr, -1,
                                                        best_t, best_key, best_prim, cnt);
            }
            if (kPrescan || kCell) fresh = false;
            if (kCount && ballrole && lane == 0) {
                cnt.ball[RT_BALL_ITERS]++;
                cnt.ball[RT_BALL_LIVE] += (uint64_t)__popcll(live);
            }
            const int batch = ballrole ? A.ball_batch : RT_READY_BATCH;
            for (;;) {
                if (wballot(phase == PH_TRAV) == 0ull) break;
                if (__popcll(wballot(phase == PH_READY)) >= batch) break;
                if (kCount && ballrole && lane == 0) cnt.ball[RT_BALL_ROUNDS]++;
                if (phase == PH_TRAV) {
                    // the slab test needs no exact division: boxes are padded (bvh.cpp)
                    Slab sl = make_slab<kSplit>(r, A.tmin);
                    uint32_t pleaf;
                    if constexpr (kLds && kWidth == 2) lnodes.prepare(sl);
                    if constexpr (kLds)
                        pleaf = descend<kWidth, kCount, kInst ? 1 : RT_DESCEND_STEPS>(lnodes, node, sl, best_t, stk, sp, cnt, dry);
                    else
                        pleaf = descend<kWidth, kCount, kInst ? 1 : RT_DESCEND_STEPS>(gnodes, node, sl, best_t, stk, sp, cnt, dry);
                    if (pleaf != RT_EMPTY_CHILD) {
                        const uint32_t first = kLds ? RT_LDS_LEAF16_FIRST(pleaf) : RT_LEAF_FIRST(pleaf),
                                       nleaf = kLds ? RT_LDS_LEAF16_COUNT(pleaf) : RT_LEAF_COUNT(pleaf);
                        // primitives in pairs: both 32-B heads are fetched before either test
                        for (uint32_t q = 0; q < nleaf; q += 2) {
                            const uint32_t ia = first + q;
                            const bool two = q + 1 < nleaf;
                            const uint32_t ib = two ? ia + 1 : ia;
                            const float4 ga = A.prims[ia * 4 + 0], ma = A.prims[ia * 4 + 1];
                            const float4 gb = A.prims[ib * 4 + 0], mb = A.prims[ib * 4 + 1];
                            auto test_pair = [&](auto kinds) {
                                constexpr int kK = decltype(kinds)::value;
                                int key, kind;
                                float t = prim_t_head<kInst, kK>(ga, ma, A.prims, A.insts, ia, r, A.tmin, key, kind);
                                if (kCount) { cnt.prim(kind); if (first_active()) cnt.w_prims++; }
                                keep_closest(true, t, key, ia, best_t, best_key, best_prim);
                                if (two) {
                                    t = prim_t_head<kInst, kK>(gb, mb, A.prims, A.insts, ib, r, A.tmin, key, kind);
                                    if (kCount) { cnt.prim(kind); if (first_active()) cnt.w_prims++; }
                                    keep_closest(true, t, key, ib, best_t, best_key, best_prim);
                                }
                            };
                            // the kinds the wave tests in this pass: a wave of spheres only or of
                            // rects only runs that kind's test alone (final(): most passes)
                            const bool ra = (fbits(ma.x) & 0xff) > RT_PRIM_MOVING_SPHERE;
                            const bool rb = two && (fbits(mb.x) & 0xff) > RT_PRIM_MOVING_SPHERE;
                            const bool sb = two && !rb;
                            if (wballot(ra || rb) == 0ull) test_pair(std::integral_constant<int, 1>());
                            else if (wballot(!ra || sb) == 0ull) test_pair(std::integral_constant<int, 2>());
                            else test_pair(std::integral_constant<int, 3>());
                        }
                    }
                    if (node == RT_EMPTY_CHILD) phase = PH_READY;   // stack empty too (popped above)
                }
            }
        }
        mark(1);
        // Lanes still searching carry on in the next iteration; the others shade.
        // Stages 4-5 keep the whole wave active (the cooperative sampler needs it).
        const bool ready = phase == PH_READY;

        // ---- 4. media after the surfaces, then the hit record -------------------
        bool have = false;
        // |r.d| once per segment, for the media and the specular materials / sky
        const float dlen = (ready && A.need_dlen) ? len(r.d) : 0.f;
        const Recip rd = recip_of(dlen, ready && A.need_dlen);   // its reciprocal, for div_rn
        Hit hr;   // read only by lanes with a hit (shade_begin / shade_finish guard on `have`)
        if (RT_SHADE_LEAN & 2) {
            hr.p = unset_v3(); hr.n = unset_v3(); hr.u = unset_f(); hr.v = unset_f(); hr.mat = 0;   // the index stays defined
        } else {
            hr.p = mk(0, 0, 0); hr.n = mk(0, 0, 0); hr.u = 0.f; hr.v = 0.f; hr.mat = 0;
        }
        if (ready) {
            have = best_prim != 0xFFFFFFFFu;
            const int med_mat = kMedia ? media_hit<kCount, kInst>(A, lds_media, (LdsMediaConsts *)&lds_mconst, r, rd, g, have,
                                                                  best_t, cnt)
                                       : -1;
            if (med_mat >= 0) {
                hr.p = at(r, best_t);
                hr.n = mk(1, 0, 0);
                hr.mat = med_mat;   // constant_medium.h:41-44 leaves u, v stale; no medium texture reads them
            } else if (have) {
                hr = prim_record<kInst, kUV>(A.prims, A.insts, A.mats, best_prim, r, best_t);
            }
        }

        mark(2);
        // ---- 5. shade (main.cpp:27-45, material.h) ------------------------------
        // Paths that end at this segment whatever the scatter draws (a miss, a light,
        // the depth limit) add their radiance, retire, claim and draw their next camera
        // sample's jitter right here, so that the new samples' lens-disk candidates run
        // in the same cooperative rounds as the scattering lanes' sphere candidates.
        typedef __attribute__((address_space(3))) const F4v LdsRanvec;
        typedef __attribute__((address_space(3))) const int LdsPerm;
        const ShadeState st = kBall ? shade_begin<kCount, kUV, kChecker>(A, ready, have, hr, depth, slots, lane, cnt,
                                                                         (LdsRanvec *)lds_ranvec, (LdsPerm *)lds_perm)
                                    : shade_begin<kCount, kUV, kChecker>(A, ready, have, hr, depth, slots, lane, cnt,
                                                                         A.ranvec, A.perm);
        const bool ends = shade_ends(ready, have, st);
        if (kCount) {   // material divergence: the scatter branches this wave pass runs (shade_finish)
            const bool sc = ready && !ends;
            if (wballot(sc) != 0ull) {
                const int kinds = (wballot(sc && st.kind == RT_MAT_LAMBERTIAN) != 0ull) +
                                  (wballot(sc && st.kind == RT_MAT_METAL) != 0ull) +
                                  (wballot(sc && st.kind == RT_MAT_DIELECTRIC) != 0ull) +
                                  (wballot(sc && st.kind == RT_MAT_ISOTROPIC) != 0ull);
                if (first_active()) { cnt.w_shade++; cnt.w_kinds += (uint64_t)kinds; }
                if (sc) cnt.l_scatter++;
            }
        }
        if (ends) end_path(mul(beta, shade_emitted(A, have, r, rd, st)));
        retire_and_claim(false);
        // (a lane left without work by a ball wave's claim, waiting for the pool, has no item)
        const bool starting = phase == PH_IDLE && !finished && (!kBall || item != 0xFFFFFFFFu);
        float cu_ = (RT_SHADE_LEAN & 8) ? unset_f() : 0.f, cv_ = (RT_SHADE_LEAN & 8) ? unset_f() : 0.f;   // starting lanes only
        camera_begin(starting, cu_, cv_);
        // material.h:41-47 for the scattering lanes, camera.h:6-12 for the new samples
        const V3 pt = coop_reject_mixed<kCount>(st.wants_sphere || starting, starting, g, slots, jt, lane, cnt);
        mark(3);
        // a scattered path and a new camera sample (disjoint lanes: a lane that started
        // a sample this iteration was idle, not ready) begin their next segment in ONE
        // place: the compiler otherwise materialises the segment state in both divergent
        // branches
        bool seg = false;
        if (ready && !ends) {
            const ShadeOut so = shade_finish(A, ready, have, r, rd, hr, st, pt, g);
            if (so.scattered) {
                beta = mul(beta, so.att);
                r = so.ray;
                ++depth;
                seg = true;
            } else {
                end_path(mul(beta, so.emitted));
            }
        }
        mark(4);
        camera_finish(starting, cu_, cv_, pt, false);
        if (seg || starting) begin_segment();
        // ---- 6. regroup (kBall): a scattered path whose new segment starts inside the
        // medium cell's ball leaves a normal wave for the ball waves' pool, one that starts
        // outside leaves a ball wave for the others' pool (while the pool has room); the
        // lane takes new work at the next claim
        if constexpr (kBall) {
            if (A.ball_waves > 0 && A.cell_n > 0) {
                // inside the ball, and not a ray leaving it from its surface (a refraction out of
                // the glass, a reflection off it): the cell would not decide those
                const V3 oc = sub(r.o, mk(A.cell_c[0], A.cell_c[1], A.cell_c[2]));
                const float o2 = dot(oc, oc);
                const bool inball = o2 < A.cell_r2 && (o2 < A.cell_rin2 || dot(oc, r.d) < 0.f);
                const bool parked = phase == PH_PARK;
                if (pool_push(ballrole ? 1 : 0, (seg && (inball != ballrole)) || parked)) {
                    phase = PH_IDLE;
                    item = 0xFFFFFFFFu;
                } else if (parked) {
                    phase = PH_TRAV;   // the pool is full: it traverses here after all
                }
            }
        }
        mark(3);
        if (kProf) {
            prof_iters++;
            if (exhausted) { dr_iters++; dr_live += (uint64_t)__popcll(live); }
        }
    }
    if (kProf && lane == 0) {
        if (kBall) {   // RT_STAT_BALL in the profile variant: the ball waves' stage cycles and iterations
            if (ballrole) {
                for (int k = 0; k < 4; ++k) atomicAdd(&A.stats[RT_STAT_BALL + k], (unsigned long long)(prof[k] + (k == 3 ? prof[4] : 0)));
                atomicAdd(&A.stats[RT_STAT_BALL + 4], (unsigned long long)prof_iters);
            }
            atomicAdd(&A.stats[RT_STAT_BALL + 5], (unsigned long long)prof_iters);
        }
        // the scatter branches' cycles count in the shade stage too
        for (int k = 0; k < 4; ++k) atomicAdd(&A.stats[RT_STAT_PROF + k], (unsigned long long)(prof[k] + (k == 3 ? prof[4] : 0)));
        atomicAdd(&A.stats[RT_STAT_SHADE + 3], (unsigned long long)prof[4]);
        // minima as maxima of the complement (the slots start at 0)
        const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
        unsigned long long *T = A.stats + RT_STAT_TIME;
        atomicMax(&T[0], ~(unsigned long long)rt_start);
        atomicMax(&T[1], ~(unsigned long long)(rt_exhaust ? rt_exhaust : rt_end));
        atomicMax(&T[2], (unsigned long long)(rt_exhaust ? rt_exhaust : rt_end));
        atomicMax(&T[3], ~rt_end);
        atomicMax(&T[4], rt_end);
        // sum of the waves' lifetimes (end - own start: no overflow of absolute clock values
        // summed over ~4,096 waves); the waves of a persistent grid start within µs of T[0]
        atomicAdd(&T[5], rt_end - (unsigned long long)rt_start);
        atomicAdd(&T[6], 1ull);
        if (A.wave_log) {   // HW_ID (cu, simd, wave slot, se) and XCC_ID through s_getreg (reads)
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
            unsigned long long *W = A.wave_log + RT_WAVE_LOG_WORDS * ((size_t)blockIdx.x * (kBlock / 64) + wave);
            W[0] = rt_start;
            W[1] = rt_exhaust ? rt_exhaust : rt_end;
            W[2] = rt_end;
            W[3] = ((unsigned long long)xcc << 32) | hw;
            W[4] = rt_items;
            W[5] = dr_iters;
            W[6] = dr_live;
            W[7] = dr_taken;
            for (int k = 0; k < 4; ++k) W[8 + k] = dr_prof[k];
        }
    }
    if (kCount) {
        uint64_t w[8] = {cnt.w_iters, cnt.w_nodes, cnt.w_prims, cnt.w_rius, cnt.l_rius, cnt.w_shade, cnt.w_kinds, cnt.l_scatter};
        for (int k = 0; k < 8; ++k) {
            uint64_t x = w[k];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off);
            if (lane == 0 && x) atomicAdd(&A.stats[k < 5 ? RT_STAT_WAVE + k : RT_STAT_SHADE + (k - 5)], (unsigned long long)x);
        }
    }

    if (kCount && kBall && lane == 0)
        for (int k = 0; k < RT_BALL_N; ++k)
            if (cnt.ball[k]) atomicAdd(&A.stats[RT_STAT_BALL + k], (unsigned long long)cnt.ball[k]);
    if (kCount) {
        uint64_t v[RT_CNT_N] = {cnt.samples, cnt.segments, cnt.nodes, cnt.spheres, cnt.mspheres, cnt.rects,
                                cnt.instanced, cnt.media, cnt.shades, cnt.noise};
        for (int k = 0; k < RT_CNT_N; ++k) {
            uint64_t x = v[k];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off);
            if (lane == 0 && x) atomicAdd(&A.stats[k], (unsigned long long)x);
        }
    }
}

#undef A

// Adds one sample batch's partial sums to each pixel's running sum, in sample
// order (main.cpp:311 `col += temp`, one add per sample with one sample per work
// item), so the image does not depend on how the samples were split into batches
// (capi.cpp bounds the slab per launch).  The last batch applies `col /= float(ns)`
// as the reciprocal multiply of vec3.h:134-141.
__global__ __launch_bounds__(256) void rt_resolve(const float *__restrict__ slab, uint32_t npix, int nchunks, float k,
                                                  float4 *__restrict__ acc, int mode,
                                                  const uint32_t *__restrict__ out_index, float *__restrict__ out) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    const uint32_t o = out_index[p];
    V3 col = mk(0, 0, 0);
    if (!(mode & RT_RESOLVE_FIRST)) {
        const float4 a = acc[p];
        col = mk(a.x, a.y, a.z);
    } else if (mode & RT_RESOLVE_SUM_IN) {
        col = mk(out[3 * (size_t)o + 0], out[3 * (size_t)o + 1], out[3 * (size_t)o + 2]);
    }
#pragma unroll 8
    for (int c = 0; c < nchunks; ++c) {   // the loads run ahead; the adds stay in sample order
        const float *v = slab + ((size_t)c * npix + p) * RT_SLAB_FLOATS;
        col = add(col, mk(v[0], v[1], v[2]));
    }
    if (!(mode & RT_RESOLVE_LAST)) {
        acc[p] = make_float4(col.x, col.y, col.z, 0.f);
        return;
    }
    if (!(mode & RT_RESOLVE_RAW)) col = scale(k, col);
    out[3 * (size_t)o + 0] = col.x;
    out[3 * (size_t)o + 1] = col.y;
    out[3 * (size_t)o + 2] = col.z;
}

// Diagnostic (rt_math_probe): the device's float transcendentals on n inputs, for the
// GPU tests to compare with glibc — fn 0 rt_sinf, 1 ocml sinf, 2 rt_asinf, 3 ocml asinf,
// 4 rt_atan2f(a, b), 5 ocml atan2f(a, b) (rt_libm.h; the ocml forms are what the
// megakernel used until round 5).
__global__ __launch_bounds__(256) void rt_math_probe_kernel(int fn, const float *__restrict__ a,
                                                            const float *__restrict__ b, float *__restrict__ out, int n) {
    rtl_lds_init(threadIdx.x);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i];
    float r;
    switch (fn) {
    case 0: r = rt_sinf(x); break;
    case 1: r = sinf(x); break;
    case 2: r = rt_asinf(x); break;
    case 3: r = asinf(x); break;
    case 4: r = rt_atan2f(x, b[i]); break;
    default: r = atan2f(x, b[i]); break;
    }
    out[i] = r;
}

#ifdef RT_KNOB_CHECK
// tests/test_device_knobs.py: a device-only build of final()'s variant (BVH2 in LDS, media)
// and cornell_box's (flat scan, instances), with a non-default value of one compile-time
// knob — seconds instead of the whole variant set's minute — so no knob value goes uncompiled.
template __global__ void rt_megakernel<false, false, 2, RT_FEAT_MEDIA, 1>(RtKernelArgs);
template __global__ void rt_megakernel<false, false, 2, RT_FEAT_INST, 2>(RtKernelArgs);
#endif
}  // namespace

#ifndef RT_KNOB_CHECK
extern "C" hipError_t rt_launch_math_probe(int fn, const float *a, const float *b, float *out, int n, hipStream_t stream) {
    hipLaunchKernelGGL(rt_math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, fn, a, b, out, n);
    return hipGetLastError();
}

// --------------------------------------------------------------- launchers
template <bool kCount, bool kProf, int kWidth, int kFeat, int kLds>
static hipError_t launch_one(const RtKernelArgs *a, int grid, hipStream_t stream) {
    auto *k = rt_megakernel<kCount, kProf, kWidth, kFeat, kLds>;
    size_t dyn = 0;
    if (kLds == 1) {
        // the variant's node layout (rt_megakernel's kSplit): dword planes need 56 KiB, float4 planes 64
        dyn = lds_node_bytes<rt_lds_split(kLds, kFeat, kWidth)>() + RT_LDS_STACK_BYTES(a->stack_depth);
        // Dynamic LDS above the default limit: the attribute (the most any scene can
        // ask for) is set once per device and variant, recorded in an atomic bit mask
        // (thread-safe; calling hipFuncSetAttribute before every launch cost ~0.6 ms
        // of host time per render step).
        static std::atomic<uint64_t> done{0};
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        const uint64_t bit = 1ull << (dev & 63);
        if (!(done.load(std::memory_order_acquire) & bit)) {
            // the most the budget leaves beside this variant's own static arrays
            hipFuncAttributes fa;
            e = hipFuncGetAttributes(&fa, (const void *)k);
            if (e != hipSuccess) return e;
            e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    RT_LDS_BUDGET - (int)fa.sharedSizeBytes);
            if (e != hipSuccess) return e;
            done.fetch_or(bit, std::memory_order_release);
        }
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kLds == 1 ? RT_LDS_BLOCK : RT_BLOCK), dyn, stream, *a);
    return hipGetLastError();
}

template <int kWidth, int kFeat, int kLds>
static hipError_t launch_variant(const RtKernelArgs *a, int grid, int mode, hipStream_t stream) {
    if (mode == 1) return launch_one<true, false, kWidth, kFeat, kLds>(a, grid, stream);
    if (mode == 2) return launch_one<false, true, kWidth, kFeat, kLds>(a, grid, stream);
    return launch_one<false, false, kWidth, kFeat, kLds>(a, grid, stream);
}

// The compiled variant that runs a scene's features (launch_features below).
static int variant_of(int features) {
    switch (features) {
    case 0:
    case RT_FEAT_MEDIA: return RT_FEAT_MEDIA;
    case RT_FEAT_INST: return RT_FEAT_INST;
    case RT_FEAT_INST | RT_FEAT_MEDIA: return RT_FEAT_INST | RT_FEAT_MEDIA;
    case RT_FEAT_CHECKER:
    case RT_FEAT_CHECKER | RT_FEAT_PRESCAN: return RT_FEAT_CHECKER | RT_FEAT_PRESCAN;
    default: return RT_FEAT_ALL;
    }
}

template <int kLds>
static hipError_t launch_features(const RtKernelArgs *a, int grid, int mode, hipStream_t stream) {
    switch (a->features) {
    case 0:
    case RT_FEAT_MEDIA: return launch_variant<2, RT_FEAT_MEDIA, kLds>(a, grid, mode, stream);
    case RT_FEAT_INST: return launch_variant<2, RT_FEAT_INST, kLds>(a, grid, mode, stream);
    case RT_FEAT_INST | RT_FEAT_MEDIA: return launch_variant<2, RT_FEAT_INST | RT_FEAT_MEDIA, kLds>(a, grid, mode, stream);
    case RT_FEAT_CHECKER:
    case RT_FEAT_CHECKER | RT_FEAT_PRESCAN:
        return launch_variant<2, RT_FEAT_CHECKER | RT_FEAT_PRESCAN, kLds>(a, grid, mode, stream);
    default: return launch_variant<2, RT_FEAT_ALL, kLds>(a, grid, mode, stream);
    }
}

// Compiled variants: every feature (any scene), media only (final(), and scenes with
// no feature), instances (cornell_box), instances + media (cornell_smoke), checker +
// pre-scan without media (the random scenes), each with the BVH2 in HBM or in LDS; the
// wide BVHs (4, 8, compressed 8) run the all-feature variant from HBM.
extern "C" hipError_t rt_launch_megakernel(const RtKernelArgs *a, int grid, int mode, hipStream_t stream) {
    if (a->scan) return launch_features<2>(a, grid, mode, stream);
    if (a->bvh_width == 4) return launch_variant<4, RT_FEAT_ALL, 0>(a, grid, mode, stream);
    if (a->bvh_width == 8) return launch_variant<8, RT_FEAT_ALL, 0>(a, grid, mode, stream);
    if (a->bvh_width == RT_BVH_CW8) return launch_variant<RT_BVH_CW8, RT_FEAT_ALL, 0>(a, grid, mode, stream);
    return a->lds_nodes ? launch_features<1>(a, grid, mode, stream) : launch_features<0>(a, grid, mode, stream);
}

extern "C" int rt_slab_floats(void) { return RT_SLAB_FLOATS; }

extern "C" hipError_t rt_launch_resolve(const float *slab, uint32_t npix, int nchunks, float k, float4 *acc, int mode,
                                        const uint32_t *out_index, float *out, hipStream_t stream) {
    int blocks = (int)((npix + 255) / 256);
    hipLaunchKernelGGL(rt_resolve, dim3(blocks), dim3(256), 0, stream, slab, npix, nchunks, k, acc, mode, out_index, out);
    return hipGetLastError();
}

template <int kWidth, int kMode>
static hipError_t occupancy_width(int *blocks_per_cu, int mode) {
    if (mode == 1)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_megakernel<true, false, kWidth, RT_FEAT_ALL, kMode>, RT_BLOCK, 0);
    if (mode == 2)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_megakernel<false, true, kWidth, RT_FEAT_ALL, kMode>, RT_BLOCK, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_megakernel<false, false, kWidth, RT_FEAT_ALL, kMode>, RT_BLOCK, 0);
}

extern "C" hipError_t rt_megakernel_occupancy(int *blocks_per_cu, int mode, int width) {
    if (width == 0) return occupancy_width<2, 2>(blocks_per_cu, mode);
    if (width == 8) return occupancy_width<8, 0>(blocks_per_cu, mode);
    if (width == RT_BVH_CW8) return occupancy_width<RT_BVH_CW8, 0>(blocks_per_cu, mode);
    return width == 4 ? occupancy_width<4, 0>(blocks_per_cu, mode) : occupancy_width<2, 0>(blocks_per_cu, mode);
}

template <int kFeat>
static int lds_static_of() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void *)rt_megakernel<false, false, 2, kFeat, 1>) != hipSuccess) return 0;
    return (int)fa.sharedSizeBytes;
}
extern "C" int rt_megakernel_lds_static_actual(void) {
    return std::max(std::max(std::max(lds_static_of<RT_FEAT_MEDIA>(), lds_static_of<RT_FEAT_INST>()),
                             lds_static_of<RT_FEAT_INST | RT_FEAT_MEDIA>()),
                    std::max(lds_static_of<RT_FEAT_CHECKER | RT_FEAT_PRESCAN>(), lds_static_of<RT_FEAT_ALL>()));
}

// LDS bytes per workgroup the BVH2-in-LDS variant for `features` needs with stacks of
// `stack_depth` entries: its static arrays (the compiled kernel's own count, or the
// estimate below where no HIP device answers), its node layout (rt_lds_split: 56 KiB of
// dword planes for the media variants, 64 KiB of float4 planes otherwise) and the
// stacks — what launch_one asks for, so the host's eligibility check and the launch agree.
extern "C" int rt_megakernel_lds_static_bytes(void);
extern "C" long rt_lds_need_bytes(int features, int stack_depth) {
    const int v = variant_of(features);
    int stat = 0;
    switch (v) {
    case RT_FEAT_MEDIA: stat = lds_static_of<RT_FEAT_MEDIA>(); break;
    case RT_FEAT_INST: stat = lds_static_of<RT_FEAT_INST>(); break;
    case RT_FEAT_INST | RT_FEAT_MEDIA: stat = lds_static_of<RT_FEAT_INST | RT_FEAT_MEDIA>(); break;
    case RT_FEAT_CHECKER | RT_FEAT_PRESCAN: stat = lds_static_of<RT_FEAT_CHECKER | RT_FEAT_PRESCAN>(); break;
    default: stat = lds_static_of<RT_FEAT_ALL>(); break;
    }
    // (the ball waves' path pools and Perlin's tables: final()'s variant only, rt_megakernel kBall)
    stat = std::max(stat, rt_megakernel_lds_static_bytes() +
                              (v == RT_FEAT_MEDIA ? (RT_BALL_POOL + RT_NORM_POOL - 2) * 80 + 255 * 16 + 767 * 4 : 0));
    const long nodes = rt_lds_split(1, v, 2) ? lds_node_bytes<1>() : lds_node_bytes<0>();
    return (long)stat + nodes + (long)RT_LDS_STACK_BYTES((long)stack_depth);
}

// the LDS variant's static arrays: stack placeholder, cooperative slots, media, camera
extern "C" int rt_megakernel_lds_static_bytes(void) {
    return (int)(4 * 64 + (RT_LDS_BLOCK / 64) * 64 * sizeof(CoopSlot) + RT_LDS_MEDIA * sizeof(MediumRec) + 6 * 16 + 16 +
                 (RT_LDS_BLOCK / 64) * RT_PRE * (8 + 8 + 8) + RT_LCG_JUMPS * 16 + 2 * 80 + 16 + 16 + 4) + 256;
}
#endif  // RT_KNOB_CHECK
