// rt_wavefront.hip — the workgroup-wavefront engine (RTNW_ENGINE=wave).
//
// Same hot path and the same arithmetic as the megakernel (rt_kernel.hip; the
// shared device code is rt_device.h), organised differently.  A persistent
// workgroup owns RT_WF_SLOTS camera paths whose state lives in HBM (SoA, one
// record per slot; the working set of a workgroup is ~50 KB and stays in L2 /
// MALL).  Each wave owns a quarter of the slots and runs three compacted phases
// on them in turn, with wave-local lists and no workgroup barriers (a wave in the
// tail of a phase idles only its own lanes; the SIMD's other waves keep issuing):
//
//   C  camera   slots whose path ended: retire / claim work items, draw the next
//               camera sample (camera.h:41-56) -> ray
//   T  trace    slots with a ray: closest hit through the BVH; lanes fetch the
//               next ray of the wave's list as they finish, so they stay busy
//               until the list runs dry (persistent while-while)
//   S  shade    slots with a hit: media, hit record, material scatter -> the
//               next ray, or the path's radiance added to the item's sum
//
// In the megakernel every stage runs inside one wave whose lanes are at
// different stages, so each stage executes with only part of the wave active
// and all path state is live in registers across all of them.  Here each phase
// runs its own code over a compacted list with the whole wave, and only that
// phase's registers are live.
//
// Determinism and parity are those of the megakernel: a slot processes its work
// item's samples in order, each sample draws from its own counter stream, and
// an item's sum goes to the partial-sum slab exactly once.
#include "rt_device.h"

#ifndef RT_WF_WAVES_PER_SIMD
#define RT_WF_WAVES_PER_SIMD 4
#endif

namespace {

constexpr int kWfSlots = RT_WF_SLOTS;                   // path slots per workgroup
constexpr int kWaveSlots = kWfSlots / (RT_BLOCK / 64);   // ... per wave
static_assert(kWaveSlots % 64 == 0, "slots per wave must be a multiple of 64");

enum : uint32_t { ST_EMPTY = 0, ST_CAMERA = 1, ST_TRACE = 2, ST_HIT = 3 };
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Orders this wave's LDS writes before its later LDS reads by other lanes.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The wave's slots of one status, compacted into `list` (slot order); returns
// the count (wave-uniform).
__device__ __forceinline__ uint32_t build_list(const uint8_t *status, uint32_t want, uint16_t *list, uint32_t lane) {
    wave_sync();
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < kWaveSlots / 64; ++k) {
        const uint32_t slot = k * 64 + lane;
        const bool mine = status[slot] == want;
        const uint64_t m = __ballot(mine);
        if (mine) list[n + lanes_below(m)] = (uint16_t)slot;
        n += (uint32_t)__popcll(m);
    }
    wave_sync();
    return n;
}

// kProf: wave-level s_memtime per phase (RT_FLAG_PROFILE; stats cycles_claim =
// phase C, cycles_traverse = phase T, cycles_media = phase S, cycles_shade =
// list building).  Diagnostic only.
template <bool kCount, bool kProf, int kWidth>
__global__ __launch_bounds__(RT_BLOCK, RT_WF_WAVES_PER_SIMD) void rt_wavefront(RtKernelArgs A) {
    __shared__ uint32_t lds_stack[RT_BLOCK / 64][RT_STACK_DEPTH][64];
    __shared__ CoopSlot lds_slots[RT_BLOCK / 64][64];
    __shared__ MediumRec lds_media[RT_LDS_MEDIA];
    __shared__ uint16_t lds_list[RT_BLOCK / 64][kWaveSlots];
    __shared__ uint8_t lds_status[RT_BLOCK / 64][kWaveSlots];

    const uint32_t lane = lane_id();
    uint32_t *stk = &lds_stack[threadIdx.x >> 6][0][lane];
    CoopSlot *slots = lds_slots[threadIdx.x >> 6];
    uint16_t *list = lds_list[threadIdx.x >> 6];
    uint8_t *status = lds_status[threadIdx.x >> 6];
    const size_t sbase = (size_t)blockIdx.x * kWfSlots + (threadIdx.x >> 6) * kWaveSlots;
    Counters cnt;
    uint64_t prof[4] = {0, 0, 0, 0};
    uint64_t stamp = kProf ? __builtin_amdgcn_s_memtime() : 0;
    auto mark = [&](int k) {
        if (kProf) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            prof[k] += now - stamp;
            stamp = now;
        }
    };

    const uint64_t skey = seed_key(A.seed);   // per-launch part of the sample keys
    // wave-uniform work-item pool (one global atomic per 64 items)
    uint32_t pool_next = 0, pool_end = 0;
    bool exhausted = false;

    load_media(A, lds_media);
    __syncthreads();
    for (int k = 0; k < kWaveSlots / 64; ++k) {
        const uint32_t slot = k * 64 + lane;
        status[slot] = ST_CAMERA;
        A.wf_samp[sbase + slot] = make_uint4(kNone, 0, 0, 0);   // item, s_cur, s_end, -
    }

    for (;;) {
        // ---- C: retire finished items, claim new ones, camera samples -------------
        mark(3);
        const uint32_t nc = build_list(status, ST_CAMERA, list, lane);
        mark(3);
        for (uint32_t b = 0; b < nc; b += 64) {
            const uint32_t i = b + lane;
            const uint32_t slot = i < nc ? list[i] : 0;
            const size_t gs = sbase + slot;
            uint4 sm = make_uint4(kNone, 0, 0, 0);
            float4 pt = make_float4(0, 0, 0, 0);
            bool need = false;
            if (i < nc) {
                sm = A.wf_samp[gs];
                if (sm.y == sm.z) {   // item done (or none yet): its sum to the slab
                    if (sm.x != kNone) A.slab[sm.x] = A.wf_part[gs];
                    need = true;
                } else {
                    pt = A.wf_part[gs];
                }
            }
            // claim: the lanes that need an item share the wave's pool
            uint64_t need_mask = __ballot(need);
            while (need_mask != 0ull && !exhausted) {
                if (pool_next == pool_end) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(A.counter, A.claim);
                    base = __shfl(base, 0);
                    if (base >= A.nitems) { exhausted = true; break; }
                    pool_next = base;
                    pool_end = min(base + A.claim, A.nitems);
                }
                const uint32_t avail = pool_end - pool_next;
                const uint32_t rank = lanes_below(need_mask);
                if (need && rank < avail) {
                    const uint32_t item = pool_next + rank;
                    const uint32_t c = item / A.npix;
                    sm.x = item;
                    sm.y = c * (uint32_t)A.chunk;
                    sm.z = min(sm.y + (uint32_t)A.chunk, (uint32_t)A.ns);
                    pt = make_float4(0, 0, 0, 0);
                    need = false;
                }
                pool_next += min((uint32_t)__popcll(need_mask), avail);
                need_mask = __ballot(need);
            }
            const bool starting = i < nc && !need;
            if (i < nc && need) status[slot] = ST_EMPTY;   // no work left for this slot
            // camera sample (main.cpp:305-308, camera.h:41-56)
            Rng g;
            g.ctr = 0;
            g.mkey = 0;
            float cu_ = 0, cv_ = 0;
            uint32_t px = 0;
            int j = 0;
            if (starting) {
                const uint32_t xy = A.job_xy[sm.x - (sm.x / A.npix) * A.npix];
                px = xy & 0xFFFFu;
                j = A.ny - 1 - (int)(xy >> 16);
                g.start(sample_key(skey, (uint32_t)(j * A.nx + (int)px), sm.y + A.sample_offset));
                cu_ = (float)((double)(int)px + g.next()) / (float)A.nx;
                cv_ = (float)((double)j + g.next()) / (float)A.ny;
            }
            const V3 disk = coop_reject<2, kCount>(starting, g, slots, lane, cnt, DiskCand());
            if (starting) {
                V3 rd = scale(A.lens, disk);
                V3 cu = mk(A.cu[0], A.cu[1], A.cu[2]), cv = mk(A.cv[0], A.cv[1], A.cv[2]);
                V3 offset = add(scale(rd.x, cu), scale(rd.y, cv));
                float time = (float)((double)A.ct0 + g.next() * (double)(A.ct1 - A.ct0));
                V3 org = mk(A.org[0], A.org[1], A.org[2]);
                V3 dir = sub(sub(add(add(mk(A.llc[0], A.llc[1], A.llc[2]), scale(cu_, mk(A.hor[0], A.hor[1], A.hor[2]))),
                                     scale(cv_, mk(A.ver[0], A.ver[1], A.ver[2]))), org), offset);
                const V3 o = add(org, offset);
                A.wf_ray_o[sbase + slot] = make_float4(o.x, o.y, o.z, time);
                A.wf_ray_d[sbase + slot] = make_float4(dir.x, dir.y, dir.z, 0.f);
                A.wf_beta[sbase + slot] = make_float4(1.f, 1.f, 1.f, __int_as_float(0));
                A.wf_rng[sbase + slot] = make_uint4((uint32_t)g.ctr, (uint32_t)(g.ctr >> 32), (uint32_t)g.mkey,
                                                    (uint32_t)(g.mkey >> 32));
                A.wf_part[sbase + slot] = pt;
                A.wf_samp[sbase + slot] = sm;
                status[slot] = ST_TRACE;
                if (kCount) { cnt.samples++; cnt.segments++; }
            }
        }
        mark(0);

        // ---- T: closest surface hits -------------------------------------------
        const uint32_t nt = build_list(status, ST_TRACE, list, lane);
        if (nt == 0) break;   // every slot of the wave is empty: its share of the job is done
        mark(3);
        {
            uint32_t slot = kNone;
            uint32_t next = 0;   // wave-uniform position in the list
            bool dry = false;
            Ray r;
            r.o = mk(0, 0, 0); r.d = mk(0, 0, 0); r.time = 0;
            Slab sl = make_slab(r, A.tmin);
            uint32_t node = 0;
            int sp = 0;
            float best_t = RT_FLT_MAX;
            int best_key = 0x7FFFFFFF;
            uint32_t best_prim = kNone;
            for (;;) {
                // lanes without a ray take the next ones from the workgroup's list
                const bool idle = slot == kNone;
                const uint64_t idle_mask = __ballot(idle);
                if (idle_mask != 0ull && !dry) {
                    const uint32_t base = next;
                    next += (uint32_t)__popcll(idle_mask);
                    if (base >= nt) dry = true;
                    const uint32_t idx = base + lanes_below(idle_mask);
                    if (idle && idx < nt) {
                        slot = list[idx];
                        const float4 ro = A.wf_ray_o[sbase + slot], rdv = A.wf_ray_d[sbase + slot];
                        r.o = mk(ro.x, ro.y, ro.z);
                        r.d = mk(rdv.x, rdv.y, rdv.z);
                        r.time = ro.w;
                        sl = make_slab(r, A.tmin);
                        node = A.root;
                        sp = 0;
                        best_t = RT_FLT_MAX;
                        best_key = 0x7FFFFFFF;
                        best_prim = kNone;
                        if (!A.has_bvh) node = RT_EMPTY_CHILD;
                    }
                }
                if (__ballot(slot != kNone) == 0ull) break;
                if (slot != kNone) {
                    // one round: descend (speculatively past the first leaf) until all
                    // but RT_DESCEND_TAIL lanes hold a leaf, then test the leaves
                    const uint32_t pleaf = descend<kWidth, kCount>(A.nodes, node, sl, best_t, stk, sp, cnt);
                    if (pleaf != RT_EMPTY_CHILD) {
                        const uint32_t first = RT_LEAF_FIRST(pleaf), nleaf = RT_LEAF_COUNT(pleaf);
                        for (uint32_t q = 0; q < nleaf; q += 2) {
                            const uint32_t ia = first + q;
                            const bool two = q + 1 < nleaf;
                            const uint32_t ib = two ? ia + 1 : ia;
                            const float4 ga = A.prims[ia * 4 + 0], ma = A.prims[ia * 4 + 1];
                            const float4 gb = A.prims[ib * 4 + 0], mb = A.prims[ib * 4 + 1];
                            int key, kind;
                            float t = prim_t_head(ga, ma, A.prims, A.insts, ia, r, A.tmin, key, kind);
                            if (kCount) cnt.prim(kind);
                            if (t < best_t || (t == best_t && key < best_key)) {
                                best_t = t; best_key = key; best_prim = ia;
                            }
                            if (two) {
                                t = prim_t_head(gb, mb, A.prims, A.insts, ib, r, A.tmin, key, kind);
                                if (kCount) cnt.prim(kind);
                                if (t < best_t || (t == best_t && key < best_key)) {
                                    best_t = t; best_key = key; best_prim = ib;
                                }
                            }
                        }
                    }
                    if (node == RT_EMPTY_CHILD) {   // search over: hand the hit to phase S
                        A.wf_hit[sbase + slot] = make_float2(best_t, __uint_as_float(best_prim));
                        status[slot] = ST_HIT;
                        slot = kNone;
                    }
                }
            }
        }
        mark(1);

        // ---- S: media, hit record, material scatter ----------------------------
        const uint32_t ns = build_list(status, ST_HIT, list, lane);
        mark(3);
        for (uint32_t b = 0; b < ns; b += 64) {
            const uint32_t i = b + lane;
            const bool ready = i < ns;
            const uint32_t slot = ready ? list[i] : 0;
            const size_t gi = sbase + slot;
            Ray r;
            r.o = mk(0, 0, 0); r.d = mk(0, 0, 0); r.time = 0;
            float best_t = 0;
            uint32_t best_prim = kNone;
            V3 beta = mk(0, 0, 0);
            int depth = 0;
            Rng g;
            g.ctr = 0;
            g.mkey = 0;
            if (ready) {
                const float4 ro = A.wf_ray_o[gi], rdv = A.wf_ray_d[gi], bt = A.wf_beta[gi];
                const float2 h = A.wf_hit[gi];
                const uint4 rg = A.wf_rng[gi];
                r.o = mk(ro.x, ro.y, ro.z);
                r.d = mk(rdv.x, rdv.y, rdv.z);
                r.time = ro.w;
                best_t = h.x;
                best_prim = __float_as_uint(h.y);
                beta = mk(bt.x, bt.y, bt.z);
                depth = __float_as_int(bt.w);
                g.ctr = (uint64_t)rg.x | ((uint64_t)rg.y << 32);
                g.mkey = (uint64_t)rg.z | ((uint64_t)rg.w << 32);
            }
            // media after the surfaces (constant_medium.h:26-50), then the record
            const float dlen = (ready && A.need_dlen) ? len(r.d) : 0.f;
            bool have = false;
            Hit hr;
            hr.p = mk(0, 0, 0); hr.n = mk(0, 0, 0); hr.u = 0.f; hr.v = 0.f; hr.mat = 0;
            if (ready) {
                have = best_prim != kNone;
                const int med_mat = media_hit<kCount>(A, lds_media, r, dlen, depth, g, have, best_t, cnt);
                if (med_mat >= 0) {
                    hr.p = at(r, best_t);
                    hr.n = mk(1, 0, 0);
                    hr.mat = med_mat;   // constant_medium.h:41-44 leaves u, v stale; no medium texture reads them
                } else if (have) {
                    hr = prim_record(A.prims, A.insts, A.mats, best_prim, r, best_t);
                }
            }
            ShadeOut so = shade<kCount>(A, ready, have, r, dlen, hr, depth, g, slots, lane, cnt);
            if (ready) {
                if (so.scattered) {
                    beta = mul(beta, so.att);
                    A.wf_ray_o[gi] = make_float4(so.ray.o.x, so.ray.o.y, so.ray.o.z, so.ray.time);
                    A.wf_ray_d[gi] = make_float4(so.ray.d.x, so.ray.d.y, so.ray.d.z, 0.f);
                    A.wf_beta[gi] = make_float4(beta.x, beta.y, beta.z, __int_as_float(depth + 1));
                    A.wf_rng[gi] = make_uint4((uint32_t)g.ctr, (uint32_t)(g.ctr >> 32), (uint32_t)g.mkey,
                                              (uint32_t)(g.mkey >> 32));
                    status[slot] = ST_TRACE;
                    if (kCount) cnt.segments++;
                } else {
                    V3 L = mul(beta, so.emitted);
                    if (!(L.x == L.x)) L.x = 0;   // de_nan, main.cpp:232-242
                    if (!(L.y == L.y)) L.y = 0;
                    if (!(L.z == L.z)) L.z = 0;
                    float4 pt = A.wf_part[gi];
                    pt = make_float4(pt.x + L.x, pt.y + L.y, pt.z + L.z, 0.f);
                    A.wf_part[gi] = pt;
                    uint4 sm = A.wf_samp[gi];
                    sm.y += 1;
                    A.wf_samp[gi] = sm;
                    status[slot] = ST_CAMERA;
                }
            }
        }
        mark(2);
    }
    if (kProf && lane == 0)
        for (int k = 0; k < 4; ++k) atomicAdd(&A.stats[RT_CNT_N + k], (unsigned long long)prof[k]);

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

}  // namespace

template <int kWidth>
static hipError_t wf_launch_width(const RtKernelArgs *a, int grid, int mode, hipStream_t stream) {
    if (mode == 1)
        hipLaunchKernelGGL((rt_wavefront<true, false, kWidth>), dim3(grid), dim3(RT_BLOCK), 0, stream, *a);
    else if (mode == 2)
        hipLaunchKernelGGL((rt_wavefront<false, true, kWidth>), dim3(grid), dim3(RT_BLOCK), 0, stream, *a);
    else
        hipLaunchKernelGGL((rt_wavefront<false, false, kWidth>), dim3(grid), dim3(RT_BLOCK), 0, stream, *a);
    return hipGetLastError();
}

extern "C" hipError_t rt_launch_wavefront(const RtKernelArgs *a, int grid, int mode, hipStream_t stream) {
    return a->bvh_width == 4 ? wf_launch_width<4>(a, grid, mode, stream) : wf_launch_width<2>(a, grid, mode, stream);
}

template <int kWidth>
static hipError_t wf_occupancy_width(int *blocks_per_cu, int mode) {
    if (mode == 1)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_wavefront<true, false, kWidth>, RT_BLOCK, 0);
    if (mode == 2)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_wavefront<false, true, kWidth>, RT_BLOCK, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_wavefront<false, false, kWidth>, RT_BLOCK, 0);
}

extern "C" hipError_t rt_wavefront_occupancy(int *blocks_per_cu, int mode, int width) {
    return width == 4 ? wf_occupancy_width<4>(blocks_per_cu, mode) : wf_occupancy_width<2>(blocks_per_cu, mode);
}
