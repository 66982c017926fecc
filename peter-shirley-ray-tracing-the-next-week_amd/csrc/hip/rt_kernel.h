// rt_kernel.h — launch interface between the host runtime (capi.cpp) and the
// megakernel (rt_kernel.hip).  Internal to librt_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RT_BLOCK 256      // 4 waves per workgroup (BVH in HBM: 4 workgroups per CU)

// LDS-resident BVH2 (RtKernelArgs.lds_nodes): one workgroup of 16 waves per CU holds
// the scene's nodes in LDS as 4 planes of RT_LDS_NODE_CAP float4, beside the waves'
// traversal stacks (RtKernelArgs.stack_depth entries per lane).
#define RT_LDS_BLOCK 1024
#define RT_LDS_NODE_CAP 1024
#define RT_LDS_NODE_BYTES (4 * RT_LDS_NODE_CAP * 16)
#define RT_LDS_NODE_BYTES_MEDIA (14 * RT_LDS_NODE_CAP * 4)   // the media variants' dword planes (rt_device.h RtSplit)
#define RT_LDS_STACK_BYTES(depth) ((RT_LDS_BLOCK / 64) * (depth) * 64 * 2)   // 16-bit entries (rt_device.h stk16_*)
#define RT_LDS_MAX_PRIMS 4096   // leaf references of the LDS copy hold 12-bit first primitives
#define RT_LDS_BUDGET 163840   // LDS bytes per CU (160 KiB)

// scene features a megakernel variant carries code for (rt_launch_megakernel)
#define RT_FEAT_INST 1      // translate / rotate_y / flip_normals chains
#define RT_FEAT_UV 2        // a material reads (u, v): image_texture
#define RT_FEAT_CHECKER 4   // checker_texture
#define RT_FEAT_PRESCAN 8   // BVH scene with pre-scanned primitives (RtKernelArgs.nprescan > 0)
#define RT_FEAT_MEDIA 16    // constant_medium (without it: no media stage, no medium-stream key per sample)
#define RT_FEAT_ALL 31

#define RT_WAVE_LOG_WORDS 12

struct RtKernelArgs {
    // scene (HBM, 16-B records; see rt_layout.h)
    const float4 *nodes;    // BVH nodes, breadth-first: 4 / 8 / 16 / 8 x float4 (width 2 / 4 / 8 / RT_BVH_CW8)
    const float4 *prims;    // 4 x float4 per surface primitive (leaf order)
    const float4 *bprims;   // 4 x float4 per media-boundary primitive
    const int4 *media;      // 1 x int4 per medium
    const float4 *mats;     // 2 x float4 per material
    const float4 *texs;     // 2 x float4 per texture
    const float4 *insts;    // 7 x float4 per instance chain
    const float4 *ranvec;   // 256 Perlin gradients (w unused)
    const int *perm;        // 3 x 256 Perlin permutations
    const uint8_t *texels;  // image_texture bytes
    uint32_t root;
    uint32_t nnodes;
    int bvh_width;          // 2, 4, 8 or RT_BVH_CW8 (compressed 8-wide)
    int has_bvh;
    int nmedia;
    int features;           // RT_FEAT_* present in the scene (selects the megakernel variant)
    int need_dlen;          // |r.d| is used: media, metal / dielectric materials or the sky
    const float4 *groups;   // flat scan: 3 x float4 per group (rt_dgroup)
    int ngroups;
    int scan;               // 1: flat scan of the groups instead of a BVH (small scenes, rt_layout.h)
    uint32_t nprims;        // surface primitives (flat scan: all copied to LDS)
    int nprescan;           // BVH modes: primitives [0, nprescan) are outside the BVH, tested first in lockstep
    int cell_first, cell_n;   // BVH modes: the medium cell's primitive copies [cell_first, cell_first + cell_n) ...
    float cell_c[3], cell_r2; //     ... and its ball (centre, squared radius): capi.cpp rt_scene_create ...
    float cell_rin2;          //     ... and the squared radius inside which a ray counts as inside whatever its direction
    int ball_waves;           // waves per workgroup that take the medium cell's paths first (LDS media variant) ...
    int ball_batch;           //     ... their ready batch (the others': RT_READY_BATCH) ...
    int ball_claim;           //     ... and the busy lanes below which they claim new samples ...
    int ball_park;            //     ... and whether their segments the cell does not decide move to normal waves
    int ball_drain;           //     ... and whether, with the claims exhausted, normal waves leave the ball's pool to them
    int lds_nodes;          // 1: BVH2 nodes copied to LDS (RT_LDS_BLOCK workgroups, one per CU)
    int stack_depth;        // traversal stack entries per lane of the LDS variant (BVH depth + 1)
    // camera (camera.h members)
    float org[3], llc[3], hor[3], ver[3], cu[3], cv[3];
    float lens, ct0, ct1;
    // render parameters
    int nx, ny, ns, max_depth;
    float rnx, rny;           // RN(1/float(nx)), RN(1/float(ny)): the camera's divisions by div_rn
    float tmin;
    int background;
    int chunk, nchunks;       // samples per work item; work items per pixel in this launch
    uint32_t sample_offset;   // sample index of this launch's first sample (batches: + batch start)
    uint64_t seed;
    // job: pixel list and outputs
    const uint32_t *job_xy;   // x | y << 16 per job pixel (image coords)
    uint32_t npix;
    uint32_t nitems;          // npix * nchunks
    uint32_t ndeep;           // the job's first ndeep pixels are claimed first, all their chunks ...
    uint32_t ndeep_items;     // ... (ndeep * nchunks items), then the other pixels' (capi.cpp prepare_job)
    uint32_t claim;           // work items per wave-level claim (a multiple of 64) ...
    uint32_t nbig;            // ... for the first nbig claims; the rest (the launch's tail) claim
    uint32_t claim_tail;      //     claim_tail items each, so that waves run dry together
    float *slab;              // [nchunks][npix] partial sums (rgb, rt_slab_floats() floats each) of this batch
    uint32_t *counter;        // work-claim counter (zeroed per launch)
    unsigned long long *stats;  // RT_CNT_N counters (count variant)
    // profile variant, RTNW_WAVE_LOG: RT_WAVE_LOG_WORDS per wave (start, dry, end, hw id, items,
    // iterations after dry, live lanes summed over them, paths taken from the pools after dry,
    // the stage cycles after dry: claim, traverse, media, shade)
    unsigned long long *wave_log;
};

extern "C" hipError_t rt_launch_megakernel(const RtKernelArgs *a, int grid, int mode, hipStream_t stream);
// Resolve of one sample batch (capi.cpp): adds the batch's partial sums to each
// pixel's running sum in sample order.  mode: RT_RESOLVE_* bits.
#define RT_RESOLVE_FIRST 1    // the first batch: start from 0 (or, with SUM_IN, from out)
#define RT_RESOLVE_LAST 2     // the last batch: write out (times k unless RAW), else keep acc
#define RT_RESOLVE_SUM_IN 4   // out holds the running sums of earlier samples on entry
#define RT_RESOLVE_RAW 8      // write the sums themselves (checkpoints), not sum * k
// floats per partial sum in the slab (3: rgb; RT_SLAB_F4=1 builds the 16-B layout, A/B only)
extern "C" int rt_slab_floats(void);
extern "C" hipError_t rt_launch_math_probe(int fn, const float *a, const float *b, float *out, int n, hipStream_t stream);
extern "C" hipError_t rt_launch_resolve(const float *slab, uint32_t npix, int nchunks, float k, float4 *acc, int mode,
                                        const uint32_t *out_index, float *out, hipStream_t stream);
// mode: 0 plain, 1 count, 2 profile; width: the scene's RtKernelArgs.bvh_width, 0: the flat-scan kernel
extern "C" hipError_t rt_megakernel_occupancy(int *blocks_per_cu, int mode, int width);
// Static LDS bytes of the LDS-BVH variant (its dynamic part: nodes + stacks).
extern "C" int rt_megakernel_lds_static_bytes(void);
// the largest static LDS (bytes) the compiler gave any LDS-BVH variant (hipFuncGetAttributes), 0 if unknown
extern "C" int rt_megakernel_lds_static_actual(void);
// LDS bytes per workgroup of the BVH2-in-LDS variant a scene with `features` (RT_FEAT_*)
// runs, with traversal stacks of `stack_depth` entries (rt_kernel.hip)
extern "C" long rt_lds_need_bytes(int features, int stack_depth);
