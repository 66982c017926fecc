// rt_layout.h — the scene's layout in HBM, shared by the host uploader
// (capi.cpp) and the megakernel (rt_kernel.hip).
//
// Everything the traversal touches is a 16-byte-aligned record read with
// dwordx4 loads: an incoherent wave fetches one whole record per lane per
// cache line instead of gathering scattered scalars.  Records are grouped by
// role (nodes / primitives / boundary primitives / materials / textures /
// instances / Perlin tables) in separate arrays.
#pragma once
#include <stdint.h>

#include "rt_hip.h"   // enum values (prim / material / texture kinds, ops)

#define RT_STACK_DEPTH 24          // traversal stack entries per lane (LDS)
#define RT_STACK_DEPTH_W8 32       // the same for the 8-wide BVHs (up to 7 pushes per node)
#define RT_MAX_BVH_DEPTH 23        // builder guarantee: a root-to-leaf path has <= 23 internal nodes
                                   // (a median split of 2^24 - 1 primitives, the ABI maximum, fits)
#define RT_MAX_LEAF 8              // primitives per leaf
#define RT_MAX_INSTANCE_OPS 6
#define RT_MAX_CHECKER_DEPTH 16

// Child reference in a node: bit 31 set = leaf, bits 24..30 = count-1, bits 0..23 = first prim.
#define RT_LEAF_BIT 0x80000000u
#define RT_EMPTY_CHILD 0xFFFFFFFFu
#define RT_LEAF_REF(first, count) (RT_LEAF_BIT | ((uint32_t)((count) - 1) << 24) | (uint32_t)(first))
#define RT_LEAF_FIRST(ref) ((ref) & 0x00FFFFFFu)
#define RT_LEAF_COUNT(ref) ((((ref) >> 24) & 0x7Fu) + 1)

// The BVH comes in four node forms (RTNW_BVH_WIDTH = 2 (default), 4, 8, 8q), nodes
// numbered breadth-first so the top levels are a prefix of the array (kept in LDS).
//
// BVH2 node, 64 B: the boxes of BOTH children, so one node fetch decides which
// children to enter:
//   b0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//   b1 = (c0.lo.z, c0.hi.z, c1.lo.x, c1.hi.x)
//   b2 = (c1.lo.y, c1.hi.y, c1.lo.z, c1.hi.z)
//   ch = (child0, child1, -, -)
struct rt_dnode2 {
    float b[3][4];
    uint32_t ch[4];
};

// BVH4 node, 128 B: the boxes of up to four children.  Each axis interval is a
// (lo, hi) pair and a float4 holds the pairs of two children, so one packed FMA
// yields both slab distances of a pair:
//   q[0] = x of c0, c1   q[1] = x of c2, c3
//   q[2] = y of c0, c1   q[3] = y of c2, c3
//   q[4] = z of c0, c1   q[5] = z of c2, c3      each (lo, hi, lo, hi)
//   ch   = child references (RT_EMPTY_CHILD: unused slot)
//   pad  = keeps nodes on 128-B lines; never read
// Builder guarantee (every width): along any root-to-leaf path the children
// beyond the first sum to <= RT_STACK_DEPTH - 1 (8-wide: RT_STACK_DEPTH_W8 - 1),
// which bounds the traversal stack.
struct rt_dnode4 {
    float q[6][4];
    uint32_t ch[4];
    uint32_t pad[4];
};

// BVH8 node (RTNW_BVH_WIDTH=8), 256 B: as BVH4 with four pairs per axis,
//   q[4a + p] = axis a of children 2p, 2p+1, (lo, hi, lo, hi);  ch = 8 references.
struct rt_dnode8 {
    float q[12][4];
    uint32_t ch[8];
    uint32_t pad[8];
};

// Compressed BVH8 node (RTNW_BVH_WIDTH=8q), 128 B: child boxes quantised to 8 bits
// per plane on a per-axis power-of-two grid anchored at the node's box (Ylitie et
// al., "Efficient incoherent ray traversal on GPUs through compressed wide BVHs",
// HPG 2017).  Plane k of child c on axis a lies at origin[a] + q * 2^(e[a] - 127),
// quantised outward (lo floored, hi ceiled), so the decoded box contains the child.
//   origin, ebits = e_x | e_y << 8 | e_z << 16
//   qa[a] = axis a: bytes of lo c0..c3, lo c4..c7, hi c0..c3, hi c4..c7
//   ch = 8 references;  pad keeps 128-B lines
#define RT_BVH_CW8 9               // RtKernelArgs.bvh_width of the compressed 8-wide layout
struct rt_dnode8q {
    float origin[3];
    uint32_t ebits;
    uint32_t qa[3][4];
    uint32_t ch[8];
    uint32_t pad[8];
};

// Primitive, 64 B, ordered so the first 32 B (g0, m) are all a sphere or rect test
// reads; only a moving sphere reads the whole record.  g0..g2 by kind:
//   sphere:        g0 = (cx, cy, cz, r)
//   moving sphere: g0 = (c0x, c0y, c0z, r), g1 = (c1x-c0x, c1y-c0y, c1z-c0z, t0), g2 = (t1-t0, ...)
//   rects:         g0 = (a0, a1, b0, b1)
// m = (kind | flip << 8 | material << 9, rect k (float bits), instance (-1 none), list order)
struct rt_dprim {
    float g0[4];
    int32_t m[4];
    float g1[4], g2[4];
};

// Flat scan (scenes of at most RT_SCAN_MAX surface primitives, capi.cpp): the
// primitives are ordered by instance chain, and each run of one chain is a group,
// 48 B: (first, count, instance (-1 none), kinds) + its world box as in a BVH node,
// (lo.x, hi.x, lo.y, hi.y), (lo.z, hi.z, n_yz, -).  Within a group the primitives
// are ordered by kind (list order within a kind): kinds = n_sphere | n_moving << 8 |
// n_xy << 16 | n_xz << 24, then n_yz yz rects.  A wave tests every group's box
// against all its rays at once, transforms its rays into the group's object space
// ONCE, and tests the group's primitives in lockstep (every lane the same one), one
// loop per kind: the instance level of a two-level structure, without per-leaf
// transforms or per-primitive kind branches.
#define RT_SCAN_MAX 64
// BVH scenes: at most this many of the largest primitives are pre-scanned (capi.cpp).
#define RT_PRESCAN_MAX 8
// The medium cell: at most this many primitives near a dense medium's ball (capi.cpp).
#define RT_CELL_MAX 4
struct rt_dgroup {
    int32_t first, count, instance, kinds;
    float bx[4], bz[2];
    int32_t nyz, pad;
};

// Material, 32 B: (kind, texture, fuzz, ref_idx) + (albedo.xyz, flags).  A dielectric
// carries (float)(1.0/(double)ref_idx), schlick r0^2 and ref_idx^2 in albedo (capi.cpp).
// flags: 1 a texture of the material reads (u, v); 2 its texture is a constant whose
// color is in albedo (textured kinds only: capi.cpp)
struct rt_dmaterial {
    int32_t kind, texture;
    float fuzz, ref_idx;
    float albedo[3];
    int32_t flags;
};

// Texture, 32 B: (kind, even, odd, scale) + (color.xyz, -)
struct rt_dtexture {
    int32_t kind, even, odd;
    float scale;
    float color[3];
    int32_t pad;
};

// Instance transform chain, 112 B: (nops, -, -, -) + 6 x (op, a, b, c), outermost first.
struct rt_dinstance {
    int32_t nops, pad[3];
    float ops[RT_MAX_INSTANCE_OPS][4];
};

// Medium, 16 B: (boundary_first, boundary_count, -(1/density), phase material).
// The float -(1/density) of constant_medium.h:36 is computed once on the host
// (IEEE division, the same value the device would get per ray).
struct rt_dmedium {
    int32_t first, count;
    float neg_inv_density;
    int32_t material;
};

// Counters of the RT_FLAG_COUNT kernel variant (uint64 each).
enum {
    RT_CNT_SAMPLES = 0, RT_CNT_SEGMENTS, RT_CNT_NODES, RT_CNT_SPHERES, RT_CNT_MSPHERES, RT_CNT_RECTS,
    RT_CNT_INSTANCED, RT_CNT_MEDIA, RT_CNT_SHADES, RT_CNT_NOISE, RT_CNT_N
};
// The rest of the stats buffer (uint64 slots after the RT_CNT_N counters): stage
// cycles (RT_FLAG_PROFILE), wave-level trip counts (RT_FLAG_COUNT), the wave
// timeline (RT_FLAG_PROFILE), the shading-stage material divergence (RT_FLAG_COUNT:
// wave shade passes, distinct scatter materials summed over them, scattering lanes;
// RT_FLAG_PROFILE: cycles in the material scatter branches).
enum {
    RT_STAT_PROF = RT_CNT_N, RT_STAT_WAVE = RT_CNT_N + 4, RT_STAT_TIME = RT_CNT_N + 9, RT_STAT_SHADE = RT_CNT_N + 16,
    RT_STAT_BALL = RT_CNT_N + 20,   // RT_FLAG_COUNT, the ball waves (rt_kernel.hip stage 6): RT_BALL_*
    RT_STATS_LEN = RT_CNT_N + 28
};
// ball-wave counters: ball-wave iterations, their live lanes and traversal rounds summed over
// them, segments the medium cell decided (in ball waves), paths a normal wave could not push
// (the ball's pool full), paths pushed into the ball's pool / the others' pool, paths taken
enum { RT_BALL_ITERS = 0, RT_BALL_LIVE, RT_BALL_ROUNDS, RT_BALL_CELL_BALL, RT_BALL_DENIED, RT_BALL_PUSH_IN,
       RT_BALL_PUSH_OUT, RT_BALL_TAKEN, RT_BALL_N };
