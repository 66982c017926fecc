// bvh.h — host BVH builder (see bvh.cpp).
#pragma once
#include <cstdint>
#include <vector>

#include "rt_hip.h"
#include "../rt_layout.h"

namespace rtnw {

struct BvhResult {
    int width = 2;                 // 2: rt_dnode2, 4: rt_dnode4 (rt_layout.h)
    std::vector<rt_dnode2> nodes2;
    std::vector<rt_dnode4> nodes4;
    std::vector<int> order;   // leaf order -> index into the input primitives
    uint32_t root = 0;
    int depth = 0;            // binary-build internal nodes on the longest root-to-leaf path
};

// Primitive boxes cover moving spheres over [min(0, time0), max(0, time1)].
// width: 2 or 4 (RTNW_BVH_WIDTH overrides).
BvhResult build_bvh(const rt_prim *prims, int n, const rt_instance *instances, float time0, float time1);

// World-space box of one primitive over the shutter span [min(0, time0), max(0, time1)],
// padded like the BVH's boxes and rounded outward to float.
void prim_bounds(const rt_prim &p, const rt_instance *instances, float time0, float time1, float lo[3], float hi[3]);

}  // namespace rtnw
