// bvh.h — host BVH builder (see bvh.cpp).
#pragma once
#include <cstdint>
#include <vector>

#include "rt_hip.h"
#include "../rt_layout.h"

namespace rtnw {

struct BvhResult {
    std::vector<rt_dnode> nodes;
    std::vector<int> order;   // leaf order -> index into the input primitives
    uint32_t root = 0;
    int depth = 0;            // internal nodes on the longest root-to-leaf path
};

// Primitive boxes cover moving spheres over [min(0, time0), max(0, time1)].
BvhResult build_bvh(const rt_prim *prims, int n, const rt_instance *instances, float time0, float time1);

}  // namespace rtnw
