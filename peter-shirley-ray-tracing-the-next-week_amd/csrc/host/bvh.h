// bvh.h — host BVH builder (see bvh.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "rt_hip.h"
#include "../rt_layout.h"

namespace rtnw {

struct BvhResult {
    int width = 2;                 // 2: rt_dnode2, 4: rt_dnode4, 8: rt_dnode8, RT_BVH_CW8: rt_dnode8q (rt_layout.h)
    std::vector<rt_dnode2> nodes2;
    std::vector<rt_dnode4> nodes4;
    std::vector<rt_dnode8> nodes8;
    std::vector<rt_dnode8q> nodes8q;
    // the node array as uploaded, and its node count
    const void *node_data() const {
        return width == 2 ? (const void *)nodes2.data() : width == 4 ? (const void *)nodes4.data()
             : width == 8 ? (const void *)nodes8.data() : (const void *)nodes8q.data();
    }
    size_t node_count() const {
        return width == 2 ? nodes2.size() : width == 4 ? nodes4.size() : width == 8 ? nodes8.size() : nodes8q.size();
    }
    size_t node_bytes() const {
        return width == 2 ? sizeof(rt_dnode2) : width == 4 ? sizeof(rt_dnode4)
             : width == 8 ? sizeof(rt_dnode8) : sizeof(rt_dnode8q);
    }
    template <class F> void for_each_ref(F f) {
        for (auto &n : nodes2) { f(n.ch[0]); f(n.ch[1]); }
        for (auto &n : nodes4) for (auto &c : n.ch) f(c);
        for (auto &n : nodes8) for (auto &c : n.ch) f(c);
        for (auto &n : nodes8q) for (auto &c : n.ch) f(c);
    }
    std::vector<int> order;   // leaf order -> index into the input primitives
    uint32_t root = 0;
    int depth = 0;            // binary-build internal nodes on the longest root-to-leaf path
};

// Primitive boxes cover moving spheres over [min(0, time0), max(0, time1)].
// width: 2 by default; RTNW_BVH_WIDTH = 4, 8 or 8q (compressed 8-wide) for A/B runs.
BvhResult build_bvh(const rt_prim *prims, int n, const rt_instance *instances, float time0, float time1);

// World-space box of one primitive over the shutter span [min(0, time0), max(0, time1)],
// padded like the BVH's boxes and rounded outward to float.
void prim_bounds(const rt_prim &p, const rt_instance *instances, float time0, float time1, float lo[3], float hi[3]);

}  // namespace rtnw
