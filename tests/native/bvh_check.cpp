// tests/native/bvh_check.cpp — invariants of the BVH builder (csrc/host/bvh.cpp) that
// the device traversal relies on, for every node width (2, 4, 8 and the compressed
// 8-wide form, whose boxes are decoded here as the device decodes them), on the built-in scenes and
// on adversarial synthetic ones (run by tests/test_host_api.py):
//   * every primitive is referenced by exactly one leaf, leaves hold <= RT_MAX_LEAF;
//   * every child box contains its subtree's primitive boxes (non-instanced prims);
//   * children are numbered after their parent (breadth-first order);
//   * the traversal stack bound max over paths of sum(children - 1) <= RT_STACK_DEPTH - 1.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "rt_hip.h"
#include "bvh.h"

namespace {

struct B { double lo[3], hi[3]; };

bool prim_box(const rt_prim &p, B &b) {
    const float *q = p.p;
    if (p.instance >= 0) return false;
    if (p.kind == RT_PRIM_SPHERE || p.kind == RT_PRIM_MOVING_SPHERE) {
        const double r = std::fabs(p.kind == RT_PRIM_SPHERE ? q[3] : q[8]);
        for (int a = 0; a < 3; a++) {
            double c0 = q[a], c1 = p.kind == RT_PRIM_SPHERE ? q[a] : q[3 + a];
            b.lo[a] = std::min(c0, c1) - r;
            b.hi[a] = std::max(c0, c1) + r;
        }
        return p.kind == RT_PRIM_SPHERE;   // moving spheres: the shutter-span extrapolation is the builder's business
    }
    int ax[3];
    if (p.kind == RT_PRIM_XY_RECT) { ax[0] = 0; ax[1] = 1; ax[2] = 2; }
    else if (p.kind == RT_PRIM_XZ_RECT) { ax[0] = 0; ax[1] = 2; ax[2] = 1; }
    else { ax[0] = 1; ax[1] = 2; ax[2] = 0; }
    b.lo[ax[0]] = q[0]; b.hi[ax[0]] = q[1];
    b.lo[ax[1]] = q[2]; b.hi[ax[1]] = q[3];
    b.lo[ax[2]] = b.hi[ax[2]] = q[4];
    return true;
}

struct Checker {
    const rt_prim *prims;
    int n;
    const rtnw::BvhResult &r;
    std::vector<int> seen;
    std::string err;

    void child(int width, uint32_t ref, const float lo[3], const float hi[3], uint32_t parent) {
        if (ref == RT_EMPTY_CHILD) return;
        if (ref & RT_LEAF_BIT) {
            const uint32_t first = RT_LEAF_FIRST(ref), cnt = RT_LEAF_COUNT(ref);
            if (cnt > RT_MAX_LEAF) err = "leaf too large";
            for (uint32_t k = 0; k < cnt; k++) {
                if (first + k >= (uint32_t)n) { err = "leaf index out of range"; return; }
                seen[first + k]++;
                B b;
                if (prim_box(prims[r.order[first + k]], b))
                    for (int a = 0; a < 3; a++)
                        if (b.lo[a] < lo[a] || b.hi[a] > hi[a]) err = "leaf box does not contain its primitive";
            }
            return;
        }
        if (ref <= parent) err = "child numbered before its parent";
        node(width, ref, lo, hi);
    }
    static int slots(int width) { return width == RT_BVH_CW8 ? 8 : width; }
    // child c of node id: its reference and its box as the device reads it
    uint32_t child_box(int width, uint32_t id, int c, float lo[3], float hi[3]) const {
        if (width == 2) {
            const rt_dnode2 &d = r.nodes2[id];
            const float *f = &d.b[0][0] + 6 * c;
            for (int a = 0; a < 3; a++) { lo[a] = f[2 * a]; hi[a] = f[2 * a + 1]; }
            return d.ch[c];
        }
        if (width == 4 || width == 8) {
            const float(*q)[4] = width == 4 ? r.nodes4[id].q : r.nodes8[id].q;
            const int per_axis = width / 2;
            for (int a = 0; a < 3; a++) {
                const float *p = q[per_axis * a + (c >> 1)] + 2 * (c & 1);
                lo[a] = p[0]; hi[a] = p[1];
            }
            return width == 4 ? r.nodes4[id].ch[c] : r.nodes8[id].ch[c];
        }
        const rt_dnode8q &d = r.nodes8q[id];
        for (int a = 0; a < 3; a++) {
            const double step = std::ldexp(1.0, (int)((d.ebits >> (8 * a)) & 0xFFu) - 127);
            const uint32_t wl = d.qa[a][c >> 2], wh = d.qa[a][2 + (c >> 2)];
            const double l = d.origin[a] + ((wl >> (8 * (c & 3))) & 0xFFu) * step;   // exact in double
            const double h = d.origin[a] + ((wh >> (8 * (c & 3))) & 0xFFu) * step;
            lo[a] = (float)l;
            hi[a] = (float)h;
            if ((double)lo[a] > l) lo[a] = std::nextafter(lo[a], -INFINITY);   // outward to float
            if ((double)hi[a] < h) hi[a] = std::nextafter(hi[a], INFINITY);
        }
        return d.ch[c];
    }
    // returns the stack bound of the subtree
    int node(int width, uint32_t id, const float plo[3], const float phi[3]) {
        int nch = 0, worst = 0;
        for (int c = 0; c < slots(width); c++) {
            float lo[3], hi[3];
            const uint32_t ref = child_box(width, id, c, lo, hi);
            if (ref == RT_EMPTY_CHILD) continue;
            nch++;
            // (a quantised box may reach up to one grid step past its parent's)
            for (int a = 0; a < 3; a++)
                if (plo && width != RT_BVH_CW8 && (lo[a] < plo[a] || hi[a] > phi[a])) err = "child box outside its parent's box";
            if (!(ref & RT_LEAF_BIT)) worst = std::max(worst, bound_of(width, ref));
            child(width, ref, lo, hi, id);
        }
        return nch;
    }
    int bound_of(int width, uint32_t id) {
        int nch = 0, worst = 0;
        for (int c = 0; c < slots(width); c++) {
            float lo[3], hi[3];
            const uint32_t ref = child_box(width, id, c, lo, hi);
            if (ref == RT_EMPTY_CHILD) continue;
            nch++;
            if (!(ref & RT_LEAF_BIT)) worst = std::max(worst, bound_of(width, ref));
        }
        return std::max(0, nch - 1) + worst;
    }
};

int check(const char *name, const rt_prim *prims, int n, const rt_instance *inst, float t0, float t1) {
    int bad = 0;
    for (int width : {2, 4, 8, RT_BVH_CW8}) {
        setenv("RTNW_BVH_WIDTH", width == RT_BVH_CW8 ? "8q" : std::to_string(width).c_str(), 1);
        const rtnw::BvhResult r = rtnw::build_bvh(prims, n, inst, t0, t1);
        if (r.width != width) { std::printf("%s: built width %d, asked %d\n", name, r.width, width); return bad + 1; }
        Checker c{prims, n, r, std::vector<int>(n, 0), ""};
        int bound = 0;
        if (n == 0) {   // no primitives: no tree (the scene renders with has_bvh = 0)
            if (r.node_count() != 0 || !r.order.empty()) c.err = "a tree for an empty scene";
        } else if (r.root & RT_LEAF_BIT) {   // a single-leaf scene: the leaf is the root
            const float lo[3] = {-INFINITY, -INFINITY, -INFINITY}, hi[3] = {INFINITY, INFINITY, INFINITY};
            c.child(width, r.root, lo, hi, 0);
            if (r.node_count() != 0) c.err = "nodes emitted for a single-leaf scene";
        } else {
            c.node(width, r.root, nullptr, nullptr);
            bound = c.bound_of(width, r.root);
        }
        for (int i = 0; i < n && c.err.empty(); i++)
            if (c.seen[i] != 1) c.err = "primitive referenced " + std::to_string(c.seen[i]) + " times";
        const int cap = (width >= 8 ? RT_STACK_DEPTH_W8 : RT_STACK_DEPTH) - 1;
        if (bound > cap) c.err = "stack bound " + std::to_string(bound) + " exceeds the LDS stack";
        std::printf("%-16s width %d prims %7d nodes %6zu depth %2d stack-bound %2d %s\n", name, width, n,
                    r.node_count(), r.depth, bound, c.err.empty() ? "ok" : c.err.c_str());
        bad += !c.err.empty();
    }
    return bad;
}

rt_prim sphere(double x, double y, double z, double rad) {
    rt_prim p{};
    p.kind = RT_PRIM_SPHERE;
    p.instance = -1;
    p.p[0] = (float)x; p.p[1] = (float)y; p.p[2] = (float)z; p.p[3] = (float)rad;
    return p;
}

}  // namespace

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    int bad = 0;
    const char *names[] = {"final", "random_scene", "cornell_box", "cornell_smoke", "random_motion", "simple_light",
                           "test", "two_spheres", "edge_empty", "edge_single", "edge_degenerate"};
    for (const char *nm : names) {
        rt_scene_desc *d = nullptr;
        if (rt_builtin_scene_desc(nm, &d) != 0) { std::printf("%s: %s\n", nm, rt_last_error()); return 2; }
        bad += check(nm, d->prims, d->nprims, d->instances, d->time0, d->time1);
        rt_scene_desc_free(d);
    }
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(-1000, 1000);
    std::vector<rt_prim> v;
    for (int i = 0; i < 200000; i++) v.push_back(sphere(U(rng), U(rng), U(rng), 0.5 + std::fabs(U(rng)) * 1e-3));
    bad += check("uniform-200k", v.data(), (int)v.size(), nullptr, 0, 1);
    v.clear();   // all identical: SAH cannot split, the depth budget must force medians
    for (int i = 0; i < 50000; i++) v.push_back(sphere(1, 2, 3, 1));
    bad += check("identical-50k", v.data(), (int)v.size(), nullptr, 0, 1);
    v.clear();   // exponentially spaced along a line: maximally unbalanced SAH splits
    for (int i = 0; i < 20000; i++) v.push_back(sphere(std::pow(1.001, i), 0, 0, 0.25));
    bad += check("geometric-20k", v.data(), (int)v.size(), nullptr, 0, 1);
    v.clear();
    v.push_back(sphere(0, 0, 0, 1));
    bad += check("single", v.data(), 1, nullptr, 0, 1);
    std::printf(bad ? "FAILED %d\n" : "OK\n", bad);
    return bad ? 1 : 0;
}
