// bvh.cpp — binned-SAH BVH over the flattened surface primitives, built binary
// and emitted breadth-first as 2-wide nodes, or collapsed into 4-wide ones.
//
// Replaces the reference's bvh_node construction (bvh.h:97-121: random axis,
// median split, recursive) with a surface-area-heuristic build, and its buggy
// slab test (aabb.h:38-39) with a correct one on the device.  Because the device
// breaks ties by list order, the traversal returns the same hit as the flat
// list whatever the tree shape, so the build is a pure performance choice.
//
// Boxes are conservative: every primitive box is padded by an absolute plus a
// relative margin, so a hit the primitive test accepts can never lie outside the
// boxes on its path.
#include "bvh.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <stdexcept>

namespace rtnw {

namespace {

struct Box {
    double lo[3], hi[3];
    Box() { for (int k = 0; k < 3; k++) { lo[k] = 1e300; hi[k] = -1e300; } }
    void grow(const double p[3]) { for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); } }
    void grow(const Box &b) { for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); } }
    bool valid() const { return lo[0] <= hi[0]; }
    double area() const {
        if (!valid()) return 0;
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2 * (dx * dy + dy * dz + dz * dx);
    }
};

// World-space box of one primitive, through its instance chain (outermost first).
Box prim_box(const rt_prim &p, const rt_instance *instances, double ta, double tb) {
    Box b;
    const float *q = p.p;
    auto add_sphere = [&](double cx, double cy, double cz, double r) {
        r = std::fabs(r);
        const double lo[3] = {cx - r, cy - r, cz - r}, hi[3] = {cx + r, cy + r, cz + r};
        b.grow(lo);
        b.grow(hi);
    };
    switch (p.kind) {
    case RT_PRIM_SPHERE: add_sphere(q[0], q[1], q[2], q[3]); break;
    case RT_PRIM_MOVING_SPHERE: {
        const double span = (double)q[7] - (double)q[6];
        for (double t : {ta, tb}) {
            const double s = span != 0 ? (t - q[6]) / span : 0.0;
            add_sphere(q[0] + s * (q[3] - q[0]), q[1] + s * (q[4] - q[1]), q[2] + s * (q[5] - q[2]), q[8]);
        }
        break;
    }
    case RT_PRIM_XY_RECT: { const double lo[3] = {q[0], q[2], q[4]}, hi[3] = {q[1], q[3], q[4]}; b.grow(lo); b.grow(hi); break; }
    case RT_PRIM_XZ_RECT: { const double lo[3] = {q[0], q[4], q[2]}, hi[3] = {q[1], q[4], q[3]}; b.grow(lo); b.grow(hi); break; }
    case RT_PRIM_YZ_RECT: { const double lo[3] = {q[4], q[0], q[2]}, hi[3] = {q[4], q[1], q[3]}; b.grow(lo); b.grow(hi); break; }
    default: throw std::runtime_error("unknown primitive kind");
    }
    if (p.instance >= 0) {
        const rt_instance &in = instances[p.instance];
        for (int k = in.nops - 1; k >= 0; --k) {   // object -> world, innermost wrapper first
            const int op = (int)in.ops[k][0];
            Box w;
            for (int c = 0; c < 8; c++) {
                double v[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
                if (op == RT_OP_TRANSLATE) {
                    for (int a = 0; a < 3; a++) v[a] += in.ops[k][1 + a];
                } else if (op == RT_OP_ROTATE_Y) {
                    const double s = in.ops[k][1], co = in.ops[k][2];
                    const double x = co * v[0] + s * v[2], z = -s * v[0] + co * v[2];
                    v[0] = x;
                    v[2] = z;
                }
                w.grow(v);
            }
            b = w;
        }
    }
    // conservative margin: 1e-3 absolute + 1e-4 of the coordinate magnitude
    for (int k = 0; k < 3; k++) {
        const double mag = std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k]));
        const double pad = 1e-3 + 1e-4 * mag;
        b.lo[k] -= pad;
        b.hi[k] += pad;
    }
    return b;
}

struct Item {
    Box box;
    double c[3];
    int idx;
};

// Binary node of the SAH build (emitted as rt_dnode2 / rt_dnode4 afterwards).
struct Node2 {
    Box box[2];
    uint32_t ch[2];
    int height;   // internal nodes on the longest path down, this one included
};

struct Builder {
    static constexpr int kMaxBins = 256;
    // SAH leaves hold at most 2 primitives: on final() that measured ~2% faster than 4 or 8
    // (tools/ab.py); RTNW_BVH_MAX_LEAF overrides (<= RT_MAX_LEAF) for experiments.
    int max_leaf = 2;
    int bins = 32;           // SAH bins per axis (<= kMaxBins)
    double trav_cost = 1.0;  // SAH node-step cost relative to one primitive test
    std::vector<Item> items;
    std::vector<Node2> nodes;
    std::vector<int> order;   // leaf order -> original prim index
    int max_depth_seen = 0;
    Box bin_box[kMaxBins];     // SAH bin scratch (split)
    int bin_count[kMaxBins];

    uint32_t leaf(int begin, int end) {
        const uint32_t first = (uint32_t)order.size();
        for (int i = begin; i < end; i++) order.push_back(items[i].idx);
        return RT_LEAF_REF(first, end - begin);
    }

    Box range_box(int begin, int end) const {
        Box b;
        for (int i = begin; i < end; i++) b.grow(items[i].box);
        return b;
    }

    // Returns the split position in [begin, end) or -1 to make a leaf.
    int split(int begin, int end, int depth) {
        const int n = end - begin;
        // depth budget: a median split from here must still fit RT_MAX_BVH_DEPTH
        int need = 0;
        for (int m = n; m > 4; m = (m + 1) / 2) need++;
        const bool force_median = depth + need + 1 >= RT_MAX_BVH_DEPTH;
        if (n <= 2 && !force_median) return -1;

        Box cb;
        for (int i = begin; i < end; i++) cb.grow(items[i].c);
        int axis = 0;
        double ext = -1;
        for (int k = 0; k < 3; k++) if (cb.hi[k] - cb.lo[k] > ext) { ext = cb.hi[k] - cb.lo[k]; axis = k; }

        if (force_median || ext <= 0) {
            if (n <= max_leaf && !force_median) return -1;
            if (n <= 4) return -1;
            const int mid = begin + n / 2;
            std::nth_element(items.begin() + begin, items.begin() + mid, items.begin() + end,
                             [axis](const Item &a, const Item &b) { return a.c[axis] < b.c[axis]; });
            return mid;
        }

        const int kBins = bins;
        const double parent_area = range_box(begin, end).area();
        double best_cost = 1e300;
        int best_axis = -1, best_bin = -1;
        for (int k = 0; k < 3; k++) {
            const double e = cb.hi[k] - cb.lo[k];
            if (e <= 0) continue;
            // only the kBins bins in use are reset (a 256-entry local array of boxes was
            // most of the build's time)
            Box *bins = bin_box;
            int *counts = bin_count;
            for (int b = 0; b < kBins; b++) { bins[b] = Box(); counts[b] = 0; }
            for (int i = begin; i < end; i++) {
                int bi = (int)((items[i].c[k] - cb.lo[k]) / e * kBins);
                bi = std::min(std::max(bi, 0), kBins - 1);
                counts[bi]++;
                bins[bi].grow(items[i].box);
            }
            double right_area[kMaxBins];
            int right_count[kMaxBins];
            Box acc;
            int cnt = 0;
            for (int b = kBins - 1; b > 0; b--) {
                acc.grow(bins[b]);
                cnt += counts[b];
                right_area[b] = acc.area();
                right_count[b] = cnt;
            }
            Box lacc;
            int lcnt = 0;
            for (int b = 1; b < kBins; b++) {
                lacc.grow(bins[b - 1]);
                lcnt += counts[b - 1];
                if (lcnt == 0 || right_count[b] == 0) continue;
                const double cost = trav_cost + (lacc.area() * lcnt + right_area[b] * right_count[b]) / parent_area;
                if (cost < best_cost) { best_cost = cost; best_axis = k; best_bin = b; }
            }
        }
        const double leaf_cost = (double)n;
        if (best_axis < 0 || (best_cost >= leaf_cost && n <= max_leaf)) {
            if (n <= max_leaf) return -1;
            const int mid = begin + n / 2;
            std::nth_element(items.begin() + begin, items.begin() + mid, items.begin() + end,
                             [axis](const Item &a, const Item &b) { return a.c[axis] < b.c[axis]; });
            return mid;
        }
        const double lo = cb.lo[best_axis], e = cb.hi[best_axis] - cb.lo[best_axis];
        auto mid_it = std::partition(items.begin() + begin, items.begin() + end, [&](const Item &it) {
            int bi = (int)((it.c[best_axis] - lo) / e * kBins);
            bi = std::min(std::max(bi, 0), kBins - 1);
            return bi < best_bin;
        });
        int mid = (int)(mid_it - items.begin());
        if (mid == begin || mid == end) mid = begin + n / 2;
        return mid;
    }

    // Builds the subtree over [begin, end); returns its child reference.
    uint32_t build(int begin, int end, int depth) {
        const int s = split(begin, end, depth);
        if (s < 0) {
            if (end - begin > RT_MAX_LEAF) throw std::runtime_error("bvh: leaf too large");
            return leaf(begin, end);
        }
        const uint32_t id = (uint32_t)nodes.size();
        nodes.push_back(Node2{});
        max_depth_seen = std::max(max_depth_seen, depth + 1);
        if (depth + 1 > RT_MAX_BVH_DEPTH) throw std::runtime_error("bvh: depth budget exceeded");
        const Box lb = range_box(begin, s), rb = range_box(s, end);
        const uint32_t l = build(begin, s, depth + 1);
        const uint32_t r = build(s, end, depth + 1);
        Node2 &n = nodes[id];
        n.box[0] = lb;
        n.box[1] = rb;
        n.ch[0] = l;
        n.ch[1] = r;
        n.height = 1 + std::max(height(l), height(r));
        return id;
    }

    int height(uint32_t ref) const { return (ref & RT_LEAF_BIT) ? 0 : nodes[ref].height; }
};

// Child `c`'s box rounded outward to float.
void float_box(const Box &b, float lo[3], float hi[3]) {
    for (int a = 0; a < 3; a++) {
        const float l = (float)b.lo[a], h = (float)b.hi[a];
        lo[a] = ((double)l > b.lo[a]) ? std::nextafter(l, -INFINITY) : l;
        hi[a] = ((double)h < b.hi[a]) ? std::nextafter(h, INFINITY) : h;
    }
}
void put_box(rt_dnode4 &n, int c, const Box &b) {
    float lo[3], hi[3];
    float_box(b, lo, hi);
    for (int a = 0; a < 3; a++) {
        float *q = n.q[2 * a + (c >> 1)] + 2 * (c & 1);
        q[0] = lo[a];
        q[1] = hi[a];
    }
}
void put_box(rt_dnode8 &n, int c, const Box &b) {
    float lo[3], hi[3];
    float_box(b, lo, hi);
    for (int a = 0; a < 3; a++) {
        float *q = n.q[4 * a + (c >> 1)] + 2 * (c & 1);
        q[0] = lo[a];
        q[1] = hi[a];
    }
}
void put_box(rt_dnode2 &n, int c, const Box &b) {
    float lo[3], hi[3];
    float_box(b, lo, hi);
    float *f = &n.b[0][0] + 6 * c;   // (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z) of child c
    for (int a = 0; a < 3; a++) {
        f[2 * a] = lo[a];
        f[2 * a + 1] = hi[a];
    }
}

// Compressed BVH8 node from the float boxes of its n children (rt_layout.h
// rt_dnode8q): the grid of axis a starts at the union's lo (rounded down to float)
// with the smallest power-of-two step whose 255 steps cover the union; each plane is
// quantised outward in double, so the decoded box contains the float box.
rt_dnode8q quantise(const rt_dnode8 &f) {
    rt_dnode8q q{};
    for (int c = 0; c < 8; c++) q.ch[c] = f.ch[c];
    uint32_t ebits = 0;
    for (int a = 0; a < 3; a++) {
        double lo = 1e300, hi = -1e300;
        for (int c = 0; c < 8; c++) {
            if (f.ch[c] == RT_EMPTY_CHILD) continue;
            const float *p = f.q[4 * a + (c >> 1)] + 2 * (c & 1);
            lo = std::min(lo, (double)p[0]);
            hi = std::max(hi, (double)p[1]);
        }
        float org = (float)lo;
        if ((double)org > lo) org = std::nextafter(org, -INFINITY);
        int e = -126;   // 2^e, e in [-126, 127]: 255 * 2^e >= hi - org
        while (e < 127 && std::ldexp(255.0, e) < hi - (double)org) e++;
        const double step = std::ldexp(1.0, e);
        q.origin[a] = org;
        ebits |= (uint32_t)(e + 127) << (8 * a);
        uint8_t qlo[8], qhi[8];
        for (int c = 0; c < 8; c++) {
            if (f.ch[c] == RT_EMPTY_CHILD) { qlo[c] = 0; qhi[c] = 0; continue; }   // empty slot: masked by its reference
            const float *p = f.q[4 * a + (c >> 1)] + 2 * (c & 1);
            const double l = std::floor(((double)p[0] - (double)org) / step);
            const double h = std::ceil(((double)p[1] - (double)org) / step);
            qlo[c] = (uint8_t)std::max(0.0, std::min(255.0, l));
            qhi[c] = (uint8_t)std::max(0.0, std::min(255.0, h));
        }
        for (int w = 0; w < 2; w++) {
            q.qa[a][w] = (uint32_t)qlo[4 * w] | (uint32_t)qlo[4 * w + 1] << 8 | (uint32_t)qlo[4 * w + 2] << 16 |
                         (uint32_t)qlo[4 * w + 3] << 24;
            q.qa[a][2 + w] = (uint32_t)qhi[4 * w] | (uint32_t)qhi[4 * w + 1] << 8 | (uint32_t)qhi[4 * w + 2] << 16 |
                             (uint32_t)qhi[4 * w + 3] << 24;
        }
    }
    q.ebits = ebits;
    return q;
}

// Emits the binary tree breadth-first, 2-wide as built or collapsed 4- or 8-wide: a
// node opens its largest-area interior child into that child's two children
// until it has `width`.  `budget`
// bounds the traversal stack below the node: a node with n children pushes at
// most n-1 of them, so a child may be opened only while (n-1) + the tallest
// remaining binary subtree (its own worst case) still fits.
template <class Node>
struct Collapser {
    const Builder &b;
    int width;
    std::vector<Node> out;

    struct Cand { uint32_t ref; Box box; };

    // Children of one wide node (n of them) for binary node `ref`.
    int expand(uint32_t ref, int budget, Cand cs[8]) const {
        const Node2 &n2 = b.nodes[ref];
        cs[0] = {n2.ch[0], n2.box[0]};
        cs[1] = {n2.ch[1], n2.box[1]};
        int n = 2;
        auto bound = [&](int skip, int extra_height, int count) {
            int h = extra_height;
            for (int i = 0; i < n; i++) if (i != skip) h = std::max(h, b.height(cs[i].ref));
            return count - 1 + h;
        };
        while (n < width) {
            int best = -1;
            double best_area = -1;
            for (int i = 0; i < n; i++) {
                if (cs[i].ref & RT_LEAF_BIT) continue;
                const Node2 &c = b.nodes[cs[i].ref];
                const int h = std::max(b.height(c.ch[0]), b.height(c.ch[1]));
                if (bound(i, h, n + 1) > budget) continue;
                const double area = cs[i].box.area();
                if (area > best_area) { best_area = area; best = i; }
            }
            if (best < 0) break;
            const Node2 &c = b.nodes[cs[best].ref];
            const Cand a = {c.ch[0], c.box[0]}, d = {c.ch[1], c.box[1]};
            cs[best] = a;
            cs[n++] = d;
        }
        return n;
    }

    // Nodes are numbered breadth-first, so the top levels are a prefix of the
    // array (the device keeps that prefix in LDS).
    uint32_t collapse(uint32_t root, int budget) {
        struct Job { uint32_t ref; int budget; uint32_t id; };
        std::vector<Job> queue;
        out.push_back(Node{});
        queue.push_back({root, budget, 0});
        for (size_t qi = 0; qi < queue.size(); ++qi) {
            const Job j = queue[qi];
            Cand cs[8];
            const int n = expand(j.ref, j.budget, cs);
            uint32_t ch[8];
            for (uint32_t &c : ch) c = RT_EMPTY_CHILD;
            for (int i = 0; i < n; i++) {
                if (cs[i].ref & RT_LEAF_BIT) {
                    ch[i] = cs[i].ref;
                } else {
                    ch[i] = (uint32_t)out.size();
                    out.push_back(Node{});
                    queue.push_back({cs[i].ref, j.budget - (n - 1), ch[i]});
                }
            }
            // 8-wide: slots by direction from the node's centre (slot bit a = + side of
            // axis a), greedily, so slot order is near-to-far for rays going + on all axes
            int slot[8] = {0, 1, 2, 3, 4, 5, 6, 7};
            if (width == 8) {
                Box all;
                for (int i = 0; i < n; i++) all.grow(cs[i].box);
                bool used_c[8] = {}, used_s[8] = {};
                for (int k = 0; k < n; k++) {
                    double best = 1e300;
                    int bc = -1, bs = -1;
                    for (int i = 0; i < n; i++) {
                        if (used_c[i]) continue;
                        for (int sl = 0; sl < 8; sl++) {
                            if (used_s[sl]) continue;
                            double cost = 0;
                            for (int a = 0; a < 3; a++) {
                                const double d = 0.5 * (cs[i].box.lo[a] + cs[i].box.hi[a]) - 0.5 * (all.lo[a] + all.hi[a]);
                                cost -= ((sl >> a) & 1) ? d : -d;
                            }
                            if (cost < best) { best = cost; bc = i; bs = sl; }
                        }
                    }
                    used_c[bc] = used_s[bs] = true;
                    slot[bc] = bs;
                }
            }
            Node &node = out[j.id];
            for (int i = 0; i < width; i++) node.ch[i] = RT_EMPTY_CHILD;
            for (int i = 0; i < n; i++) {
                put_box(node, slot[i], cs[i].box);
                node.ch[slot[i]] = ch[i];
            }
        }
        return 0;
    }
};

}  // namespace

void prim_bounds(const rt_prim &p, const rt_instance *instances, float time0, float time1, float lo[3], float hi[3]) {
    const Box b = prim_box(p, instances, std::min(0.0, (double)time0), std::max(0.0, (double)time1));
    float_box(b, lo, hi);
}

BvhResult build_bvh(const rt_prim *prims, int n, const rt_instance *instances, float time0, float time1) {
    BvhResult res;
    int width = 2;
    bool quant = false;
    if (const char *e = std::getenv("RTNW_BVH_WIDTH")) {
        const int w = std::atoi(e);
        width = (w == 4 || w == 8) ? w : 2;
        quant = width == 8 && std::strchr(e, 'q') != nullptr;
    }
    res.width = quant ? RT_BVH_CW8 : width;
    if (n <= 0) return res;
    const double ta = std::min(0.0, (double)time0), tb = std::max(0.0, (double)time1);
    Builder b;
    if (const char *e = std::getenv("RTNW_SAH_BINS")) b.bins = std::max(2, std::min(Builder::kMaxBins, std::atoi(e)));
    if (const char *e = std::getenv("RTNW_SAH_TRAV")) b.trav_cost = std::atof(e);
    if (const char *e = std::getenv("RTNW_BVH_MAX_LEAF")) b.max_leaf = std::max(1, std::min(RT_MAX_LEAF, std::atoi(e)));
    b.items.resize(n);
    for (int i = 0; i < n; i++) {
        Item &it = b.items[i];
        it.box = prim_box(prims[i], instances, ta, tb);
        for (int k = 0; k < 3; k++) it.c[k] = 0.5 * (it.box.lo[k] + it.box.hi[k]);
        it.idx = i;
    }
    const uint32_t root2 = b.build(0, n, 0);
    auto emit = [&](auto &out_nodes, auto node_tag) {
        using Node = decltype(node_tag);
        Collapser<Node> c{b, width, {}};
        if (root2 & RT_LEAF_BIT) {   // tiny scene: the single leaf is the root (no nodes)
            res.depth = 0;
            res.root = root2;
            out_nodes = std::move(c.out);
            return;
        }
        c.collapse(root2, RT_STACK_DEPTH - 1);
        res.depth = b.max_depth_seen;
        res.root = 0;
        out_nodes = std::move(c.out);
    };
    if (width == 4) {
        emit(res.nodes4, rt_dnode4{});
    } else if (width == 8) {
        Collapser<rt_dnode8> c{b, 8, {}};
        if (root2 & RT_LEAF_BIT) {
            res.depth = 0;
            res.root = root2;
        } else {
            c.collapse(root2, RT_STACK_DEPTH_W8 - 1);
            res.depth = b.max_depth_seen;
            res.root = 0;
        }
        if (quant) {
            for (const rt_dnode8 &nd : c.out) res.nodes8q.push_back(quantise(nd));
        } else {
            res.nodes8 = std::move(c.out);
        }
    } else {
        emit(res.nodes2, rt_dnode2{});
    }
    res.order = std::move(b.order);
    return res;
}

}  // namespace rtnw
