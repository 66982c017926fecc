// capi.cpp — the C ABI of librt_hip.so (include/rt_hip.h): scene upload to HBM,
// job setup, megakernel + resolve launches, timing, and host helpers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_hip.h"
#include "../rt_layout.h"
#include "../hip/rt_kernel.h"
#include "bvh.h"
#include "rtnw.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    return fail(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

template <class T>
int upload(void **dst, const std::vector<T> &v) {
    *dst = nullptr;
    if (v.empty()) return RT_OK;
    HIP_TRY(hipMalloc(dst, v.size() * sizeof(T)));
    HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return RT_OK;
}

// The scene's arrays share one device allocation filled by one copy (scene creation
// was a dozen hipMalloc + hipMemcpy round trips): stage() appends an array to the
// host image at a 256-B aligned offset, commit() uploads it and sets the pointers.
// An empty array is staged as one zeroed 256-B sentinel: no scene pointer the kernel
// receives is ever null, so a load the compiler speculates out of its branch (e.g. a
// texture record read for lanes that have none) reads zeros instead of faulting on an
// empty scene (edge_empty's illegal access).
struct Arena {
    std::vector<uint8_t> host;
    std::vector<std::pair<void **, size_t>> fix;
};
template <class T>
void stage(Arena &a, void **dst, const std::vector<T> &v) {
    *dst = nullptr;
    const size_t off = (a.host.size() + 255) & ~(size_t)255;
    const size_t bytes = v.empty() ? std::max<size_t>(256, sizeof(T)) : v.size() * sizeof(T);
    a.host.resize(off + bytes, 0);
    if (!v.empty()) std::memcpy(a.host.data() + off, v.data(), bytes);
    a.fix.push_back({dst, off});
}
int commit(Arena &a, void **base) {
    *base = nullptr;
    if (a.host.empty()) return RT_OK;
    HIP_TRY(hipMalloc(base, a.host.size()));
    HIP_TRY(hipMemcpy(*base, a.host.data(), a.host.size(), hipMemcpyHostToDevice));
    for (auto &f : a.fix) *f.first = (uint8_t *)*base + f.second;
    return RT_OK;
}

// Resident workgroups per CU of the megakernel, per launch mode and BVH width: a
// property of the code objects, queried once per process.
hipError_t occupancy(int *mega, int mode, int width) {
    static std::mutex mu;
    static int cache[3][5] = {};   // [mode][BVH2, BVH4, flat scan, BVH8, compressed BVH8]
    std::lock_guard<std::mutex> lock(mu);
    int &c = cache[mode][width == 4 ? 1 : width == 0 ? 2 : width == 8 ? 3 : width == RT_BVH_CW8 ? 4 : 0];
    if (!c) {
        hipError_t e;
        if ((e = rt_megakernel_occupancy(&c, mode, width)) != hipSuccess) { c = 0; return e; }
    }
    *mega = c;
    return hipSuccess;
}

int ibits(float f) { int i; std::memcpy(&i, &f, 4); return i; }
float fbits(int i) { float f; std::memcpy(&f, &i, 4); return f; }

rt_dprim to_dprim(const rt_prim &p, int order) {
    rt_dprim d{};
    const float *q = p.p;
    switch (p.kind) {
    case RT_PRIM_SPHERE:
        d.g0[0] = q[0]; d.g0[1] = q[1]; d.g0[2] = q[2]; d.g0[3] = q[3];
        break;
    case RT_PRIM_MOVING_SPHERE:
        // center(t) = c0 + ((t - t0) / (t1 - t0)) * (c1 - c0): the two differences
        // are float subtractions of the reference (sphere.h:82), computed once here.
        d.g0[0] = q[0]; d.g0[1] = q[1]; d.g0[2] = q[2]; d.g0[3] = q[8];
        d.g1[0] = q[3] - q[0]; d.g1[1] = q[4] - q[1]; d.g1[2] = q[5] - q[2]; d.g1[3] = q[6];
        d.g2[0] = q[7] - q[6];
        break;
    default:   // rects (k goes to m[1])
        d.g0[0] = q[0]; d.g0[1] = q[1]; d.g0[2] = q[2]; d.g0[3] = q[3];
        break;
    }
    d.m[0] = p.kind | (p.flip ? 1 << 8 : 0) | (p.material << 9);
    if (p.kind >= RT_PRIM_XY_RECT) {
        d.m[1] = ibits(q[4]);   // rect plane k
    } else {                    // spheres: RN(1/radius) for the normal's div_rn, 0 if not a normal float
        const float y = 1.0f / d.g0[3];
        d.m[1] = (std::isnormal(y)) ? ibits(y) : 0;
    }
    d.m[2] = p.instance;
    d.m[3] = order;
    return d;
}

// SURVEY §8d byte model (bytes the algorithm must read or write, independent of
// this implementation's record padding):
//   node fetch: the bytes loaded per visit (BVH2 64 B, BVH4 112 B, BVH8 224 B, compressed
//   BVH8 96 B); sphere 16 B; moving sphere 36 B;
//   rect 24 B; instance chain entered 32 B; medium record 16 B; material +
//   texture per shade 16 + 16 B; Perlin turbulence 7 octaves x 8 gradient gathers
//   x (12 B gradient + 3 x 4 B permutation) = 1344 B; per work item the 4-B job
//   pixel read and the 16-B partial sum written.  (rt_resolve's own traffic — the
//   partial sums read back, the output index and the 12-B pixel — is not the
//   megakernel's.)
double algorithmic_bytes(const rt_stats &st, double items, int bvh_width) {
    const double node = bvh_width == 4 ? 112.0 : bvh_width == 8 ? 224.0 : bvh_width == RT_BVH_CW8 ? 96.0 : 64.0;
    return node * st.node_visits + 16.0 * st.sphere_tests + 36.0 * st.moving_sphere_tests + 24.0 * st.rect_tests +
           32.0 * st.instanced_tests + 16.0 * st.medium_tests + 32.0 * st.shades + 1344.0 * st.noise_evals +
           20.0 * items;
}

}  // namespace

// shared with dist.cpp: sets the thread-local message rt_last_error() returns
int rt_internal_fail(int code, const std::string &msg) { return fail(code, msg); }

struct rt_scene {
    int device = 0;
    int cus = 0;
    int grid[3] = {0, 0, 0};      // persistent megakernel grid per variant (plain, count, profile)
    bool lds_nodes = false;       // the BVH2 fits the LDS variant (one RT_LDS_BLOCK workgroup per CU)
    int stack_depth = 0;          // its traversal stack entries per lane
    hipStream_t own_stream = nullptr;
    // scene in HBM: one allocation (arena) holding the arrays below
    void *arena = nullptr;
    void *nodes = nullptr, *prims = nullptr, *bprims = nullptr, *media = nullptr, *mats = nullptr, *texs = nullptr,
         *insts = nullptr, *ranvec = nullptr, *perm = nullptr, *texels = nullptr, *groups = nullptr;
    bool scan = false;            // flat scan of the primitive groups instead of the BVH (small scenes)
    int nprescan = 0;             // BVH scenes: largest primitives tested in lockstep before the BVH
    // medium cell (rt_scene_create): primitives [cell_first, cell_first + cell_n) are copies of those near the ball
    int cell_first = 0, cell_n = 0;
    float cell_c[3] = {0, 0, 0}, cell_r2 = 0, cell_rin2 = 0;
    int ngroups = 0;
    uint32_t root = 0;
    int has_bvh = 0, nmedia = 0, bvh_depth = 0, nnodes = 0, nprims = 0, bvh_width = 2, ninstances = 0;
    bool has_moving = false;
    bool has_uv = false;       // a material reads (u, v)
    bool has_checker = false;  // a checker_texture exists
    bool has_specular = false; // a metal or dielectric material exists
    float time0 = 0, time1 = 1;
    // job cache
    std::vector<int32_t> job_tiles;
    uint32_t job_ndeep = 0;                 // the job's first job_ndeep pixels are the deep ones (prepare_job)
    std::vector<float> deep_balls;          // dense media's boundary balls (cx, cy, cz, r), rt_scene_create
    uint32_t npix = 0;
    void *job_xy = nullptr, *job_out = nullptr;
    void *slab = nullptr;
    size_t slab_bytes = 0;
    void *acc = nullptr;          // per-pixel running sums between sample batches
    size_t acc_bytes = 0;
    void *counter = nullptr, *stats = nullptr;
    void *host_out = nullptr;
    size_t host_out_bytes = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
};

// The kernel features (RT_FEAT_*) a scene's launches carry code for: the launcher runs the
// smallest compiled variant covering them (rt_kernel.hip launch_features).  RTNW_FEAT_ALL=1
// runs the all-feature variant (the one the wide BVHs use): A/B runs only.
static int scene_features(const rt_scene *s) {
    if (const char *e = std::getenv("RTNW_FEAT_ALL"))
        if (std::atoi(e)) return RT_FEAT_ALL;
    return (s->ninstances > 0 ? RT_FEAT_INST : 0) | (s->has_uv ? RT_FEAT_UV : 0) |
           (s->has_checker ? RT_FEAT_CHECKER : 0) | (s->nprescan > 0 ? RT_FEAT_PRESCAN : 0) |
           (s->nmedia > 0 ? RT_FEAT_MEDIA : 0);
}

extern "C" {

const char *rt_last_error(void) { return g_err.c_str(); }
const char *rt_version(void) { return "rt_hip 1 (gfx950 persistent megakernel)"; }

int rt_device_count(int *out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *out = 0; return hip_fail(e, "hipGetDeviceCount"); }
    *out = n;
    return RT_OK;
}

int rt_device_alloc(int device, uint64_t bytes, void **out) {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMalloc(out, bytes));
    return RT_OK;
}
int rt_device_free(void *ptr) {
    HIP_TRY(hipFree(ptr));
    return RT_OK;
}
int rt_copy_to_host(void *dst, const void *src, uint64_t bytes) {
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_math_probe(int fn, const float *a, const float *b, float *out, int64_t n) {
    if (fn < 0 || fn > 5 || n < 0 || n > (1 << 30) || (n && (!a || !out || (fn >= 4 && !b))))
        return fail(RT_ERR_INVALID, "rt_math_probe: bad arguments");
    if (n == 0) return RT_OK;
    const size_t bytes = (size_t)n * sizeof(float);
    float *d = nullptr;
    HIP_TRY(hipMalloc((void **)&d, 3 * bytes));
    hipError_t e = hipMemcpy(d, a, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && fn >= 4) e = hipMemcpy(d + n, b, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rt_launch_math_probe(fn, d, d + n, d + 2 * n, (int)n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 2 * n, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "rt_math_probe");
    return RT_OK;
}

int rt_camera_init(rt_camera_desc *out, const float lookfrom[3], const float lookat[3], const float vup[3], float vfov,
                   float aspect, float aperture, float focus_dist, float t0, float t1) {
    if (!out || !lookfrom || !lookat || !vup) return fail(RT_ERR_INVALID, "rt_camera_init: null argument");
    rtnw::camera c(rtnw::vec3(lookfrom[0], lookfrom[1], lookfrom[2]), rtnw::vec3(lookat[0], lookat[1], lookat[2]),
                   rtnw::vec3(vup[0], vup[1], vup[2]), vfov, aspect, aperture, focus_dist, t0, t1);
    *out = c.desc();
    return RT_OK;
}

static int validate_desc(const rt_scene_desc *d) {
    if (!d) return fail(RT_ERR_INVALID, "null scene descriptor");
    if (d->abi_version != RT_ABI_VERSION) return fail(RT_ERR_INVALID, "rt_scene_desc.abi_version mismatch");
    if (d->nprims < 0 || d->nboundary < 0 || d->nmedia < 0 || d->nmaterials < 0 || d->ntextures < 0 || d->ninstances < 0)
        return fail(RT_ERR_INVALID, "negative count in scene descriptor");
    if (d->nprims > (1 << 24) - 1 || d->nboundary > (1 << 24) - 1) return fail(RT_ERR_INVALID, "too many primitives");
    if (d->nmaterials > (1 << 22)) return fail(RT_ERR_INVALID, "too many materials");
    if (!d->perlin_ranvec || !d->perlin_perm) return fail(RT_ERR_INVALID, "missing Perlin tables");
    if (d->nimages < 0 || d->image_bytes < 0 || (d->nimages > 0 && (!d->images || !d->image_data)))
        return fail(RT_ERR_INVALID, "bad image arrays");
    auto check_prim = [&](const rt_prim &p) -> int {
        if (p.kind < RT_PRIM_SPHERE || p.kind > RT_PRIM_YZ_RECT) return fail(RT_ERR_INVALID, "bad primitive kind");
        if (p.material < 0 || p.material >= d->nmaterials) return fail(RT_ERR_INVALID, "primitive material out of range");
        if (p.instance < -1 || p.instance >= d->ninstances) return fail(RT_ERR_INVALID, "primitive instance out of range");
        return RT_OK;
    };
    for (int i = 0; i < d->nprims; i++) if (int rc = check_prim(d->prims[i])) return rc;
    for (int i = 0; i < d->nboundary; i++) if (int rc = check_prim(d->boundary_prims[i])) return rc;
    for (int i = 0; i < d->nmedia; i++) {
        const rt_medium &m = d->media[i];
        if (m.boundary_first < 0 || m.boundary_count < 0 || m.boundary_first + m.boundary_count > d->nboundary)
            return fail(RT_ERR_INVALID, "medium boundary range out of range");
        if (m.material < 0 || m.material >= d->nmaterials) return fail(RT_ERR_INVALID, "medium material out of range");
    }
    for (int i = 0; i < d->ninstances; i++) {
        const rt_instance &in = d->instances[i];
        if (in.nops < 0 || in.nops > RT_MAX_INSTANCE_OPS) return fail(RT_ERR_INVALID, "instance chain too long");
        for (int k = 0; k < in.nops; k++) {
            const int op = (int)in.ops[k][0];
            if (op < RT_OP_TRANSLATE || op > RT_OP_FLIP) return fail(RT_ERR_INVALID, "bad instance op");
        }
    }
    for (int i = 0; i < d->ntextures; i++) {
        const rt_texture &t = d->textures[i];
        if (t.kind < RT_TEX_CONSTANT || t.kind > RT_TEX_IMAGE) return fail(RT_ERR_INVALID, "bad texture kind");
        if (t.kind == RT_TEX_IMAGE) {
            if (t.image < 0 || t.image >= d->nimages) return fail(RT_ERR_INVALID, "image texture index out of range");
            const rt_image &im = d->images[t.image];
            if (im.nx <= 0 || im.ny <= 0 || im.offset < 0 ||
                im.offset + (int64_t)3 * im.nx * im.ny > d->image_bytes || im.offset > 0x7FFFFFFF)
                return fail(RT_ERR_INVALID, "image texels out of range");
        }
        if (t.kind == RT_TEX_CHECKER) {
            if (t.even < 0 || t.even >= d->ntextures || t.odd < 0 || t.odd >= d->ntextures)
                return fail(RT_ERR_INVALID, "checker child out of range");
        }
    }
    // checker chains must terminate within the device's depth guard
    for (int i = 0; i < d->ntextures; i++) {
        std::vector<int> stack{i};
        std::vector<int> depth{0};
        while (!stack.empty()) {
            int t = stack.back(), dd = depth.back();
            stack.pop_back(); depth.pop_back();
            if (dd >= RT_MAX_CHECKER_DEPTH) return fail(RT_ERR_UNSUPPORTED, "checker textures nested too deep (or cyclic)");
            if (d->textures[t].kind == RT_TEX_CHECKER) {
                stack.push_back(d->textures[t].even); depth.push_back(dd + 1);
                stack.push_back(d->textures[t].odd); depth.push_back(dd + 1);
            }
        }
    }
    for (int i = 0; i < d->nmaterials; i++) {
        const rt_material &m = d->materials[i];
        if (m.kind < RT_MAT_LAMBERTIAN || m.kind > RT_MAT_ISOTROPIC) return fail(RT_ERR_INVALID, "bad material kind");
        const bool textured = m.kind == RT_MAT_LAMBERTIAN || m.kind == RT_MAT_DIFFUSE_LIGHT || m.kind == RT_MAT_ISOTROPIC;
        if (textured && (m.texture < 0 || m.texture >= d->ntextures)) return fail(RT_ERR_INVALID, "material texture out of range");
    }
    return RT_OK;
}

void rt_scene_destroy(rt_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (void *p : {s->arena, s->job_xy, s->job_out, s->slab, s->acc, s->counter, s->host_out})
        if (p) (void)hipFree(p);
    for (auto &e : s->ev) if (e) (void)hipEventDestroy(e);
    if (s->own_stream) (void)hipStreamDestroy(s->own_stream);
    delete s;
}

int rt_scene_create(const rt_scene_desc *d, int device, rt_scene **out) {
    if (!out) return fail(RT_ERR_INVALID, "rt_scene_create: null out");
    *out = nullptr;
    if (int rc = validate_desc(d)) return rc;
    // RTNW_TRACE: per-phase times of the scene setup on stderr (diagnostics)
    const bool trace_on = std::getenv("RTNW_TRACE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto trace = [&](const char *what) {
        if (!trace_on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "rt_scene_create: %-28s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t_last).count());
        t_last = now;
    };
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return fail(RT_ERR_HIP, "no HIP device available (the path tracer has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    trace("device check");

    // Pre-scan (BVH scenes): the largest primitives — box area >= RTNW_PRESCAN_AREA
    // (default 10 %) of the scene box's, at most RT_PRESCAN_MAX — stay out of the BVH
    // and are tested in lockstep before every descent (rt_kernel.hip): a primitive
    // whose box spans the scene sits at the BVH's root and nearly every ray tests it
    // anyway.  random_motion's ground sphere: c3 55.57 -> 52.15 ms; final()'s six
    // largest (0.5 %: 2-3 % each) 59.08 -> 62.27 ms, so the threshold leaves them in
    // the BVH.  RTNW_PRESCAN=0 keeps every primitive in the BVH.
    std::vector<int> big, rest;
    {
        bool want = d->nprims > RT_SCAN_MAX;
        if (const char *e = std::getenv("RTNW_PRESCAN")) want = want && std::atoi(e) != 0;
        double frac = 0.10;
        if (const char *e = std::getenv("RTNW_PRESCAN_AREA")) frac = std::atof(e);
        std::vector<double> area(d->nprims, 0.0);
        if (want) {
            double slo[3] = {1e300, 1e300, 1e300}, shi[3] = {-1e300, -1e300, -1e300};
            for (int i = 0; i < d->nprims; i++) {
                float lo[3], hi[3];
                rtnw::prim_bounds(d->prims[i], d->instances, d->time0, d->time1, lo, hi);
                for (int k = 0; k < 3; k++) { slo[k] = std::min(slo[k], (double)lo[k]); shi[k] = std::max(shi[k], (double)hi[k]); }
                const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
                area[i] = 2 * (x * y + y * z + z * x);
            }
            const double x = shi[0] - slo[0], y = shi[1] - slo[1], z = shi[2] - slo[2];
            const double sa = 2 * (x * y + y * z + z * x);
            std::vector<int> cand;
            for (int i = 0; i < d->nprims; i++) if (area[i] >= frac * sa) cand.push_back(i);
            std::stable_sort(cand.begin(), cand.end(), [&](int p, int q) { return area[p] > area[q]; });
            if ((int)cand.size() > RT_PRESCAN_MAX) cand.resize(RT_PRESCAN_MAX);
            std::sort(cand.begin(), cand.end());
            big = cand;
        }
        std::vector<char> is_big(d->nprims, 0);
        for (int i : big) is_big[i] = 1;
        for (int i = 0; i < d->nprims; i++) if (!is_big[i]) rest.push_back(i);
    }
    std::vector<rt_prim> rest_prims;
    rest_prims.reserve(rest.size());
    for (int i : rest) rest_prims.push_back(d->prims[i]);

    rtnw::BvhResult bvh;
    try {
        bvh = rtnw::build_bvh(rest_prims.data(), (int)rest_prims.size(), d->instances, d->time0, d->time1);
    } catch (const std::exception &ex) {
        return fail(RT_ERR_INVALID, std::string("BVH build failed: ") + ex.what());
    }
    // leaf order -> input primitive, the pre-scanned ones first; leaf refs shifted past them
    for (int &o : bvh.order) o = rest[o];
    if (!big.empty()) {
        const uint32_t K = (uint32_t)big.size();
        auto shift = [&](uint32_t &ref) {
            if (ref != RT_EMPTY_CHILD && (ref & RT_LEAF_BIT))
                ref = RT_LEAF_REF(RT_LEAF_FIRST(ref) + K, RT_LEAF_COUNT(ref));
        };
        bvh.for_each_ref(shift);
        shift(bvh.root);
        bvh.order.insert(bvh.order.begin(), big.begin(), big.end());
    }
    trace("BVH build");

    auto *s = new rt_scene();
    s->device = device;
    s->time0 = d->time0;
    s->time1 = d->time1;
    auto cleanup = [&](int rc) { rt_scene_destroy(s); return rc; };

    // Flat scan instead of the BVH for scenes of at most RT_SCAN_MAX primitives
    // (rt_layout.h rt_dgroup; RTNW_SCAN=0 keeps the BVH): primitives ordered by
    // instance chain (list order within a chain), one group per chain.
    {
        bool want = true;
        if (const char *e = std::getenv("RTNW_SCAN")) want = std::atoi(e) != 0;
        s->scan = want && d->nprims >= 1 && d->nprims <= RT_SCAN_MAX && bvh.width == 2;
    }
    std::vector<int> order = bvh.order;
    std::vector<rt_dgroup> groups;
    if (s->scan) {
        order.resize(d->nprims);
        for (int i = 0; i < d->nprims; i++) order[i] = i;
        // by chain, then by kind within a chain (rt_dgroup: one loop per kind)
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
            const rt_prim &px = d->prims[x], &py = d->prims[y];
            return px.instance != py.instance ? px.instance < py.instance : px.kind < py.kind;
        });
        for (int i = 0; i < d->nprims; i++) {
            const rt_prim &pr = d->prims[order[i]];
            float lo[3], hi[3];
            rtnw::prim_bounds(pr, d->instances, d->time0, d->time1, lo, hi);
            if (groups.empty() || groups.back().instance != pr.instance) {
                rt_dgroup g{};
                g.first = i;
                g.instance = pr.instance;
                g.bx[0] = lo[0]; g.bx[1] = hi[0]; g.bx[2] = lo[1]; g.bx[3] = hi[1];
                g.bz[0] = lo[2]; g.bz[1] = hi[2];
                groups.push_back(g);
            }
            rt_dgroup &g = groups.back();
            // scan_group (rt_device.h) walks a group's runs in the enum order of the kinds,
            // from 8-bit counts packed at 8 * kind in `kinds` (yz rects in nyz)
            static_assert(RT_PRIM_SPHERE == 0 && RT_PRIM_MOVING_SPHERE == 1 && RT_PRIM_XY_RECT == 2 &&
                              RT_PRIM_XZ_RECT == 3 && RT_PRIM_YZ_RECT == 4,
                          "rt_dgroup.kinds packs the primitive kinds 0..3 by their enum value");
            static_assert(RT_SCAN_MAX < 256, "rt_dgroup.kinds holds 8-bit counts");
            g.count++;
            if (pr.kind == RT_PRIM_YZ_RECT) g.nyz++;
            else g.kinds += 1 << (8 * pr.kind);     // count <= RT_SCAN_MAX < 256 per kind
            g.bx[0] = std::min(g.bx[0], lo[0]); g.bx[1] = std::max(g.bx[1], hi[0]);
            g.bx[2] = std::min(g.bx[2], lo[1]); g.bx[3] = std::max(g.bx[3], hi[1]);
            g.bz[0] = std::min(g.bz[0], lo[2]); g.bz[1] = std::max(g.bz[1], hi[2]);
        }
    }
    for (const rt_dgroup &g : groups) {   // the per-kind runs cover the group exactly
        const int runs = (g.kinds & 0xff) + ((g.kinds >> 8) & 0xff) + ((g.kinds >> 16) & 0xff) +
                         ((g.kinds >> 24) & 0xff) + g.nyz;
        if (runs != g.count) return cleanup(fail(RT_ERR_INVALID, "flat scan: a group's kind counts do not add up"));
    }
    // Medium cell (BVH modes; rt_kernel.hip stages 3 and 6): a path inside a dense medium
    // scatters there segment after segment (final(): a third of all segments start inside
    // the subsurface sphere), and every segment's closest-hit search starts from the BVH
    // root.  For one medium bounded by a sphere (c, R) — the densest such — the primitives
    // whose boxes reach within R + m of c (m = R / 64 + 1e-3 |c|) are listed (at most
    // RT_CELL_MAX, appended to the device primitives as copies: same record, same key); a
    // ray starting within R + m / 2 of c tests just them, and if the nearest lies before the
    // ray leaves that ball, no other primitive (all are outside R + m) can be nearer: the
    // search ends there with the same (t, key) winner as the full one.  The kernel's ball
    // waves gather such paths (RtKernelArgs.ball_waves).  RTNW_CELL=0 disables it.
    s->cell_n = 0;
    if (!s->scan && d->nprims > 0) {
        bool want = true;
        if (const char *e = std::getenv("RTNW_CELL")) want = std::atoi(e) != 0;
        double best_density = -1;
        std::vector<int> cell;
        for (int i = 0; want && i < d->nmedia; i++) {
            const rt_medium &m = d->media[i];
            if (m.boundary_count != 1) continue;
            const rt_prim &bp = d->boundary_prims[m.boundary_first];
            if (bp.kind != RT_PRIM_SPHERE || bp.instance >= 0 || !(m.density > best_density)) continue;
            const double c[3] = {bp.p[0], bp.p[1], bp.p[2]}, R = std::fabs((double)bp.p[3]);
            const double cmax = std::max(std::fabs(c[0]), std::max(std::fabs(c[1]), std::fabs(c[2])));
            const double mg = R / 64 + 1e-3 * cmax, reach = R + mg;
            if (!(R > 0) || !std::isfinite(reach)) continue;
            std::vector<int> near;
            for (int q = 0; q < d->nprims && (int)near.size() <= RT_CELL_MAX; q++) {
                float lo[3], hi[3];
                rtnw::prim_bounds(d->prims[q], d->instances, d->time0, d->time1, lo, hi);
                double d2 = 0;
                for (int k = 0; k < 3; k++) {
                    const double v = std::max(std::max((double)lo[k] - c[k], c[k] - (double)hi[k]), 0.0);
                    d2 += v * v;
                }
                if (!(d2 > reach * reach)) near.push_back(q);   // (a NaN box counts as near)
            }
            if (near.empty() || (int)near.size() > RT_CELL_MAX) continue;
            best_density = m.density;
            s->cell_n = (int)near.size();
            for (int k = 0; k < 3; k++) s->cell_c[k] = (float)c[k];
            const double rk = R + mg / 2, rin = R * (1 - 1.0 / 1024);
            s->cell_r2 = (float)(rk * rk);
            s->cell_rin2 = (float)(rin * rin);   // (routing only: rays nearer the surface count as inside when heading in)
            cell = near;
        }
        s->cell_first = (int)order.size();
        for (int q : cell) order.push_back(q);
    }
    std::vector<rt_dprim> prims(order.size()), bprims(d->nboundary);
    for (int i = 0; i < (int)order.size(); i++) {
        const int src = order[i];
        prims[i] = to_dprim(d->prims[src], src);
        s->has_moving |= d->prims[src].kind == RT_PRIM_MOVING_SPHERE;
    }
    for (int i = 0; i < d->nboundary; i++) {
        bprims[i] = to_dprim(d->boundary_prims[i], i);
        s->has_moving |= d->boundary_prims[i].kind == RT_PRIM_MOVING_SPHERE;
    }
    // a material whose texture tree reaches an image needs the hit's (u, v)
    auto reads_uv = [&](int t) {
        std::vector<int> st{t};
        while (!st.empty()) {
            const int x = st.back();
            st.pop_back();
            if (x < 0) continue;
            if (d->textures[x].kind == RT_TEX_IMAGE) return true;
            if (d->textures[x].kind == RT_TEX_CHECKER) { st.push_back(d->textures[x].even); st.push_back(d->textures[x].odd); }
        }
        return false;
    };
    std::vector<rt_dmaterial> mats(d->nmaterials);
    for (int i = 0; i < d->nmaterials; i++) {
        const rt_material &m = d->materials[i];
        rt_dmaterial &o = mats[i];
        o.kind = m.kind;
        o.texture = m.texture;
        o.fuzz = m.fuzz;
        o.ref_idx = m.ref_idx;
        for (int k = 0; k < 3; k++) o.albedo[k] = m.albedo[k];
        if (m.kind == RT_MAT_DIELECTRIC) {
            // a dielectric has no albedo (material.h:99): its slots carry the per-material
            // constants of material.h:103-116 in the reference's float/double arithmetic
            const float r0 = (1 - m.ref_idx) / (1 + m.ref_idx);
            o.albedo[0] = (float)(1.0 / (double)m.ref_idx);   // ni_over_nt entering
            o.albedo[1] = r0 * r0;                            // schlick's r0^2
            o.albedo[2] = m.ref_idx * m.ref_idx;              // ref_idx^2 of the exit cosine
        }
        o.flags = (m.texture >= 0 && reads_uv(m.texture)) ? 1 : 0;
        s->has_uv |= o.flags != 0;
        // a textured material (lambertian, isotropic, diffuse_light) whose texture is a
        // constant: its color in the unused albedo slots, flag 2 (shade_begin then reads
        // no texture record: one dependent load fewer per shade)
        const bool textured = m.kind == RT_MAT_LAMBERTIAN || m.kind == RT_MAT_ISOTROPIC || m.kind == RT_MAT_DIFFUSE_LIGHT;
        if (textured && m.texture >= 0 && m.texture < d->ntextures &&
            d->textures[m.texture].kind == RT_TEX_CONSTANT) {
            for (int k = 0; k < 3; k++) o.albedo[k] = d->textures[m.texture].color[k];
            o.flags |= 2;
        }
        s->has_specular |= m.kind == RT_MAT_METAL || m.kind == RT_MAT_DIELECTRIC;
    }
    std::vector<rt_dtexture> texs(d->ntextures);
    for (int i = 0; i < d->ntextures; i++) {
        const rt_texture &t = d->textures[i];
        rt_dtexture &o = texs[i];
        o.kind = t.kind;
        o.even = t.even;
        o.odd = t.odd;
        s->has_checker |= t.kind == RT_TEX_CHECKER;
        o.scale = t.scale;
        for (int k = 0; k < 3; k++) o.color[k] = t.color[k];
        if (t.kind == RT_TEX_IMAGE) {   // (kind, nx, ny, byte offset)
            const rt_image &im = d->images[t.image];
            o.even = im.nx;
            o.odd = im.ny;
            o.scale = fbits((int)im.offset);
        }
    }
    std::vector<rt_dinstance> insts(d->ninstances);
    for (int i = 0; i < d->ninstances; i++) {
        const rt_instance &in = d->instances[i];
        rt_dinstance &o = insts[i];
        o.nops = in.nops;
        for (int k = 0; k < in.nops; k++) {
            o.ops[k][0] = fbits((int)in.ops[k][0]);   // op code as integer bits
            for (int c = 1; c < 4; c++) o.ops[k][c] = in.ops[k][c];
        }
    }
    std::vector<rt_dmedium> media(d->nmedia);
    for (int i = 0; i < d->nmedia; i++) {
        media[i].first = d->media[i].boundary_first;
        media[i].count = d->media[i].boundary_count;
        media[i].neg_inv_density = -(1 / d->media[i].density);   // constant_medium.h:36
        media[i].material = d->media[i].material;
    }
    std::vector<float> ranvec(256 * 4, 0.0f);
    for (int i = 0; i < 256; i++) for (int k = 0; k < 3; k++) ranvec[4 * i + k] = d->perlin_ranvec[3 * i + k];
    std::vector<int32_t> perm(d->perlin_perm, d->perlin_perm + 768);
    std::vector<uint8_t> texels(d->image_data, d->image_data + (d->nimages > 0 ? d->image_bytes : 0));
    for (int v : perm) if (v < 0 || v > 255) return cleanup(fail(RT_ERR_INVALID, "Perlin permutation entry out of range"));

    Arena arena;
    if (bvh.width == 4) stage(arena, &s->nodes, bvh.nodes4);
    else if (bvh.width == 8) stage(arena, &s->nodes, bvh.nodes8);
    else if (bvh.width == RT_BVH_CW8) stage(arena, &s->nodes, bvh.nodes8q);
    else stage(arena, &s->nodes, bvh.nodes2);
    stage(arena, &s->prims, prims);
    stage(arena, &s->bprims, bprims);
    stage(arena, &s->media, media);
    stage(arena, &s->mats, mats);
    stage(arena, &s->texs, texs);
    stage(arena, &s->insts, insts);
    stage(arena, &s->groups, groups);
    stage(arena, &s->ranvec, ranvec);
    stage(arena, &s->perm, perm);
    stage(arena, &s->texels, texels);
    trace("device records");
    if (int rc = commit(arena, &s->arena)) return cleanup(rc);
    trace("upload (one allocation)");
    s->root = bvh.root;
    s->has_bvh = d->nprims > 0;
    s->nmedia = d->nmedia;
    // Dense media (mean free path below half the boundary sphere's radius: final()'s
    // subsurface sphere, not its scene-wide fog): paths that enter one random-walk to the
    // depth cap, so the job lists the pixels whose primary rays enter one first and the
    // kernel claims all their samples before the others' (prepare_job): the launch's
    // last claims then hold few such paths, whose latency chains are its drain.
    for (int i = 0; i < d->nmedia; i++) {
        const rt_medium &m = d->media[i];
        if (m.boundary_count != 1 || !(m.density > 0)) continue;
        const rt_prim &bp = d->boundary_prims[m.boundary_first];
        const float R = std::fabs(bp.p[3]);
        if (bp.kind != RT_PRIM_SPHERE || bp.instance >= 0 || !(1.0f / m.density < 0.5f * R)) continue;
        s->deep_balls.insert(s->deep_balls.end(), {bp.p[0], bp.p[1], bp.p[2], R});
    }
    s->bvh_depth = bvh.depth;
    s->nnodes = (int)bvh.node_count();
    s->bvh_width = bvh.width;
    s->nprims = d->nprims;
    s->ninstances = d->ninstances;
    s->ngroups = (int)groups.size();
    s->nprescan = s->scan ? 0 : (int)big.size();

    if ((e = hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
        return cleanup(hip_fail(e, "hipDeviceGetAttribute"));
    for (int mode = 0; mode < 3; mode++) {
        int bpc = 0;
        if ((e = occupancy(&bpc, mode, s->scan ? 0 : s->bvh_width)) != hipSuccess)
            return cleanup(hip_fail(e, "occupancy query"));
        // RTNW_BLOCKS_PER_CU caps the resident workgroups per CU (occupancy experiments only)
        if (const char *e = std::getenv("RTNW_BLOCKS_PER_CU")) bpc = std::min(bpc, std::max(1, std::atoi(e)));
        s->grid[mode] = std::max(1, bpc) * s->cus;
    }
    // LDS-resident BVH2 (rt_kernel.h): nodes as 4 planes + one stack per lane of the
    // scene's own depth, if both fit the CU's LDS beside the variant's static arrays.
    // RTNW_LDS_BVH=0 keeps the nodes in HBM (A/B, tests).  Primitive heads in LDS as
    // well (with 16-bit stack entries to make room) measured no faster: 60.27 vs
    // 60.29 ms on c4, both behind 32-bit entries with the nodes alone.
    {
        s->stack_depth = s->bvh_depth + 1;
        // the variant this scene launches (its static arrays and node layout: rt_lds_need_bytes)
        const long need_actual = rt_lds_need_bytes(scene_features(s), s->stack_depth);
        bool want = true;
        if (const char *e = std::getenv("RTNW_LDS_BVH")) want = std::atoi(e) != 0;
        // the budget is this device's LDS per CU (160 KiB on gfx950), and the static part
        // the compiled variant's own (hipFuncGetAttributes) if larger than the estimate:
        // a scene that does not fit keeps its nodes in HBM instead of failing to launch
        int lds_cu = RT_LDS_BUDGET;
        if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess ||
            lds_cu <= 0)
            lds_cu = 0;
        s->lds_nodes = want && !s->scan && s->bvh_width == 2 && s->has_bvh && !(s->root & RT_LEAF_BIT) &&
                       s->nnodes <= RT_LDS_NODE_CAP && d->nprims < RT_LDS_MAX_PRIMS &&
                       need_actual <= std::min<long>(RT_LDS_BUDGET, lds_cu);
        if (s->lds_nodes)
            for (int mode = 0; mode < 3; mode++) s->grid[mode] = s->cus;
    }
    trace("device attributes");
    // the work counter (64 B) and the statistics counters in one allocation
    if ((e = hipMalloc(&s->counter, 64 + RT_STATS_LEN * sizeof(unsigned long long))) != hipSuccess)
        return cleanup(hip_fail(e, "hipMalloc counters"));
    s->stats = (uint8_t *)s->counter + 64;
    trace("counters");
    for (auto &ev : s->ev)
        if ((e = hipEventCreate(&ev)) != hipSuccess) return cleanup(hip_fail(e, "hipEventCreate"));
    trace("events");
    // the scene's own stream (rt_render_tile's host-buffer path) is created on first
    // use: creating a stream next to a framework's can take milliseconds
    *out = s;
    return RT_OK;
}

// Waves per LDS workgroup that gather the medium cell's paths (rt_kernel.hip stage 6);
// env RTNW_BALL_WAVES (0: none) for A/B runs.  Their ready batch (RTNW_BALL_BATCH) and the
// busy lanes below which they claim new samples (RTNW_BALL_CLAIM): 56 and 48 against 48 and
// 64, c4 48.87 -> 48.50 ms, the share of 8 25.20 -> 25.05 ms (profiles/r06/knobs3_ab.log).
#define RT_BALL_WAVES 3
#define RT_BALL_BATCH 56
#define RT_BALL_CLAIM 48
static int env_int(const char *name, int dflt, int lo, int hi) {
    if (const char *e = std::getenv(name)) return std::max(lo, std::min(hi, std::atoi(e)));
    return dflt;
}
static int ball_waves() {
    if (const char *e = std::getenv("RTNW_BALL_WAVES")) return std::max(0, std::min(RT_LDS_BLOCK / 64, std::atoi(e)));
    return RT_BALL_WAVES;
}

// Small claims per wave at the end of a launch (render_tiles' claim sizes).
#define RT_TAIL_CLAIMS 32

// Partial-sum slab budget per launch (bytes; env RTNW_SLAB_BUDGET overrides, for tests).
// A job whose slab would be larger runs as several launches over sample batches.
// 16 GiB of the 288 GiB HBM: config 5 on one GPU (1e9 samples, 12 GB) is one launch,
// one launch-end drain; 8 GiB made it two.
#define RT_SLAB_BUDGET (16ull << 30)
static uint64_t slab_budget() {
    if (const char *e = std::getenv("RTNW_SLAB_BUDGET")) {
        const unsigned long long v = std::strtoull(e, nullptr, 10);
        if (v > 0) return v;
    }
    return RT_SLAB_BUDGET;
}

// Job pixel order: tiles in the order given; inside a tile, bands of 8 rows listed
// column by column (8 pixels per column), so that ANY 64 consecutive items — a wave
// claim, wherever it starts — are 8 neighbouring columns of one band (coherent
// primary rays), also when the tile width is not a multiple of 8 (500 = 62.5 x 8).
static bool deep_pixel(const rt_scene *s, const rt_camera_desc *cam, int x, int y, int nx, int ny) {
    // the pixel centre's primary ray (main.cpp:305-306, camera.h:52-55 without jitter or lens)
    const float u = (x + 0.5f) / nx, v = (ny - 1 - y + 0.5f) / ny;
    float o[3], d[3];
    for (int k = 0; k < 3; k++) {
        o[k] = cam->origin[k];
        d[k] = cam->lower_left_corner[k] + u * cam->horizontal[k] + v * cam->vertical[k] - o[k];
    }
    for (size_t b = 0; b + 3 < s->deep_balls.size(); b += 4) {
        const float *c = &s->deep_balls[b];
        const double oc[3] = {o[0] - (double)c[0], o[1] - (double)c[1], o[2] - (double)c[2]};
        const double a = (double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2];
        const double bb = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
        const double cc = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - (double)c[3] * c[3];
        if (bb * bb - a * cc > 0 && (bb < 0 || cc < 0)) return true;
    }
    return false;
}

static int prepare_job(rt_scene *s, const int32_t *tiles, int ntiles, int nx, int ny, const rt_camera_desc *cam) {
    std::vector<int32_t> key(tiles, tiles + 4 * ntiles);
    // the deep-first order depends on the camera: its rays' frame joins the cache key
    bool deep_first = !s->deep_balls.empty();
    if (const char *e = std::getenv("RTNW_DEEP_FIRST")) deep_first = deep_first && std::atoi(e) != 0;
    key.push_back(nx);
    key.push_back(ny);
    key.push_back(deep_first ? 1 : 0);
    if (deep_first) {
        const float *cf[4] = {cam->origin, cam->lower_left_corner, cam->horizontal, cam->vertical};
        for (const float *f : cf)
            for (int k = 0; k < 3; k++) { int32_t b; std::memcpy(&b, &f[k], 4); key.push_back(b); }
    }
    if (key == s->job_tiles && s->job_xy) return RT_OK;
    std::vector<uint32_t> xy, oi;
    uint32_t base = 0;
    for (int t = 0; t < ntiles; t++) {
        const int x0 = tiles[4 * t], y0 = tiles[4 * t + 1], w = tiles[4 * t + 2], h = tiles[4 * t + 3];
        if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > nx || y0 + h > ny || nx > 65535 || ny > 65535)
            return fail(RT_ERR_INVALID, "tile outside the image");
        for (int by = 0; by < h; by += 8)
            for (int xx = 0; xx < w; xx++)
                for (int yy = by; yy < std::min(by + 8, h); yy++) {
                    xy.push_back((uint32_t)(x0 + xx) | ((uint32_t)(y0 + yy) << 16));
                    oi.push_back(base + (uint32_t)(yy * w + xx));
                }
        base += (uint32_t)(w * h);
    }
    // deep pixels first, each group in the band order above (a claim of 64 consecutive
    // items stays 64 neighbouring pixels of one group)
    uint32_t ndeep = 0;
    if (deep_first) {
        std::vector<uint32_t> dxy, doi, rxy, roi;
        for (size_t i = 0; i < xy.size(); i++) {
            const bool deep = deep_pixel(s, cam, (int)(xy[i] & 0xFFFFu), (int)(xy[i] >> 16), nx, ny);
            (deep ? dxy : rxy).push_back(xy[i]);
            (deep ? doi : roi).push_back(oi[i]);
        }
        ndeep = (uint32_t)dxy.size();
        if (ndeep == xy.size()) ndeep = 0;   // all deep: one group
        dxy.insert(dxy.end(), rxy.begin(), rxy.end());
        doi.insert(doi.end(), roi.begin(), roi.end());
        xy.swap(dxy);
        oi.swap(doi);
    }
    if (s->job_xy) { (void)hipFree(s->job_xy); s->job_xy = nullptr; }
    if (s->job_out) { (void)hipFree(s->job_out); s->job_out = nullptr; }
    s->job_tiles.clear();
    if (int rc = upload(&s->job_xy, xy)) return rc;
    if (int rc = upload(&s->job_out, oi)) return rc;
    s->npix = (uint32_t)xy.size();
    s->job_ndeep = ndeep;
    s->job_tiles = key;
    return RT_OK;
}

int rt_render_tiles(rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p, const int32_t *tiles, int ntiles,
                    float *out_dev, void *stream_v, rt_stats *stats) {
    if (!s || !cam || !p || ntiles < 0) return fail(RT_ERR_INVALID, "rt_render_tiles: bad argument");
    if (ntiles == 0) {   // a rank with no tiles (more ranks than tiles) has nothing to do
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    if (!tiles || !out_dev) return fail(RT_ERR_INVALID, "rt_render_tiles: null tiles or output");
    if (p->nx <= 0 || p->ny <= 0 || p->spp <= 0 || p->max_depth < 0) return fail(RT_ERR_INVALID, "bad render parameters");
    if (s->has_moving && (cam->time0 < s->time0 || cam->time1 > s->time1))
        return fail(RT_ERR_INVALID, "camera shutter outside the scene's time span (moving-sphere bounds)");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t stream = (hipStream_t)stream_v;
    if (int rc = prepare_job(s, tiles, ntiles, p->nx, p->ny, cam)) return rc;

    // Work item = `chunk` samples of one pixel, one by default: short items keep each
    // wave's lanes on neighbouring pixels (a wave deals its claims to lanes as they free
    // up; long items let its pixels drift apart): 16 -> 1 sample per item is 92.2 ->
    // 81.8 ms on c4.  The partial-sum slab holds one rgb (12 B) per item
    // of a launch; a job whose slab would pass the budget runs as several launches
    // over sample batches (whole chunks), and the resolve adds every batch to a
    // per-pixel running sum in sample order — so the sum is the same sequence of
    // float adds whatever the batch size, i.e. the image does not depend on the job's
    // size (one GPU or a rank's share of eight).
    const int chunk = p->chunk > 0 ? p->chunk : 1;
    const uint64_t nchunks_total = ((uint64_t)p->spp + chunk - 1) / chunk;
    const uint64_t max_items = 0xFFFFFFFFull - 64;
    if ((uint64_t)s->npix > max_items) return fail(RT_ERR_INVALID, "job too large (pixels >= 2^32)");
    const uint64_t item_bytes = 4 * (uint64_t)rt_slab_floats();   // one partial sum (rgb)
    uint64_t per = std::max<uint64_t>(1, slab_budget() / ((uint64_t)s->npix * item_bytes));
    per = std::min<uint64_t>(per, max_items / s->npix);
    per = std::min<uint64_t>(per, nchunks_total);
    const uint64_t nbatches = (nchunks_total + per - 1) / per;
    per = (nchunks_total + nbatches - 1) / nbatches;   // batches of (nearly) equal size, as many
    const size_t slab_bytes = (size_t)s->npix * per * item_bytes;
    if (slab_bytes > s->slab_bytes) {
        if (s->slab) (void)hipFree(s->slab);
        s->slab = nullptr;
        s->slab_bytes = 0;
        HIP_TRY(hipMalloc(&s->slab, slab_bytes));
        s->slab_bytes = slab_bytes;
    }
    const size_t acc_bytes = nbatches > 1 ? (size_t)s->npix * 16 : 0;
    if (acc_bytes > s->acc_bytes) {
        if (s->acc) (void)hipFree(s->acc);
        s->acc = nullptr;
        s->acc_bytes = 0;
        HIP_TRY(hipMalloc(&s->acc, acc_bytes));
        s->acc_bytes = acc_bytes;
    }
    const bool count = (p->flags & RT_FLAG_COUNT) != 0;
    const bool prof = !count && (p->flags & RT_FLAG_PROFILE) != 0;
    const bool sum_in = (p->flags & RT_FLAG_SUM_IN) != 0, sum_out = (p->flags & RT_FLAG_SUM_OUT) != 0;
    const int mode = count ? 1 : (prof ? 2 : 0);
    if (count || prof) HIP_TRY(hipMemsetAsync(s->stats, 0, RT_STATS_LEN * sizeof(unsigned long long), stream));

    RtKernelArgs a{};
    a.nodes = (const float4 *)s->nodes;
    a.prims = (const float4 *)s->prims;
    a.bprims = (const float4 *)s->bprims;
    a.media = (const int4 *)s->media;
    a.mats = (const float4 *)s->mats;
    a.texs = (const float4 *)s->texs;
    a.insts = (const float4 *)s->insts;
    a.ranvec = (const float4 *)s->ranvec;
    a.perm = (const int *)s->perm;
    a.texels = (const uint8_t *)s->texels;
    a.root = s->root;
    a.nnodes = (uint32_t)s->nnodes;
    a.bvh_width = s->bvh_width;
    a.has_bvh = s->has_bvh;
    a.nmedia = s->nmedia;
    a.need_dlen = s->nmedia > 0 || s->has_specular || p->background == RT_BG_SKY;
    a.lds_nodes = s->lds_nodes ? 1 : 0;
    a.scan = s->scan ? 1 : 0;
    a.groups = (const float4 *)s->groups;
    a.ngroups = s->ngroups;
    a.nprescan = s->nprescan;
    a.cell_first = s->cell_first;
    a.cell_n = s->cell_n;
    for (int k = 0; k < 3; k++) a.cell_c[k] = s->cell_c[k];
    a.cell_r2 = s->cell_r2;
    a.cell_rin2 = s->cell_rin2;
    a.ball_waves = ball_waves();
    a.ball_batch = env_int("RTNW_BALL_BATCH", RT_BALL_BATCH, 1, 64);
    a.ball_claim = env_int("RTNW_BALL_CLAIM", RT_BALL_CLAIM, 1, 64);
    a.ball_park = env_int("RTNW_BALL_PARK", 1, 0, 1);
    a.ball_drain = env_int("RTNW_BALL_DRAIN", 1, 0, 1);
    a.nprims = (uint32_t)s->nprims;
    a.stack_depth = s->stack_depth;
    a.features = scene_features(s);
    for (int k = 0; k < 3; k++) {
        a.org[k] = cam->origin[k];
        a.llc[k] = cam->lower_left_corner[k];
        a.hor[k] = cam->horizontal[k];
        a.ver[k] = cam->vertical[k];
        a.cu[k] = cam->u[k];
        a.cv[k] = cam->v[k];
    }
    a.lens = cam->lens_radius;
    a.ct0 = cam->time0;
    a.ct1 = cam->time1;
    a.nx = p->nx;
    a.ny = p->ny;
    a.rnx = 1.0f / (float)p->nx;   // nx, ny >= 1: normal reciprocals (div_rn, rt_device.h)
    a.rny = 1.0f / (float)p->ny;
    a.ns = p->spp;
    a.max_depth = p->max_depth;
    a.tmin = p->t_min;
    a.background = p->background;
    a.chunk = chunk;
    a.seed = p->seed;
    a.job_xy = (const uint32_t *)s->job_xy;
    a.npix = s->npix;
    a.slab = (float *)s->slab;
    a.counter = (uint32_t *)s->counter;
    a.stats = (unsigned long long *)s->stats;
    // RTNW_WAVE_LOG=<file> with RT_FLAG_PROFILE: every wave's timeline appended to the
    // file as 5 uint64 (start, pool dry, end in s_memrealtime ticks, xcc << 32 | HW_ID,
    // items claimed) per wave and batch (tools/tail_probe.py --wave-log; diagnostics)
    const char *wave_log_path = prof ? std::getenv("RTNW_WAVE_LOG") : nullptr;
    unsigned long long *wave_log = nullptr;
    struct FreeOnExit {   // every return below, error paths included, frees the log buffer
        unsigned long long *&p;
        ~FreeOnExit() { if (p) (void)hipFree(p); }
    } wave_log_guard{wave_log};
    const size_t wave_log_n = (size_t)s->grid[2] * ((s->lds_nodes ? RT_LDS_BLOCK : RT_BLOCK) / 64) * RT_WAVE_LOG_WORDS;
    if (wave_log_path) {
        HIP_TRY(hipMalloc(&wave_log, wave_log_n * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(wave_log, 0, wave_log_n * sizeof(unsigned long long), stream));
    }
    a.wave_log = wave_log;

    // vec3::operator/= (vec3.h:134-141): col *= float(1.0 / ns)
    const uint32_t ns_total = sum_in ? p->sample_offset + (uint32_t)p->spp : (uint32_t)p->spp;
    const float k = (float)(1.0 / (double)(float)ns_total);
    const uint64_t waves = (uint64_t)s->grid[mode] * ((s->lds_nodes ? RT_LDS_BLOCK : RT_BLOCK) / 64);
    double kernel_ms = 0, resolve_ms = 0;
    for (uint64_t b = 0; b < nbatches; ++b) {
        const uint64_t c0 = b * per, c1 = std::min(c0 + per, nchunks_total);
        const uint64_t s0 = c0 * (uint64_t)chunk, s1 = std::min<uint64_t>(c1 * (uint64_t)chunk, (uint64_t)p->spp);
        a.ns = (int)(s1 - s0);                                   // samples of this batch
        a.sample_offset = p->sample_offset + (uint32_t)s0;       // their first sample index
        a.nchunks = (int)(c1 - c0);
        const uint64_t nitems = (uint64_t)s->npix * (c1 - c0);
        a.nitems = (uint32_t)nitems;
        a.ndeep = s->job_ndeep;
        a.ndeep_items = (uint32_t)((uint64_t)s->job_ndeep * (c1 - c0));
        // Claim size: up to 512 items per atomic (64 -> 512 is 81.6 -> 76.9 ms on c4:
        // fewer round trips to the one contended counter), at least 8
        // claims per wave so that small jobs still spread over every wave.
        // The last RT_TAIL_CLAIMS claims per wave are of 64 items: with 512-item claims
        // to the end, the waves ran dry over 2.4 ms (the first found the pool empty at
        // 54.1 ms of a 57.1-ms launch, the last at 56.5; with 64-item claims over 0.5 ms,
        // but every claim is a round trip to the one device-scope counter:
        // tools/tail_probe.py).
        {
            uint64_t c = std::min<uint64_t>(std::max<uint64_t>(nitems / (waves * 8) / 64 * 64, 64), 512);
            uint64_t tail = 64 * RT_TAIL_CLAIMS * waves;
            if (const char *e = std::getenv("RTNW_CLAIM")) c = (uint64_t)std::max(1, std::atoi(e)) * 64;   // x 64 items
            if (const char *e = std::getenv("RTNW_TAIL_CLAIMS")) tail = 64 * (uint64_t)std::max(0, std::atoi(e)) * waves;
            a.claim = (uint32_t)c;
            a.claim_tail = 64;
            a.nbig = (uint32_t)(nitems > tail ? (nitems - tail) / c : 0);
        }
        const int rmode = (b == 0 ? RT_RESOLVE_FIRST : 0) | (b + 1 == nbatches ? RT_RESOLVE_LAST : 0) |
                          (sum_in ? RT_RESOLVE_SUM_IN : 0) | (sum_out ? RT_RESOLVE_RAW : 0);
        HIP_TRY(hipMemsetAsync(s->counter, 0, 64, stream));
        // the wave timeline describes the last batch: its slots start from zero each launch
        if (prof)
            HIP_TRY(hipMemsetAsync((unsigned long long *)s->stats + RT_STAT_TIME, 0, 7 * sizeof(unsigned long long), stream));
        HIP_TRY(hipEventRecord(s->ev[0], stream));
        HIP_TRY(rt_launch_megakernel(&a, s->grid[mode], mode, stream));
        HIP_TRY(hipEventRecord(s->ev[1], stream));
        HIP_TRY(rt_launch_resolve((const float *)s->slab, s->npix, a.nchunks, k, (float4 *)s->acc, rmode,
                                  (const uint32_t *)s->job_out, out_dev, stream));
        HIP_TRY(hipEventRecord(s->ev[2], stream));
        if (wave_log) {
            std::vector<unsigned long long> h(wave_log_n);   // the render stream may be non-blocking
            HIP_TRY(hipMemcpyAsync(h.data(), wave_log, h.size() * sizeof h[0], hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (FILE *f = std::fopen(wave_log_path, "ab")) {
                std::fwrite(h.data(), sizeof h[0], h.size(), f);
                std::fclose(f);
            }
        }
        if (stats) {   // one batch at a time: the events are reused
            HIP_TRY(hipEventSynchronize(s->ev[2]));
            float ms0 = 0, ms1 = 0;
            HIP_TRY(hipEventElapsedTime(&ms0, s->ev[0], s->ev[1]));
            HIP_TRY(hipEventElapsedTime(&ms1, s->ev[1], s->ev[2]));
            kernel_ms += ms0;
            resolve_ms += ms1;
        }
    }

    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->samples = (double)s->npix * (double)p->spp;
        stats->chunk = (double)chunk;
        stats->batches = (double)nbatches;
        stats->kernel_ms = kernel_ms;
        stats->resolve_ms = resolve_ms;
        if (count) {
            unsigned long long c[RT_CNT_N];
            HIP_TRY(hipMemcpy(c, s->stats, sizeof c, hipMemcpyDeviceToHost));
            stats->samples = (double)c[RT_CNT_SAMPLES];
            stats->segments = (double)c[RT_CNT_SEGMENTS];
            stats->node_visits = (double)c[RT_CNT_NODES];
            stats->sphere_tests = (double)c[RT_CNT_SPHERES];
            stats->moving_sphere_tests = (double)c[RT_CNT_MSPHERES];
            stats->rect_tests = (double)c[RT_CNT_RECTS];
            stats->instanced_tests = (double)c[RT_CNT_INSTANCED];
            stats->medium_tests = (double)c[RT_CNT_MEDIA];
            stats->shades = (double)c[RT_CNT_SHADES];
            stats->noise_evals = (double)c[RT_CNT_NOISE];
            stats->algorithmic_bytes = algorithmic_bytes(*stats, (double)s->npix * (double)nchunks_total, s->bvh_width);
            unsigned long long w[5];
            HIP_TRY(hipMemcpy(w, (unsigned long long *)s->stats + RT_STAT_WAVE, sizeof w, hipMemcpyDeviceToHost));
            stats->wave_iterations = (double)w[0];
            stats->wave_node_trips = (double)w[1];
            stats->wave_prim_trips = (double)w[2];
            stats->wave_sphere_draw_trips = (double)w[3];
            stats->lane_sphere_draw_trips = (double)w[4];
            unsigned long long sh[3];
            HIP_TRY(hipMemcpy(sh, (unsigned long long *)s->stats + RT_STAT_SHADE, sizeof sh, hipMemcpyDeviceToHost));
            stats->wave_shade_passes = (double)sh[0];
            stats->wave_shade_kinds = (double)sh[1];
            stats->lane_scatters = (double)sh[2];
            if (std::getenv("RTNW_TRACE")) {   // the ball waves (rt_kernel.hip stage 6), diagnostics only
                unsigned long long b[RT_BALL_N];
                HIP_TRY(hipMemcpy(b, (unsigned long long *)s->stats + RT_STAT_BALL, sizeof b, hipMemcpyDeviceToHost));
                std::fprintf(stderr,
                             "rtnw ball waves: iterations %llu, live lanes / iteration %.1f, traversal rounds / iteration %.2f, "
                             "cell-decided segments in ball waves %llu, pushes refused (pool full) %llu (of %.0f segments), pushed in %llu, "
                             "pushed out %llu, taken %llu\n",
                             b[RT_BALL_ITERS], b[RT_BALL_ITERS] ? (double)b[RT_BALL_LIVE] / b[RT_BALL_ITERS] : 0.0,
                             b[RT_BALL_ITERS] ? (double)b[RT_BALL_ROUNDS] / b[RT_BALL_ITERS] : 0.0, b[RT_BALL_CELL_BALL],
                             b[RT_BALL_DENIED], stats->segments, b[RT_BALL_PUSH_IN], b[RT_BALL_PUSH_OUT], b[RT_BALL_TAKEN]);
            }
        }
        if (prof) {
            unsigned long long c[RT_STATS_LEN];
            HIP_TRY(hipMemcpy(c, s->stats, sizeof c, hipMemcpyDeviceToHost));
            if (std::getenv("RTNW_TRACE")) {   // the ball waves' share of the stage cycles (diagnostics only)
                const unsigned long long *b = c + RT_STAT_BALL;
                std::fprintf(stderr,
                             "rtnw ball waves (profile): iterations %llu of %llu; cycles claim %llu of %llu, traverse %llu of "
                             "%llu, media %llu of %llu, shade %llu of %llu\n",
                             b[4], b[5], b[0], c[RT_STAT_PROF], b[1], c[RT_STAT_PROF + 1], b[2], c[RT_STAT_PROF + 2], b[3],
                             c[RT_STAT_PROF + 3]);
            }
            stats->cycles_claim = (double)c[RT_STAT_PROF + 0];
            stats->cycles_traverse = (double)c[RT_STAT_PROF + 1];
            stats->cycles_media = (double)c[RT_STAT_PROF + 2];
            stats->cycles_shade = (double)c[RT_STAT_PROF + 3];
            stats->cycles_scatter = (double)c[RT_STAT_SHADE + 3];
            // wave timeline of the last batch, s_memrealtime at 100 MHz (kernel: kProf)
            const unsigned long long *T = c + RT_STAT_TIME;
            const double t0 = (double)~T[0], us = 0.01;
            stats->wave_exhaust_first_us = ((double)~T[1] - t0) * us;
            stats->wave_exhaust_last_us = ((double)T[2] - t0) * us;
            stats->wave_end_first_us = ((double)~T[3] - t0) * us;
            stats->wave_end_last_us = ((double)T[4] - t0) * us;
            stats->wave_end_mean_us = T[6] ? (double)T[5] / (double)T[6] * us : 0.0;   // T[5]: sum of lifetimes
        }
        stats->grid = (double)s->grid[mode];
        stats->lds_level = s->lds_nodes ? 1.0 : 0.0;
        stats->scan_groups = s->scan ? (double)s->ngroups : 0.0;
        stats->prescan = (double)s->nprescan;
        stats->stack_depth = (double)(s->lds_nodes ? s->stack_depth : s->bvh_width >= 8 ? RT_STACK_DEPTH_W8 : RT_STACK_DEPTH);
    }
    return RT_OK;
}

int rt_render_tile(rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p, int x0, int y0, int w, int h,
                   float *out_rgb, rt_stats *stats) {
    if (!s || !out_rgb) return fail(RT_ERR_INVALID, "rt_render_tile: bad argument");
    HIP_TRY(hipSetDevice(s->device));
    const size_t bytes = (size_t)w * h * 3 * sizeof(float);
    if (w <= 0 || h <= 0) return fail(RT_ERR_INVALID, "empty tile");
    if (bytes > s->host_out_bytes) {
        if (s->host_out) (void)hipFree(s->host_out);
        s->host_out = nullptr;
        s->host_out_bytes = 0;
        HIP_TRY(hipMalloc(&s->host_out, bytes));
        s->host_out_bytes = bytes;
    }
    if (!s->own_stream) HIP_TRY(hipStreamCreateWithFlags(&s->own_stream, hipStreamNonBlocking));
    const int32_t tile[4] = {x0, y0, w, h};
    if (p && (p->flags & RT_FLAG_SUM_IN))   // the running sums come from the caller's buffer
        HIP_TRY(hipMemcpyAsync(s->host_out, out_rgb, bytes, hipMemcpyHostToDevice, s->own_stream));
    rt_stats local;
    if (int rc = rt_render_tiles(s, cam, p, tile, 1, (float *)s->host_out, s->own_stream, stats ? stats : &local)) return rc;
    HIP_TRY(hipMemcpyAsync(out_rgb, s->host_out, bytes, hipMemcpyDeviceToHost, s->own_stream));
    HIP_TRY(hipStreamSynchronize(s->own_stream));
    return RT_OK;
}

// ---------------------------------------------------------------- resolve
void rt_quantize(const float *mean, int64_t n, uint8_t *rgb) {   // main.cpp:316-325
    for (int64_t q = 0; q < n; q++) {
        for (int k = 0; k < 3; k++) {
            const float c = std::sqrt(mean[3 * q + k]);
            int iv = int(255.99 * c);
            iv = iv > 255 ? 255 : iv;
            rgb[3 * q + k] = (uint8_t)iv;
        }
    }
}

int64_t rt_ppm_text(const uint8_t *rgb, int nx, int ny, char *buf, int64_t cap) {   // main.cpp:297, 327-330
    std::string s = "P3\n" + std::to_string(nx) + " " + std::to_string(ny) + "\n255\n";
    for (int64_t q = 0; q < (int64_t)nx * ny; q++)
        s += std::to_string(rgb[3 * q]) + " " + std::to_string(rgb[3 * q + 1]) + " " + std::to_string(rgb[3 * q + 2]) + "\n";
    if (buf && cap >= (int64_t)s.size()) std::memcpy(buf, s.data(), s.size());
    return (int64_t)s.size();
}

// ------------------------------------------------ checkpoint / resume
// File = rt_checkpoint header, `count` floats (the per-pixel sums as rt_render_tiles
// packs them), FNV-1a 64 of those bytes.  Written to <path>.tmp, then renamed, so a
// crash leaves either the previous checkpoint or the new one, never a torn file (the
// reference's row-by-row PPM write, main.cpp:330, leaves a truncated image).
static uint64_t fnv1a(const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}

int rt_checkpoint_write(const char *path, const rt_checkpoint *hdr, const float *sums) {
    if (!path || !hdr || (!sums && hdr->count)) return fail(RT_ERR_INVALID, "rt_checkpoint_write: null argument");
    rt_checkpoint h = *hdr;
    h.magic = RT_CHECKPOINT_MAGIC;
    h.version = RT_CHECKPOINT_VERSION;
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return fail(RT_ERR_INVALID, std::string("cannot open ") + tmp);
    const size_t bytes = (size_t)h.count * sizeof(float);
    const uint64_t sum = fnv1a(sums, bytes);
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && (bytes == 0 || std::fwrite(sums, 1, bytes, f) == bytes) &&
              std::fwrite(&sum, sizeof sum, 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        return fail(RT_ERR_INVALID, std::string("cannot write checkpoint ") + path);
    }
    return RT_OK;
}

int rt_checkpoint_read(const char *path, rt_checkpoint *hdr, float *sums, uint64_t cap) {
    if (!path || !hdr) return fail(RT_ERR_INVALID, "rt_checkpoint_read: null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(RT_ERR_INVALID, std::string("cannot open ") + path);
    rt_checkpoint h;
    int rc = RT_OK;
    // the file's own size bounds `count` before anyone sizes a buffer by it: header +
    // count floats + the 8-byte checksum, and count = 3 x (pixels of a job <= nx x ny)
    long fsize = -1;
    if (std::fseek(f, 0, SEEK_END) == 0) fsize = std::ftell(f);
    std::rewind(f);
    if (std::fread(&h, sizeof h, 1, f) != 1 || h.magic != RT_CHECKPOINT_MAGIC || h.version != RT_CHECKPOINT_VERSION) {
        rc = fail(RT_ERR_INVALID, std::string("not a checkpoint: ") + path);
    } else if (h.nx <= 0 || h.ny <= 0 || h.count % 3 != 0 || h.count > 3ull * (uint64_t)h.nx * (uint64_t)h.ny ||
               fsize < (long)(sizeof h + sizeof(uint64_t)) ||
               // the payload's size by division: count * 4 would wrap for a crafted count
               ((uint64_t)fsize - sizeof h - sizeof(uint64_t)) % sizeof(float) != 0 ||
               ((uint64_t)fsize - sizeof h - sizeof(uint64_t)) / sizeof(float) != h.count) {
        rc = fail(RT_ERR_INVALID, std::string("corrupt checkpoint header (count / image size / file size): ") + path);
    } else if (sums) {   // sums == NULL: header only (to size the buffer)
        if (h.count > cap) {
            rc = fail(RT_ERR_INVALID, "checkpoint larger than the buffer");
        } else {
            const size_t bytes = (size_t)h.count * sizeof(float);
            uint64_t sum = 0;
            if ((bytes && std::fread(sums, 1, bytes, f) != bytes) || std::fread(&sum, sizeof sum, 1, f) != 1)
                rc = fail(RT_ERR_INVALID, std::string("truncated checkpoint: ") + path);
            else if (sum != fnv1a(sums, bytes))
                rc = fail(RT_ERR_INVALID, std::string("checkpoint checksum mismatch: ") + path);
        }
    }
    std::fclose(f);
    if (rc == RT_OK) *hdr = h;
    return rc;
}

// ------------------------------------------------------- host scene building
static std::mutex g_desc_mu;
static std::map<const rt_scene_desc *, std::unique_ptr<rtnw::flat_scene>> g_descs;

int rt_builtin_scene_desc(const char *name, rt_scene_desc **out) {
    if (!name || !out) return fail(RT_ERR_INVALID, "rt_builtin_scene_desc: null argument");
    std::lock_guard<std::mutex> lk(g_desc_mu);
    float t0, t1;
    rtnw::hitable *world = rtnw::build_named_scene(name, &t0, &t1);
    if (!world) return fail(RT_ERR_INVALID, std::string("unknown scene: ") + name);
    std::unique_ptr<rtnw::flat_scene> fs;
    try {
        fs = rtnw::flatten_world(world, t0, t1);
    } catch (const std::exception &ex) {
        return fail(RT_ERR_UNSUPPORTED, ex.what());
    }
    *out = &fs->desc;
    g_descs[&fs->desc] = std::move(fs);
    return RT_OK;
}

void rt_scene_desc_free(rt_scene_desc *d) {
    std::lock_guard<std::mutex> lk(g_desc_mu);
    g_descs.erase(d);
}

int64_t rt_scene_desc_dump(const rt_scene_desc *d, char *buf, int64_t cap) {
    if (!d) return fail(RT_ERR_INVALID, "null descriptor");
    const std::string s = rtnw::dump_desc(d);
    if (buf && cap >= (int64_t)s.size()) std::memcpy(buf, s.data(), s.size());
    return (int64_t)s.size();
}

}  // extern "C"
