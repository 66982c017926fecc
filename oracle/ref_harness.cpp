// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Builds the *unmodified* reference renderer from the sources where they lie
// (/root/reference/Peter-Shirley-Project Code/main.cpp and its headers) and wraps
// it in a parameterised driver so the reference itself can serve as the oracle:
//
//   * `int main()` of main.cpp is renamed with a macro before the #include so this
//     file can provide its own CLI driver (the reference's main is not called).
//   * The pixel loop below follows main.cpp:299-332 (jitter, get_ray, color,
//     de_nan, `col += temp`, `col /= float(ns)`, sqrt gamma, int(255.99*c), clamp).
//   * `color()` of main.cpp:25-46 is called as-is for black-background depth-50
//     t_min=0.001 configs; a sky-background / other-depth variant (`color_ex`) is
//     restated here for configs c1/c3 (miss branch of TNW/Chapter03:29-31).
//   * RNG instrumentation: this executable defines `drand48` itself, so every call
//     the reference makes resolves here.  In "canonical" mode it is glibc's own
//     generator (erand48 on a private state that starts at 0, exactly the state
//     an unseeded glibc drand48 starts from).  In "counter" mode each camera sample
//     draws from its own counter-keyed stream (the spec shared with the GPU kernel,
//     see DESIGN.md §RNG), and constant_medium draws come from a (sample, bounce,
//     medium) keyed stream — selected by wrapping each medium in `medium_tag`.
//
// Nothing from the reference is copied into the repository; outputs go to
// oracle/_ref/ (git-ignored).  Build recipe: oracle/Makefile.

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <string>
#include <vector>
#include <unistd.h>



#define main psrt_reference_main_unused
#include "main.cpp"
#undef main

// ---------------------------------------------------------------- RNG plumbing
static unsigned short g_canon_state[3] = {0, 0, 0};
static int g_mode = 0;            // 0 canonical, 1 counter
static uint64_t g_key = 0;        // counter mode: per-sample stream key
static uint64_t g_x = 0;          // counter mode: the sample's drand48 state (restarted at key mod 2^48)
static int g_med_ctx = -1;        // >=0 while a constant_medium (ordinal k) is being hit
static int g_bounce = 0;          // top-level world->hit calls in this sample
static int g_nmedia = 0;          // constant_media in the scene (tag_media's count)

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t sample_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return mix64(mix64(seed ^ 0x5851F42D4C957F2Dull) ^ (((uint64_t)pixel << 32) | sample));
}

extern "C" double drand48(void) noexcept {
    if (g_mode == 0) return erand48(g_canon_state);
    if (g_med_ctx >= 0) {
        // the medium stream: drand48's generator from mix64(key ^ ..) mod 2^48, stepped
        // once per medium and segment; this draw is its (bounce * nmedia + k + 1)-th value
        uint64_t x = mix64(g_key ^ 0xD1B54A32D192ED03ull) & 0xFFFFFFFFFFFFull;
        const uint64_t n = (uint64_t)g_bounce * (uint64_t)g_nmedia + (uint64_t)g_med_ctx + 1;
        for (uint64_t i = 0; i < n; i++) x = (0x5DEECE66Dull * x + 0xBull) & 0xFFFFFFFFFFFFull;
        return (double)x * 0x1p-48;
    }
    // drand48's own step on the sample's state (x = a x + c mod 2^48, x / 2^48)
    g_x = (0x5DEECE66Dull * g_x + 0xBull) & 0xFFFFFFFFFFFFull;
    return (double)g_x * 0x1p-48;
}

// -------------------------------------------------------- instrumentation nodes
struct medium_tag : public hitable {
    hitable *inner; int k;
    medium_tag(hitable *h, int ordinal) : inner(h), k(ordinal) {}
    virtual bool hit(const ray &r, float a, float b, hit_record &rec) const {
        int prev = g_med_ctx; g_med_ctx = k;
        bool h = inner->hit(r, a, b, rec);
        g_med_ctx = prev;
        return h;
    }
    virtual bool bounding_box(float t0, float t1, aabb &box) const { return inner->bounding_box(t0, t1, box); }
};

struct bounce_counter : public hitable {
    hitable *inner; int *bounce_out;
    explicit bounce_counter(hitable *h) : inner(h) {}
    virtual bool hit(const ray &r, float a, float b, hit_record &rec) const {
        bool h = inner->hit(r, a, b, rec);
        g_bounce++;
        return h;
    }
    virtual bool bounding_box(float t0, float t1, aabb &box) const { return inner->bounding_box(t0, t1, box); }
};

// Replace every constant_medium reachable through lists / wrappers by a tagged
// proxy, numbering media in depth-first list order (the order the flat list
// tests them in, hitable_list.h:24).
static void tag_media(hitable **slot, int &next) {
    hitable *h = *slot;
    if (auto *m = dynamic_cast<constant_medium *>(h)) { *slot = new medium_tag(m, next++); return; }
    if (auto *l = dynamic_cast<hitable_list *>(h)) { for (int i = 0; i < l->list_size; i++) tag_media(&l->list[i], next); return; }
    if (auto *f = dynamic_cast<flip_normals *>(h)) { tag_media(&f->ptr, next); return; }
    if (auto *t = dynamic_cast<translate *>(h)) { tag_media(&t->ptr, next); return; }
    if (auto *r = dynamic_cast<rotate_y *>(h)) { tag_media(&r->ptr, next); return; }
    if (auto *b = dynamic_cast<box *>(h)) { tag_media(&b->list_ptr, next); return; }
    if (auto *n = dynamic_cast<bvh_node *>(h)) { tag_media(&n->left, next); if (n->right != n->left) tag_media(&n->right, next); return; }
}

// --------------------------------------------- corrected BVH (CPU baseline only)
// The reference's bvh_node (bvh.h:29-54 hit, bvh.h:97-121 ctor: random axis, qsort by
// box.min with the reference's own comparators bvh.h:58-95, split n/2) with ONE
// change: the slab test uses the ray origin where aabb::hit (aabb.h:38-39) subtracts
// the direction.  With the bug the reference's BVH misses hits, which is why the
// shipped main renders final() as a flat list (main.cpp:291); this class gives the
// "reference with a corrected BVH" throughput figure of BASELINE.md (--accel bvh).
// Its ties go right (bvh.h:37-40), so images differ from the flat list in rare ties:
// it is a timing baseline, never a parity oracle.
static bool fixed_slab_hit(const aabb &b, const ray &r, float tmin, float tmax) {
    for (int a = 0; a < 3; a++) {   // aabb.h:33-49 with origin()
        float invD = 1.0f / r.direction()[a];
        float t0 = (b.min()[a] - r.origin()[a]) * invD;
        float t1 = (b.max()[a] - r.origin()[a]) * invD;
        if (invD < 0.0f) std::swap(t0, t1);
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax <= tmin) return false;
    }
    return true;
}
class fixed_bvh : public hitable {
public:
    fixed_bvh(hitable **l, int n, float time0, float time1) {
        int axis = int(3 * drand48());
        qsort(l, n, sizeof(hitable *), axis == 0 ? box_x_compare : (axis == 1 ? box_y_compare : box_z_compare));
        if (n == 1) left = right = l[0];
        else if (n == 2) { left = l[0]; right = l[1]; }
        else { left = new fixed_bvh(l, n / 2, time0, time1); right = new fixed_bvh(l + n / 2, n - n / 2, time0, time1); }
        aabb bl, br;
        left->bounding_box(time0, time1, bl);
        right->bounding_box(time0, time1, br);
        box = surrounding_box(bl, br);
    }
    virtual bool hit(const ray &r, float tmin, float tmax, hit_record &rec) const {
        if (!fixed_slab_hit(box, r, tmin, tmax)) return false;
        hit_record lr, rr;
        bool hl = left->hit(r, tmin, tmax, lr), hr = right->hit(r, tmin, tmax, rr);
        if (hl && hr) { rec = lr.t < rr.t ? lr : rr; return true; }
        if (hl) { rec = lr; return true; }
        if (hr) { rec = rr; return true; }
        return false;
    }
    virtual bool bounding_box(float, float, aabb &b) const { b = box; return true; }
    hitable *left, *right;
    aabb box;
};

// ------------------------------------------------------------ extra scenes
// c3: the Chapter-1 motion-blur random scene (TNW/Chapter01:36-67) expressed with
// the main.cpp texture API (checker ground main.cpp:54-57, constant textures).
// Draw order is pinned explicitly (x before y before z, left factor first), the
// order clang gives the reference's argument lists.
static hitable *random_scene_motion() {
    hitable **list = new hitable *[501];
    texture *checker = new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)),
                                           new constant_texture(vec3(0.9, 0.9, 0.9)));
    list[0] = new sphere(vec3(0, -700, 0), 700, new lambertian(checker));
    int i = 1;
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            float choose_mat = drand48();
            double dx = drand48(); double dz = drand48();
            vec3 center(a + 0.9 * dx, 0.2, b + 0.9 * dz);
            if ((center - vec3(4, 0.2, 0)).length() > 0.9) {
                if (choose_mat < 0.8) {
                    double dy = drand48();
                    vec3 c1 = center + vec3(0, 0.5 * dy, 0);
                    double r0 = drand48(); double r1 = drand48();
                    double g0 = drand48(); double g1 = drand48();
                    double b0 = drand48(); double b1 = drand48();
                    list[i++] = new moving_sphere(center, c1, 0.0, 1.0, 0.2,
                        new lambertian(new constant_texture(vec3(r0 * r1, g0 * g1, b0 * b1))));
                } else if (choose_mat < 0.95) {
                    double x = drand48(); double y = drand48(); double z = drand48();
                    double f = drand48();
                    list[i++] = new sphere(center, 0.2, new metal(vec3(0.5 * (1 + x), 0.5 * (1 + y), 0.5 * (1 + z)), 0.5 * f));
                } else {
                    list[i++] = new sphere(center, 0.2, new dielectric(1.5));
                }
            }
        }
    }
    list[i++] = new sphere(vec3(0, 1, 0), 1.0, new dielectric(2.5));
    list[i++] = new sphere(vec3(-4, 1, 0), 1.0, new lambertian(new constant_texture(vec3(0.4, 0.2, 0.1))));
    list[i++] = new sphere(vec3(4, 1, 0), 1.0, new metal(vec3(1, 1, 1), 0.0));
    return new hitable_list(list, i);
}

// ------------------------------------------------------------ integrator
static int g_bg = 0;         // 0 black, 1 sky
static int g_max_depth = 50;
static float g_tmin = 0.001f;

// main.cpp:25-46 with a configurable depth cap / t_min and the sky miss branch of
// TNW/Chapter03:29-31.  Used only when the config differs from the reference main.
static vec3 color_ex(const ray &r, hitable *world, int depth) {
    hit_record rec;
    if (world->hit(r, g_tmin, MAXFLOAT, rec)) {
        ray scattered;
        vec3 attenuation;
        vec3 emitted = rec.mat_ptr->emitted(rec.u, rec.v, rec.p);
        if (depth < g_max_depth && rec.mat_ptr->scatter(r, rec, attenuation, scattered))
            return emitted + attenuation * color_ex(scattered, world, depth + 1);
        return emitted;
    }
    if (g_bg == 1) {
        vec3 unit_direction = unit_vector(r.direction());
        float t = 0.5 * (unit_direction.y() + 1.0);
        return (1.0 - t) * vec3(1.0, 1.0, 1.0) + t * vec3(0.5, 0.7, 1.0);
    }
    return vec3(0, 0, 0);
}

// --------------------------------------------------------------- scene dump
// Writes every leaf primitive in depth-first list order with its wrappers, as
// hex floats, so the product's scene builders can be checked field by field.
static FILE *g_dump;
static std::vector<const void *> g_mats, g_texs;
static int ptr_id(std::vector<const void *> &v, const void *p) {
    for (size_t i = 0; i < v.size(); i++) if (v[i] == p) return (int)i;
    v.push_back(p); return (int)v.size() - 1;
}
static void dump_tex(const texture *t) {
    if (auto *c = dynamic_cast<const constant_texture *>(t)) { fprintf(g_dump, "(const %a %a %a)", c->color[0], c->color[1], c->color[2]); return; }
    if (auto *k = dynamic_cast<const checker_texture *>(t)) { fprintf(g_dump, "(checker even="); dump_tex(k->even); fprintf(g_dump, " odd="); dump_tex(k->odd); fprintf(g_dump, ")"); return; }
    if (auto *n = dynamic_cast<const noise_texture *>(t)) { fprintf(g_dump, "(noise %a)", n->scale); return; }
    if (auto *im = dynamic_cast<const image_texture *>(t)) {
        uint32_t h = 2166136261u;   // FNV-1a over the texels value() can address (stride 3)
        for (long b = 0; b < 3L * im->nx * im->ny; b++) h = (h ^ im->data[b]) * 16777619u;
        fprintf(g_dump, "(image %d %d %08x)", im->nx, im->ny, h);
        return;
    }
    fprintf(g_dump, "(unknown texture)");
}
static void dump_mat(const material *m) {
    fprintf(g_dump, " mat%d=", ptr_id(g_mats, m));
    if (auto *l = dynamic_cast<const lambertian *>(m)) { fprintf(g_dump, "lambertian"); dump_tex(l->albedo); return; }
    if (auto *me = dynamic_cast<const metal *>(m)) { fprintf(g_dump, "metal(%a %a %a fuzz %a)", me->albedo[0], me->albedo[1], me->albedo[2], me->fuzz); return; }
    if (auto *d = dynamic_cast<const dielectric *>(m)) { fprintf(g_dump, "dielectric(%a)", d->ref_idx); return; }
    if (auto *e = dynamic_cast<const diffuse_light *>(m)) { fprintf(g_dump, "light"); dump_tex(e->emit); return; }
    if (auto *i = dynamic_cast<const isotropic *>(m)) { fprintf(g_dump, "isotropic"); dump_tex(i->albedo); return; }
}
static void dump_node(const hitable *h, const std::string &wrap) {
    if (auto *l = dynamic_cast<const hitable_list *>(h)) { for (int i = 0; i < l->list_size; i++) dump_node(l->list[i], wrap); return; }
    if (auto *b = dynamic_cast<const box *>(h)) { dump_node(b->list_ptr, wrap); return; }
    if (auto *f = dynamic_cast<const flip_normals *>(h)) { dump_node(f->ptr, wrap + "flip "); return; }
    if (auto *t = dynamic_cast<const translate *>(h)) {
        char buf[160]; snprintf(buf, sizeof buf, "translate(%a %a %a) ", t->offset[0], t->offset[1], t->offset[2]);
        dump_node(t->ptr, wrap + buf); return; }
    if (auto *r = dynamic_cast<const rotate_y *>(h)) {
        char buf[160]; snprintf(buf, sizeof buf, "rotate_y(sin %a cos %a) ", r->sin_theta, r->cos_theta);
        dump_node(r->ptr, wrap + buf); return; }
    if (auto *n = dynamic_cast<const bvh_node *>(h)) { dump_node(n->left, wrap); dump_node(n->right, wrap); return; }
    if (auto *m = dynamic_cast<const medium_tag *>(h)) { dump_node(m->inner, wrap); return; }
    if (auto *cm = dynamic_cast<const constant_medium *>(h)) {
        fprintf(g_dump, "%smedium density %a", wrap.c_str(), cm->density); dump_mat(cm->phase_function);
        fprintf(g_dump, " boundary{\n"); dump_node(cm->boundary, "  "); fprintf(g_dump, "}\n"); return; }
    if (auto *s = dynamic_cast<const sphere *>(h)) {
        fprintf(g_dump, "%ssphere %a %a %a r %a", wrap.c_str(), s->center[0], s->center[1], s->center[2], s->radius);
        dump_mat(s->mat_ptr); fprintf(g_dump, "\n"); return; }
    if (auto *s = dynamic_cast<const moving_sphere *>(h)) {
        fprintf(g_dump, "%smoving_sphere %a %a %a -> %a %a %a t %a %a r %a", wrap.c_str(), s->center0[0], s->center0[1], s->center0[2],
                s->center1[0], s->center1[1], s->center1[2], s->time0, s->time1, s->radius);
        dump_mat(s->mat_ptr); fprintf(g_dump, "\n"); return; }
    if (auto *x = dynamic_cast<const xy_rect *>(h)) { fprintf(g_dump, "%sxy_rect %a %a %a %a k %a", wrap.c_str(), x->x0, x->x1, x->y0, x->y1, x->k); dump_mat(x->mp); fprintf(g_dump, "\n"); return; }
    if (auto *x = dynamic_cast<const xz_rect *>(h)) { fprintf(g_dump, "%sxz_rect %a %a %a %a k %a", wrap.c_str(), x->x0, x->x1, x->z0, x->z1, x->k); dump_mat(x->mp); fprintf(g_dump, "\n"); return; }
    if (auto *x = dynamic_cast<const yz_rect *>(h)) { fprintf(g_dump, "%syz_rect %a %a %a %a k %a", wrap.c_str(), x->y0, x->y1, x->z0, x->z1, x->k); dump_mat(x->mp); fprintf(g_dump, "\n"); return; }
    fprintf(g_dump, "%sunknown\n", wrap.c_str());
}

// ------------------------------------------------------------ edge scenes
// Edge cases of this build's tests, written with the reference's own classes so
// the oracle's restatement is pinned on them as on the book's scenes (the same
// three scenes: oracle/rt_oracle.c build_edge_*, csrc/host/rtnw.cpp edge_*).
static hitable *edge_empty() { return new hitable_list(new hitable *[1], 0); }
static hitable *edge_single() {
    hitable **l = new hitable *[1];
    l[0] = new sphere(vec3(0, 1, 0), 1, new lambertian(new constant_texture(vec3(0.5, 0.5, 0.5))));
    return new hitable_list(l, 1);
}
static hitable *edge_degenerate() {
    hitable **l = new hitable *[11];
    int i = 0;
    material *glass = new dielectric(1.5);
    l[i++] = new sphere(vec3(0, -1000, 0), 1000, new lambertian(new constant_texture(vec3(0.5, 0.5, 0.5))));
    l[i++] = new sphere(vec3(0, 1, 0), 0, new lambertian(new constant_texture(vec3(0.8, 0.3, 0.3))));   // zero radius
    l[i++] = new sphere(vec3(-2.5, 1, 0), -1, glass);                                                  // negative radius
    l[i++] = new sphere(vec3(2.5, 1, 0), 1, glass);                                                    // hollow bubble
    l[i++] = new sphere(vec3(2.5, 1, 0), -0.9, glass);
    l[i++] = new xz_rect(-1, -1, -1, 1, 0.5, new diffuse_light(new constant_texture(vec3(4, 4, 4))));   // zero width
    l[i++] = new moving_sphere(vec3(1, 0.5, 1.5), vec3(1, 0.5, 2), 0.5, 0.5, 0.5,                        // zero shutter span
                               new lambertian(new constant_texture(vec3(0.2, 0.8, 0.2))));
    l[i++] = new sphere(vec3(-1, 0.7, 1.5), 0.7, new metal(vec3(0.7, 0.6, 0.5), 1.5));                  // fuzz clamped to 1
    l[i++] = new constant_medium(new sphere(vec3(1, 0.5, -1.5), 0.5, glass), 0, new constant_texture(vec3(1, 1, 1)));
    l[i++] = new constant_medium(new sphere(vec3(-1, 0.5, -1.5), 0.5, glass), 1e30,
                                 new constant_texture(vec3(0.9, 0.9, 0.9)));
    l[i++] = new flip_normals(new xy_rect(-3, 3, 0, 3, -3, new diffuse_light(new constant_texture(vec3(2, 2, 2)))));
    return new hitable_list(l, i);
}

// ----------------------------------------------------------------------- CLI
static void usage() {
    fprintf(stderr,
        "ref_render --scene NAME [--nx N --ny N --ns N --depth D --bg black|sky --tmin T]\n"
        "           [--cam cornell|random|final_alt] [--rng canonical|counter --seed S]\n"
        "           [--rows J0:J1] [--ppm FILE] [--fb FILE] [--dump FILE] [--perlin FILE] [--time] [--accel flat|bvh]\n"
        "  scenes: random_scene random_motion cornell_box cornell_smoke final simple_light two_spheres test\n"
        "          edge_empty edge_single edge_degenerate (sky, random camera)\n");
    exit(2);
}

int main(int argc, char **argv) {
    std::string scene = "final", cam_name = "", bg = "", rng = "canonical", ppm, fb, dump, perlin_out, assets, accel = "flat";
    int nx = 40, ny = 40, ns = 4, depth = -1, j_lo = 0, j_hi = -1; bool timing = false;
    double tmin = 0.001; uint64_t seed = 0;
    for (int a = 1; a < argc; a++) {
        std::string k = argv[a];
        auto val = [&]() -> const char * { if (a + 1 >= argc) usage(); return argv[++a]; };
        if (k == "--scene") scene = val();
        else if (k == "--nx") nx = atoi(val());
        else if (k == "--ny") ny = atoi(val());
        else if (k == "--ns") ns = atoi(val());
        else if (k == "--depth") depth = atoi(val());
        else if (k == "--bg") bg = val();
        else if (k == "--tmin") tmin = atof(val());
        else if (k == "--cam") cam_name = val();
        else if (k == "--rng") rng = val();
        else if (k == "--seed") seed = strtoull(val(), nullptr, 0);
        else if (k == "--rows") { const char *v = val(); if (sscanf(v, "%d:%d", &j_lo, &j_hi) != 2) usage(); }
        else if (k == "--ppm") ppm = val();
        else if (k == "--fb") fb = val();
        else if (k == "--dump") dump = val();
        else if (k == "--perlin") perlin_out = val();
        else if (k == "--time") timing = true;
        else if (k == "--assets") assets = val();
        else if (k == "--accel") accel = val();
        else usage();
    }
    if (j_hi < 0) j_hi = ny;

    if (!perlin_out.empty()) {   // tables as produced by the static initialisers (perlin.h:108-111)
        FILE *f = fopen(perlin_out.c_str(), "wb");
        for (int i = 0; i < 256; i++) fwrite(perlin::ranvec[i].e, sizeof(float), 3, f);
        fwrite(perlin::perm_x, sizeof(int), 256, f);
        fwrite(perlin::perm_y, sizeof(int), 256, f);
        fwrite(perlin::perm_z, sizeof(int), 256, f);
        fclose(f);
    }

    // Scene construction consumes the canonical stream right after the Perlin
    // static initialisers, exactly as the reference program does.
    std::streambuf *saved = std::cout.rdbuf(nullptr);   // final() prints its boxes
    hitable *world = nullptr;
    bool sky_default = false; int depth_default = 50; std::string cam_default = "cornell";
    if (scene == "final") world = final();
    else if (scene == "cornell_box") world = cornell_box();
    else if (scene == "cornell_smoke") world = cornell_smoke();
    else if (scene == "random_scene") { world = random_scene(); sky_default = true; depth_default = 8; cam_default = "random"; }
    else if (scene == "random_motion") { world = random_scene_motion(); sky_default = true; cam_default = "random"; }
    else if (scene == "simple_light") { world = simple_light(); cam_default = "random"; }
    else if (scene == "two_spheres") { world = two_spheres(); cam_default = "random"; }
    else if (scene == "test") { world = test(); cam_default = "random"; }
    else if (scene == "edge_empty") { world = edge_empty(); sky_default = true; cam_default = "random"; }
    else if (scene == "edge_single") { world = edge_single(); sky_default = true; cam_default = "random"; }
    else if (scene == "edge_degenerate") { world = edge_degenerate(); sky_default = true; cam_default = "random"; }
    else if (scene == "earth") {   // stbi_load("picture.png") reads the working directory (main.cpp:93)
        if (!assets.empty() && chdir(assets.c_str()) != 0) { perror("chdir"); return 2; }
        world = earth();
    }
    else usage();
    std::cout.rdbuf(saved);

    if (!dump.empty()) {
        g_dump = fopen(dump.c_str(), "w");
        dump_node(world, "");
        fclose(g_dump);
    }

    if (accel == "bvh") {   // corrected BVH over the world's list (timing baseline only)
        auto *hl = dynamic_cast<hitable_list *>(world);
        if (!hl || rng != "canonical") usage();
        unsigned short saved_state[3];
        memcpy(saved_state, g_canon_state, sizeof saved_state);   // the samples keep their draws
        if (hl->list_size > 0) world = new fixed_bvh(hl->list, hl->list_size, 0.0f, 1.0f);
        memcpy(g_canon_state, saved_state, sizeof saved_state);
    } else if (accel != "flat") usage();

    if (bg.empty()) bg = sky_default ? "sky" : "black";
    if (depth < 0) depth = depth_default;
    if (cam_name.empty()) cam_name = cam_default;
    g_bg = (bg == "sky"); g_max_depth = depth; g_tmin = (float)tmin;
    bool use_reference_color = (g_bg == 0 && depth == 50 && g_tmin == 0.001f);

    vec3 lookfrom, lookat; float vfov, aperture, dist_to_focus = 10.0;
    if (cam_name == "cornell") { lookfrom = vec3(228, 278, -800); lookat = vec3(278, 278, 0); vfov = 40.0; aperture = 0.0; }
    else if (cam_name == "random") { lookfrom = vec3(13, 2, 3); lookat = vec3(0, 0, 0); vfov = 20; aperture = 0.1; }
    else if (cam_name == "final_alt") { lookfrom = vec3(478, 278, -600); lookat = vec3(278, 278, 0); vfov = 20; aperture = 0.0; }
    else usage();
    camera cam(lookfrom, lookat, vec3(0, 1, 0), vfov, float(nx) / float(ny), aperture, dist_to_focus, 0.0, 1.0);

    bounce_counter *counted = nullptr;
    if (rng == "counter") {
        int next = 0; tag_media(&world, next); g_nmedia = next;
        counted = new bounce_counter(world);
        world = counted;
        g_mode = 1;
    } else if (rng != "canonical") usage();

    int rows = j_hi - j_lo;
    std::vector<float> out((size_t)rows * nx * 3);
    std::string text;
    auto t0 = std::chrono::steady_clock::now();
    for (int j = j_hi - 1; j >= j_lo; j--) {            // main.cpp:299 (top row first)
        for (int i = 0; i < nx; i++) {
            vec3 col(0, 0, 0);
            for (int s = 0; s < ns; s++) {
                if (g_mode == 1) { g_key = sample_key(seed, (uint32_t)(j * nx + i), (uint32_t)s); g_x = g_key & 0xFFFFFFFFFFFFull; g_bounce = 0; }
                float u = float(i + drand48()) / float(nx);
                float v = float(j + drand48()) / float(ny);
                ray r = cam.get_ray(u, v);
                vec3 temp = use_reference_color ? color(r, world, 0) : color_ex(r, world, 0);
                temp = de_nan(temp);
                col += temp;
            }
            col /= float(ns);
            float *o = &out[((size_t)(j_hi - 1 - j) * nx + i) * 3];
            o[0] = col[0]; o[1] = col[1]; o[2] = col[2];
            col = vec3(sqrt(col[0]), sqrt(col[1]), sqrt(col[2]));
            int ir = int(255.99 * col[0]), ig = int(255.99 * col[1]), ib = int(255.99 * col[2]);
            ir = ir > 255 ? 255 : ir; ig = ig > 255 ? 255 : ig; ib = ib > 255 ? 255 : ib;
            text += std::to_string(ir) + " " + std::to_string(ig) + " " + std::to_string(ib) + "\n";
        }
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    if (!ppm.empty()) {
        FILE *f = fopen(ppm.c_str(), "w");
        fprintf(f, "P3\n%d %d\n255\n", nx, rows);
        fwrite(text.data(), 1, text.size(), f);
        fclose(f);
    }
    if (!fb.empty()) {
        FILE *f = fopen(fb.c_str(), "wb");
        fwrite(out.data(), sizeof(float), out.size(), f);
        fclose(f);
    }
    if (timing) {
        double samples = (double)rows * nx * ns;
        printf("{\"samples\": %.0f, \"seconds\": %.6f, \"samples_per_s\": %.3f}\n", samples, secs, samples / secs);
    }
    return 0;
}
