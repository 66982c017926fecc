// flatten.cpp — turns a hitable tree into the rt_scene_desc the device consumes.
//
// Leaves are emitted in depth-first list order, the order hitable_list::hit
// (hitable_list.h:24) tests them in; that order is what the device's closest-hit
// search uses to break ties, so the GPU picks the same object the reference
// picks.  Wrappers become either a per-leaf flag (a flip_normals directly around
// the leaf) or an interned transform chain (translate / rotate_y / flip between
// them), outermost first.  Materials and textures are interned by identity, as
// the reference shares them by pointer.
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>

#include "rtnw.h"

namespace rtnw {

struct flat_ctx {
    flat_scene *out;
    std::map<const material *, int> mat_ids;
    std::map<const texture *, int> tex_ids;
    std::vector<std::array<float, 4>> chain;   // current transform chain, outermost first
    int flip = 0;                              // flips since the innermost transform
    bool in_boundary = false;
    bool in_medium_scope = false;

    int material_id(const material *m) {
        auto it = mat_ids.find(m);
        if (it != mat_ids.end()) return it->second;
        const int id = m->flatten(*this);
        mat_ids[m] = id;
        return id;
    }
    int texture_id(const texture *t) {
        auto it = tex_ids.find(t);
        if (it != tex_ids.end()) return it->second;
        const int id = t->flatten(*this);
        tex_ids[t] = id;
        return id;
    }
    int add_material(const rt_material &m) { out->materials.push_back(m); return (int)out->materials.size() - 1; }
    int add_texture(const rt_texture &t) { out->textures.push_back(t); return (int)out->textures.size() - 1; }

    int intern_chain() {
        if (chain.empty()) return -1;
        if (chain.size() > 6) throw std::runtime_error("transform chain deeper than 6 wrappers");
        rt_instance in{};
        in.nops = (int32_t)chain.size();
        for (size_t i = 0; i < chain.size(); i++)
            for (int k = 0; k < 4; k++) in.ops[i][k] = chain[i][k];
        for (size_t i = 0; i < out->instances.size(); i++)
            if (std::memcmp(&out->instances[i], &in, sizeof in) == 0) return (int)i;
        out->instances.push_back(in);
        return (int)out->instances.size() - 1;
    }
    void emit(int kind, const material *m, std::initializer_list<float> p) {
        rt_prim pr{};
        pr.kind = kind;
        pr.material = material_id(m);
        pr.instance = intern_chain();
        pr.flip = flip;
        int i = 0;
        for (float v : p) pr.p[i++] = v;
        (in_boundary ? out->boundary : out->prims).push_back(pr);
    }
    // Runs `body` inside one more transform wrapper.
    template <class F>
    void wrapped(std::array<float, 4> op, F body) {
        const size_t saved = chain.size();
        const int saved_flip = flip;
        if (flip) {   // a flip between this transform and the next one out
            chain.push_back({(float)RT_OP_FLIP, 0, 0, 0});
            flip = 0;
        }
        chain.push_back(op);
        body();
        chain.resize(saved);
        flip = saved_flip;
    }
};

// ------------------------------------------------------------------ textures
int constant_texture::flatten(flat_ctx &cx) const {
    rt_texture t{};
    t.kind = RT_TEX_CONSTANT;
    t.even = t.odd = -1;
    for (int i = 0; i < 3; i++) t.color[i] = color[i];
    return cx.add_texture(t);
}
int checker_texture::flatten(flat_ctx &cx) const {
    rt_texture t{};
    t.kind = RT_TEX_CHECKER;
    t.even = cx.texture_id(even);
    t.odd = cx.texture_id(odd);
    return cx.add_texture(t);
}
int noise_texture::flatten(flat_ctx &cx) const {
    rt_texture t{};
    t.kind = RT_TEX_NOISE;
    t.even = t.odd = -1;
    t.scale = scale;
    return cx.add_texture(t);
}
int image_texture::flatten(flat_ctx &cx) const {
    rt_texture t{};
    t.kind = RT_TEX_IMAGE;
    t.even = t.odd = -1;
    // the texels value() can address: 3 bytes per texel (surface_texture.h:26-28)
    rt_image im{};
    im.offset = (int64_t)cx.out->image_data.size();
    im.nx = nx;
    im.ny = ny;
    const size_t n = data ? (size_t)3 * (size_t)nx * (size_t)ny : 0;
    if (!data || nx <= 0 || ny <= 0) throw std::runtime_error("image_texture without pixels (stbi_load failed?)");
    cx.out->image_data.insert(cx.out->image_data.end(), data, data + n);
    cx.out->images.push_back(im);
    t.image = (int32_t)cx.out->images.size() - 1;
    return cx.add_texture(t);
}

// ----------------------------------------------------------------- materials
static rt_material mat_of(int kind, int tex) {
    rt_material m{};
    m.kind = kind;
    m.texture = tex;
    return m;
}
int lambertian::flatten(flat_ctx &cx) const { return cx.add_material(mat_of(RT_MAT_LAMBERTIAN, cx.texture_id(albedo))); }
int diffuse_light::flatten(flat_ctx &cx) const { return cx.add_material(mat_of(RT_MAT_DIFFUSE_LIGHT, cx.texture_id(emit))); }
int isotropic::flatten(flat_ctx &cx) const { return cx.add_material(mat_of(RT_MAT_ISOTROPIC, cx.texture_id(albedo))); }
int metal::flatten(flat_ctx &cx) const {
    rt_material m = mat_of(RT_MAT_METAL, -1);
    for (int i = 0; i < 3; i++) m.albedo[i] = albedo[i];
    m.fuzz = fuzz;
    return cx.add_material(m);
}
int dielectric::flatten(flat_ctx &cx) const {
    rt_material m = mat_of(RT_MAT_DIELECTRIC, -1);
    m.ref_idx = ref_idx;
    return cx.add_material(m);
}

// ------------------------------------------------------------------ hitables
void hitable_list::flatten(flat_ctx &cx) const { for (int i = 0; i < list_size; i++) list[i]->flatten(cx); }
void sphere::flatten(flat_ctx &cx) const { cx.emit(RT_PRIM_SPHERE, mat_ptr, {center[0], center[1], center[2], radius}); }
void moving_sphere::flatten(flat_ctx &cx) const {
    cx.emit(RT_PRIM_MOVING_SPHERE, mat_ptr, {center0[0], center0[1], center0[2], center1[0], center1[1], center1[2],
                                             time0, time1, radius});
}
void xy_rect::flatten(flat_ctx &cx) const { cx.emit(RT_PRIM_XY_RECT, mp, {x0, x1, y0, y1, k}); }
void xz_rect::flatten(flat_ctx &cx) const { cx.emit(RT_PRIM_XZ_RECT, mp, {x0, x1, z0, z1, k}); }
void yz_rect::flatten(flat_ctx &cx) const { cx.emit(RT_PRIM_YZ_RECT, mp, {y0, y1, z0, z1, k}); }
void box::flatten(flat_ctx &cx) const { list_ptr->flatten(cx); }
void flip_normals::flatten(flat_ctx &cx) const {
    cx.flip ^= 1;
    ptr->flatten(cx);
    cx.flip ^= 1;
}
void translate::flatten(flat_ctx &cx) const {
    cx.wrapped({(float)RT_OP_TRANSLATE, offset[0], offset[1], offset[2]}, [&] { ptr->flatten(cx); });
}
void rotate_y::flatten(flat_ctx &cx) const {
    cx.wrapped({(float)RT_OP_ROTATE_Y, sin_theta, cos_theta, 0.0f}, [&] { ptr->flatten(cx); });
}
void bvh_node::flatten(flat_ctx &cx) const {
    left->flatten(cx);
    if (right != left) right->flatten(cx);
}
void constant_medium::flatten(flat_ctx &cx) const {
    if (!cx.chain.empty() || cx.flip || cx.in_boundary)
        throw std::runtime_error("constant_medium under a transform or inside another medium is not supported");
    rt_medium m{};
    m.material = cx.material_id(phase_function);
    m.density = density;
    m.order = (int32_t)cx.out->prims.size();
    m.boundary_first = (int32_t)cx.out->boundary.size();
    cx.in_boundary = true;
    boundary->flatten(cx);
    cx.in_boundary = false;
    m.boundary_count = (int32_t)cx.out->boundary.size() - m.boundary_first;
    cx.out->media.push_back(m);
}

std::unique_ptr<flat_scene> flatten_world(const hitable *world, float time0, float time1) {
    auto fs = std::make_unique<flat_scene>();
    flat_ctx cx;
    cx.out = fs.get();
    world->flatten(cx);
    fs->ranvec.resize(768);
    fs->perm.resize(768);
    for (int i = 0; i < 256; i++) {
        for (int k = 0; k < 3; k++) fs->ranvec[3 * i + k] = perlin::ranvec[i][k];
        fs->perm[i] = perlin::perm_x[i];
        fs->perm[256 + i] = perlin::perm_y[i];
        fs->perm[512 + i] = perlin::perm_z[i];
    }
    rt_scene_desc &d = fs->desc;
    d.abi_version = RT_ABI_VERSION;
    d.nprims = (int32_t)fs->prims.size();
    d.nboundary = (int32_t)fs->boundary.size();
    d.nmedia = (int32_t)fs->media.size();
    d.nmaterials = (int32_t)fs->materials.size();
    d.ntextures = (int32_t)fs->textures.size();
    d.ninstances = (int32_t)fs->instances.size();
    d.prims = fs->prims.data();
    d.boundary_prims = fs->boundary.data();
    d.media = fs->media.data();
    d.materials = fs->materials.data();
    d.textures = fs->textures.data();
    d.instances = fs->instances.data();
    d.perlin_ranvec = fs->ranvec.data();
    d.perlin_perm = fs->perm.data();
    d.time0 = time0;
    d.time1 = time1;
    d.nimages = (int32_t)fs->images.size();
    d.images = fs->images.data();
    d.image_data = fs->image_data.data();
    d.image_bytes = (int64_t)fs->image_data.size();
    return fs;
}

// ---------------------------------------------------------------------- dump
// Same text as oracle/ref_harness.cpp --dump, reconstructed from the descriptor,
// so a test can check the host builders + flattener against the reference.
namespace {
struct dumper {
    const rt_scene_desc *d;
    std::string s;
    std::map<int, int> ids;
    void put(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        char tmp[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(tmp, sizeof tmp, fmt, ap);
        va_end(ap);
        s += tmp;
    }
    void tex(int t) {
        const rt_texture &x = d->textures[t];
        if (x.kind == RT_TEX_CONSTANT) put("(const %a %a %a)", x.color[0], x.color[1], x.color[2]);
        else if (x.kind == RT_TEX_CHECKER) { put("(checker even="); tex(x.even); put(" odd="); tex(x.odd); put(")"); }
        else if (x.kind == RT_TEX_NOISE) put("(noise %a)", x.scale);
        else {
            const rt_image &im = d->images[x.image];
            uint32_t h = 2166136261u;   // FNV-1a over the addressable texels
            for (int64_t b = 0; b < (int64_t)3 * im.nx * im.ny; b++) h = (h ^ d->image_data[im.offset + b]) * 16777619u;
            put("(image %d %d %08x)", im.nx, im.ny, h);
        }
    }
    void mat(int m) {
        auto it = ids.find(m);
        int id = it == ids.end() ? (int)ids.size() : it->second;
        ids.emplace(m, id);
        put(" mat%d=", id);
        const rt_material &x = d->materials[m];
        switch (x.kind) {
        case RT_MAT_LAMBERTIAN: put("lambertian"); tex(x.texture); break;
        case RT_MAT_METAL: put("metal(%a %a %a fuzz %a)", x.albedo[0], x.albedo[1], x.albedo[2], x.fuzz); break;
        case RT_MAT_DIELECTRIC: put("dielectric(%a)", x.ref_idx); break;
        case RT_MAT_DIFFUSE_LIGHT: put("light"); tex(x.texture); break;
        case RT_MAT_ISOTROPIC: put("isotropic"); tex(x.texture); break;
        }
    }
    void prim(const rt_prim &p, const char *lead) {
        s += lead;
        if (p.instance >= 0) {
            const rt_instance &in = d->instances[p.instance];
            for (int k = 0; k < in.nops; k++) {
                const int op = (int)in.ops[k][0];
                if (op == RT_OP_TRANSLATE) put("translate(%a %a %a) ", in.ops[k][1], in.ops[k][2], in.ops[k][3]);
                else if (op == RT_OP_ROTATE_Y) put("rotate_y(sin %a cos %a) ", in.ops[k][1], in.ops[k][2]);
                else if (op == RT_OP_FLIP) put("flip ");
            }
        }
        if (p.flip) put("flip ");
        const float *q = p.p;
        switch (p.kind) {
        case RT_PRIM_SPHERE: put("sphere %a %a %a r %a", q[0], q[1], q[2], q[3]); break;
        case RT_PRIM_MOVING_SPHERE:
            put("moving_sphere %a %a %a -> %a %a %a t %a %a r %a", q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8]);
            break;
        case RT_PRIM_XY_RECT: put("xy_rect %a %a %a %a k %a", q[0], q[1], q[2], q[3], q[4]); break;
        case RT_PRIM_XZ_RECT: put("xz_rect %a %a %a %a k %a", q[0], q[1], q[2], q[3], q[4]); break;
        case RT_PRIM_YZ_RECT: put("yz_rect %a %a %a %a k %a", q[0], q[1], q[2], q[3], q[4]); break;
        }
        mat(p.material);
        put("\n");
    }
    void medium(const rt_medium &m) {
        put("medium density %a", m.density);
        mat(m.material);
        put(" boundary{\n");
        for (int b = 0; b < m.boundary_count; b++) prim(d->boundary_prims[m.boundary_first + b], "  ");
        put("}\n");
    }
    void run() {
        int mi = 0;
        for (int i = 0; i <= d->nprims; i++) {
            while (mi < d->nmedia && d->media[mi].order == i) medium(d->media[mi++]);
            if (i < d->nprims) prim(d->prims[i], "");
        }
    }
};
}  // namespace

std::string dump_desc(const rt_scene_desc *d) {
    dumper u;
    u.d = d;
    u.run();
    return u.s;
}

}  // namespace rtnw
