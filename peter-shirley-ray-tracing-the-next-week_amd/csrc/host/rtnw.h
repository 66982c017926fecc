// rtnw.h — host-side scene API of the MI355X path tracer.
//
// The class names, constructor signatures and public members are those of the
// reference's scene-building API (vec3.h, ray.h, camera.h, hitable.h,
// hitable_list.h, sphere.h, aarect.h, box.h, constant_medium.h, bvh.h,
// material.h, texture.h, perlin.h, surface_texture.h), so scene builders such
// as random_scene(), cornell_box() and final() (main.cpp:49-230) compile
// against it unchanged (see compat/ for the reference header names).
//
// What differs: the ray/scatter/texture *evaluation* methods (hit, scatter,
// value, emitted) do not exist on the host.  The hot path runs on the GPU; a
// world is turned into an rt_scene_desc by `flatten_world()` and rendered through
// the C ABI in include/rt_hip.h.  Each class contributes its part of the
// descriptor through the `flatten` visitor.
#pragma once

#include <array>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <iosfwd>
#include <memory>
#include <string>
#include <vector>

#include "rt_hip.h"

namespace rtnw {

// -------------------------------------------------------------------- random
// The reference draws from libc drand48() (scene construction: main.cpp:61-72,
// 204, 226; bvh.h:99; perlin.h:85-92).  The host API draws from the same
// process-wide libc stream so that a drop-in scene builder sees the same values.
double drand48();
// Puts the libc stream back where an unseeded reference process starts
// main(): state 0, then the 1533 draws of the Perlin static initialisers.
void reset_reference_rng();

// ---------------------------------------------------------------------- vec3
class vec3 {
public:
    float e[3];
    vec3() {}
    vec3(float e0, float e1, float e2) { e[0] = e0; e[1] = e1; e[2] = e2; }
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    float r() const { return e[0]; }
    float g() const { return e[1]; }
    float b() const { return e[2]; }
    const vec3 &operator+() const { return *this; }
    vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
    float operator[](int i) const { return e[i]; }
    float &operator[](int i) { return e[i]; }
    vec3 &operator+=(const vec3 &o) { for (int i = 0; i < 3; ++i) e[i] += o.e[i]; return *this; }
    vec3 &operator-=(const vec3 &o) { for (int i = 0; i < 3; ++i) e[i] -= o.e[i]; return *this; }
    vec3 &operator*=(const vec3 &o) { for (int i = 0; i < 3; ++i) e[i] *= o.e[i]; return *this; }
    vec3 &operator/=(const vec3 &o) { for (int i = 0; i < 3; ++i) e[i] /= o.e[i]; return *this; }
    vec3 &operator*=(const float t) { for (int i = 0; i < 3; ++i) e[i] *= t; return *this; }
    // reciprocal multiply, as the reference's operator/= (vec3.h:134-141)
    vec3 &operator/=(const float t) { const float k = 1.0 / t; for (int i = 0; i < 3; ++i) e[i] *= k; return *this; }
    float squared_length() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    float length() const { return std::sqrt(squared_length()); }
    void make_unit_vector() { const float k = 1.0 / std::sqrt(squared_length()); e[0] *= k; e[1] *= k; e[2] *= k; }
};

inline vec3 operator+(const vec3 &a, const vec3 &b) { return vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline vec3 operator-(const vec3 &a, const vec3 &b) { return vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline vec3 operator*(const vec3 &a, const vec3 &b) { return vec3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline vec3 operator/(const vec3 &a, const vec3 &b) { return vec3(a.e[0] / b.e[0], a.e[1] / b.e[1], a.e[2] / b.e[2]); }
inline vec3 operator*(float t, const vec3 &v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3 &v, float t) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator/(vec3 v, float t) { return vec3(v.e[0] / t, v.e[1] / t, v.e[2] / t); }
inline float dot(const vec3 &a, const vec3 &b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline vec3 cross(const vec3 &a, const vec3 &b) {
    return vec3(a.e[1] * b.e[2] - a.e[2] * b.e[1], -(a.e[0] * b.e[2] - a.e[2] * b.e[0]), a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
inline vec3 unit_vector(vec3 v) { return v / v.length(); }
std::ostream &operator<<(std::ostream &os, const vec3 &t);
std::istream &operator>>(std::istream &is, vec3 &t);

// ----------------------------------------------------------------------- ray
class ray {
public:
    vec3 A, B;
    float _time;
    ray() {}
    ray(const vec3 &a, const vec3 &b, float ti = 0.0) : A(a), B(b), _time(ti) {}
    vec3 origin() const { return A; }
    vec3 direction() const { return B; }
    float time() const { return _time; }
    vec3 point_at_parameter(float t) const { return A + t * B; }
};

// ---------------------------------------------------------------------- aabb
inline float ffmin(float a, float b) { return a < b ? a : b; }
inline float ffmax(float a, float b) { return a > b ? a : b; }

class aabb {
public:
    vec3 _min, _max;
    aabb() {}
    aabb(const vec3 a, const vec3 &b) : _min(a), _max(b) {}
    vec3 min() const { return _min; }
    vec3 max() const { return _max; }
    // Slab test.  The reference's aabb::hit (aabb.h:33-49) subtracts the ray
    // direction where the origin belongs; this is the corrected form.
    bool hit(const ray &r, float tmin, float tmax) const;
};
aabb surrounding_box(aabb box0, aabb box1);

// --------------------------------------------------------------- flattening
struct flat_ctx;   // defined in flatten.cpp

// ------------------------------------------------------------------ textures
class texture {
public:
    virtual ~texture() {}
    virtual int flatten(flat_ctx &cx) const = 0;   // returns the texture index
};

class constant_texture : public texture {
public:
    vec3 color;
    constant_texture() {}
    constant_texture(vec3 c) : color(c) {}
    int flatten(flat_ctx &cx) const override;
};

class checker_texture : public texture {
public:
    texture *odd;
    texture *even;
    checker_texture() {}
    checker_texture(texture *t0, texture *t1) : odd(t1), even(t0) {}
    int flatten(flat_ctx &cx) const override;
};

// Gradient noise tables, generated from drand48 during static initialisation
// exactly as perlin.h:82-111 does (shared by every noise_texture).
class perlin {
public:
    static vec3 *ranvec;
    static int *perm_x;
    static int *perm_y;
    static int *perm_z;
    static void regenerate();   // re-run the static initialisers' draws
};

class noise_texture : public texture {
public:
    perlin noise;
    float scale;
    noise_texture() {}
    noise_texture(float sc) : scale(sc) {}
    int flatten(flat_ctx &cx) const override;
};

class image_texture : public texture {
public:
    unsigned char *data;
    int nx, ny;
    image_texture() {}
    image_texture(unsigned char *pixels, int A, int B) : data(pixels), nx(A), ny(B) {}
    int flatten(flat_ctx &cx) const override;
};

// PNG reader standing in for the vendored stb_image the reference calls (main.cpp:93):
// same signature and result (channels as stored when req_comp == 0), 8-bit PNG only.
unsigned char *stbi_load(const char *filename, int *x, int *y, int *comp, int req_comp);
unsigned char *png_decode(const unsigned char *buf, size_t len, int *x, int *y, int *comp, std::string *err);

// ----------------------------------------------------------------- materials
class material {
public:
    virtual ~material() {}
    virtual int flatten(flat_ctx &cx) const = 0;   // returns the material index
};

class lambertian : public material {
public:
    texture *albedo;
    lambertian(texture *a) : albedo(a) {}
    int flatten(flat_ctx &cx) const override;
};

class metal : public material {
public:
    vec3 albedo;
    float fuzz;
    metal(const vec3 &a, float f) : albedo(a) { fuzz = f < 1 ? f : 1; }
    int flatten(flat_ctx &cx) const override;
};

class dielectric : public material {
public:
    float ref_idx;
    dielectric(float ri) : ref_idx(ri) {}
    int flatten(flat_ctx &cx) const override;
};

class diffuse_light : public material {
public:
    texture *emit;
    diffuse_light(texture *a) : emit(a) {}
    int flatten(flat_ctx &cx) const override;
};

class isotropic : public material {
public:
    texture *albedo;
    isotropic(texture *a) : albedo(a) {}
    int flatten(flat_ctx &cx) const override;
};

// ------------------------------------------------------------------ hitables
class hitable {
public:
    virtual ~hitable() {}
    virtual bool bounding_box(float t0, float t1, aabb &box) const = 0;
    virtual void flatten(flat_ctx &cx) const = 0;
};

class hitable_list : public hitable {
public:
    hitable **list;
    int list_size;
    hitable_list() {}
    hitable_list(hitable **l, int n) : list(l), list_size(n) {}
    // Same result as hitable_list.h:34-50, including its use of list[0]'s box
    // for every element (it only matters for bvh_node's sort order).
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class sphere : public hitable {
public:
    vec3 center;
    float radius;
    material *mat_ptr;
    sphere() {}
    sphere(vec3 cen, float r, material *m) : center(cen), radius(r), mat_ptr(m) {}
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class moving_sphere : public hitable {
public:
    vec3 center0, center1;
    float time0, time1;
    float radius;
    material *mat_ptr;
    moving_sphere() {}
    moving_sphere(vec3 cen0, vec3 cen1, float t0, float t1, float r, material *m)
        : center0(cen0), center1(cen1), time0(t0), time1(t1), radius(r), mat_ptr(m) {}
    vec3 center(float time) const { return center0 + ((time - time0) / (time1 - time0)) * (center1 - center0); }
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class xy_rect : public hitable {
public:
    material *mp;
    float x0, x1, y0, y1, k;
    xy_rect() {}
    xy_rect(float _x0, float _x1, float _y0, float _y1, float _k, material *mat)
        : mp(mat), x0(_x0), x1(_x1), y0(_y0), y1(_y1), k(_k) {}
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class xz_rect : public hitable {
public:
    material *mp;
    float x0, x1, z0, z1, k;
    xz_rect() {}
    xz_rect(float _x0, float _x1, float _z0, float _z1, float _k, material *mat)
        : mp(mat), x0(_x0), x1(_x1), z0(_z0), z1(_z1), k(_k) {}
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class yz_rect : public hitable {
public:
    material *mp;
    float y0, y1, z0, z1, k;
    yz_rect() {}
    yz_rect(float _y0, float _y1, float _z0, float _z1, float _k, material *mat)
        : mp(mat), y0(_y0), y1(_y1), z0(_z0), z1(_z1), k(_k) {}
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class box : public hitable {
public:
    vec3 pmin, pmax;
    hitable *list_ptr;
    box() {}
    box(const vec3 &p0, const vec3 &p1, material *ptr);
    bool bounding_box(float t0, float t1, aabb &b) const override { b = aabb(pmin, pmax); return true; }
    void flatten(flat_ctx &cx) const override;
};

class flip_normals : public hitable {
public:
    hitable *ptr;
    flip_normals(hitable *p) : ptr(p) {}
    bool bounding_box(float t0, float t1, aabb &box) const override { return ptr->bounding_box(t0, t1, box); }
    void flatten(flat_ctx &cx) const override;
};

class translate : public hitable {
public:
    hitable *ptr;
    vec3 offset;
    translate(hitable *p, const vec3 &displacement) : ptr(p), offset(displacement) {}
    bool bounding_box(float t0, float t1, aabb &box) const override;
    void flatten(flat_ctx &cx) const override;
};

class rotate_y : public hitable {
public:
    hitable *ptr;
    float sin_theta;
    float cos_theta;
    bool hasbox;
    aabb bbox;
    rotate_y(hitable *p, float angle);
    bool bounding_box(float t0, float t1, aabb &box) const override { box = bbox; return hasbox; }
    void flatten(flat_ctx &cx) const override;
};

class constant_medium : public hitable {
public:
    hitable *boundary;
    float density;
    material *phase_function;
    constant_medium(hitable *b, float d, texture *a) : boundary(b), density(d) { phase_function = new isotropic(a); }
    bool bounding_box(float t0, float t1, aabb &box) const override { return boundary->bounding_box(t0, t1, box); }
    void flatten(flat_ctx &cx) const override;
};

// bvh.h:11-121.  The constructor consumes drand48 and orders the list exactly as
// the reference's (random axis, qsort by box minimum, split n/2), so a scene that
// wraps its list in a bvh_node keeps the reference's RNG state.  On the device
// the node is a container: its leaves join the GPU's own SAH BVH.
class bvh_node : public hitable {
public:
    hitable *left;
    hitable *right;
    aabb box;
    bvh_node() {}
    bvh_node(hitable **l, int n, float time0, float time1);
    bool bounding_box(float t0, float t1, aabb &b) const override { b = box; return true; }
    void flatten(flat_ctx &cx) const override;
};

// -------------------------------------------------------------------- camera
class camera {
public:
    vec3 origin;
    vec3 u, v, w;
    vec3 horizontal;
    vec3 vertical;
    vec3 lower_left_corner;
    float len_radius;
    float time0, time1;
    camera(vec3 lookfrom, vec3 lookat, vec3 vup, float vfov, float aspect, float aperture, float focus_dist,
           float t0, float t1);
    rt_camera_desc desc() const;
};

// ------------------------------------------------------------- flatten output
// Owns the arrays an rt_scene_desc points to.
struct flat_scene {
    std::vector<rt_prim> prims, boundary;
    std::vector<rt_medium> media;
    std::vector<rt_material> materials;
    std::vector<rt_texture> textures;
    std::vector<rt_instance> instances;
    std::vector<float> ranvec;      // 768
    std::vector<int32_t> perm;      // 768
    std::vector<rt_image> images;
    std::vector<uint8_t> image_data;
    rt_scene_desc desc{};           // points into the vectors above
};
// Flattens `world`; time0/time1 is the shutter span rays may carry.
std::unique_ptr<flat_scene> flatten_world(const hitable *world, float time0 = 0.0f, float time1 = 1.0f);
// Leaf listing in the format of oracle/ref_harness.cpp --dump.
std::string dump_desc(const rt_scene_desc *d);

// ------------------------------------------------------------- scene builders
// The reference's builders (main.cpp:49-230), restated against this API.  Where
// the reference passes several drand48() calls in one argument list (whose
// evaluation order C++ leaves unspecified) they are drawn left to right, the
// order clang gives the reference.
hitable *random_scene();         // main.cpp:49-85
hitable *random_scene_motion();  // TNW/Chapter01:36-67 with the main.cpp texture API
hitable *two_spheres();          // main.cpp:99-110
hitable *edge_empty();           // the tests' edge scenes (oracle/ref_harness.cpp edge_*)
hitable *edge_single();
hitable *edge_degenerate();
hitable *simple_light();         // main.cpp:122-133
hitable *test_scene();           // main.cpp:135-145 (`test`)
hitable *cornell_box();          // main.cpp:148-166
hitable *cornell_smoke();        // main.cpp:169-188
hitable *final_scene();          // main.cpp:190-230 (`final`)
// main.cpp:87-97 (`earth`); the reference reads "picture.png" from the working
// directory; build_named_scene("earth") reads $RTNW_EARTH_PNG if set.
hitable *earth(const char *png_path = "picture.png");

// Builds a named scene as a fresh reference process would (reset_reference_rng first).
hitable *build_named_scene(const std::string &name, float *time0, float *time1);

}  // namespace rtnw
