// rtnw.cpp — host scene API: constructors, bounding boxes, the Perlin tables and
// the reference's scene builders restated against this API.
#include "rtnw.h"

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <stdexcept>

namespace rtnw {

double drand48() { return ::drand48(); }

std::ostream &operator<<(std::ostream &os, const vec3 &t) { return os << t.e[0] << " " << t.e[1] << " " << t.e[2]; }
std::istream &operator>>(std::istream &is, vec3 &t) { return is >> t.e[0] >> t.e[1] >> t.e[2]; }

// ---------------------------------------------------------------------- aabb
bool aabb::hit(const ray &r, float tmin, float tmax) const {
    for (int a = 0; a < 3; a++) {
        const float invD = 1.0f / r.direction()[a];
        float t0 = (_min[a] - r.origin()[a]) * invD;
        float t1 = (_max[a] - r.origin()[a]) * invD;
        if (invD < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax <= tmin) return false;
    }
    return true;
}

aabb surrounding_box(aabb box0, aabb box1) {   // aabb.h:54-62
    vec3 lo(std::fmin(box0.min().x(), box1.min().x()), std::fmin(box0.min().y(), box1.min().y()),
            std::fmin(box0.min().z(), box1.min().z()));
    vec3 hi(std::fmax(box0.max().x(), box1.max().x()), std::fmax(box0.max().y(), box1.max().y()),
            std::fmax(box0.max().z(), box1.max().z()));
    return aabb(lo, hi);
}

// -------------------------------------------------------------------- perlin
// perlin.h:82-111: 256 unit gradients, then three permutations, all from
// drand48 in declaration order (ranvec, perm_x, perm_y, perm_z).
static vec3 *make_gradients() {
    vec3 *p = new vec3[256];
    for (int i = 0; i < 256; ++i) {
        const double x = -1 + 2 * drand48();
        const double y = -1 + 2 * drand48();
        const double z = -1 + 2 * drand48();
        p[i] = unit_vector(vec3((float)x, (float)y, (float)z));
    }
    return p;
}
static int *make_permutation() {
    int *p = new int[256];
    for (int i = 0; i < 256; i++) p[i] = i;
    for (int i = 255; i > 0; i--) {
        const int target = int(drand48() * (i + 1));
        const int tmp = p[i];
        p[i] = p[target];
        p[target] = tmp;
    }
    return p;
}
vec3 *perlin::ranvec = make_gradients();
int *perlin::perm_x = make_permutation();
int *perlin::perm_y = make_permutation();
int *perlin::perm_z = make_permutation();

void perlin::regenerate() {
    vec3 *rv = make_gradients();
    int *px = make_permutation(), *py = make_permutation(), *pz = make_permutation();
    for (int i = 0; i < 256; i++) {
        ranvec[i] = rv[i];
        perm_x[i] = px[i];
        perm_y[i] = py[i];
        perm_z[i] = pz[i];
    }
    delete[] rv; delete[] px; delete[] py; delete[] pz;
}

void reset_reference_rng() {
    unsigned short zero[3] = {0, 0, 0};
    ::seed48(zero);          // an unseeded glibc stream starts at state 0
    perlin::regenerate();    // the static initialisers' 1533 draws
}

// ------------------------------------------------------------- bounding boxes
bool hitable_list::bounding_box(float t0, float t1, aabb &box) const {   // hitable_list.h:34-50
    if (list_size < 1) return false;
    aabb temp_box;
    if (!list[0]->bounding_box(t0, t1, temp_box)) return false;
    box = temp_box;
    for (int i = 1; i < list_size; i++) {
        if (list[0]->bounding_box(t0, t1, temp_box)) box = surrounding_box(box, temp_box);
        else return false;
    }
    return true;
}
bool sphere::bounding_box(float, float, aabb &box) const {
    box = aabb(center - vec3(radius, radius, radius), center + vec3(radius, radius, radius));
    return true;
}
bool moving_sphere::bounding_box(float t0, float t1, aabb &box) const {
    aabb box0(center(t0) - vec3(radius, radius, radius), center(t0) + vec3(radius, radius, radius));
    aabb box1(center(t1) - vec3(radius, radius, radius), center(t1) + vec3(radius, radius, radius));
    box = surrounding_box(box0, box1);
    return true;
}
bool xy_rect::bounding_box(float, float, aabb &box) const { box = aabb(vec3(x0, y0, k - 0.0001), vec3(x1, y1, k + 0.0001)); return true; }
bool xz_rect::bounding_box(float, float, aabb &box) const { box = aabb(vec3(x0, k - 0.0001, z0), vec3(x1, k + 0.0001, z1)); return true; }
bool yz_rect::bounding_box(float, float, aabb &box) const { box = aabb(vec3(k - 0.0001, y0, z0), vec3(k + 0.0001, y1, z1)); return true; }
bool translate::bounding_box(float t0, float t1, aabb &box) const {
    if (!ptr->bounding_box(t0, t1, box)) return false;
    box = aabb(box.min() + offset, box.max() + offset);
    return true;
}

box::box(const vec3 &p0, const vec3 &p1, material *ptr) : pmin(p0), pmax(p1) {   // box.h:23-34
    hitable **l = new hitable *[6];
    l[0] = new xy_rect(p0.x(), p1.x(), p0.y(), p1.y(), p1.z(), ptr);
    l[1] = new flip_normals(new xy_rect(p0.x(), p1.x(), p0.y(), p1.y(), p0.z(), ptr));
    l[2] = new xz_rect(p0.x(), p1.x(), p0.z(), p1.z(), p1.y(), ptr);
    l[3] = new flip_normals(new xz_rect(p0.x(), p1.x(), p0.z(), p1.z(), p0.y(), ptr));
    l[4] = new yz_rect(p0.y(), p1.y(), p0.z(), p1.z(), p1.x(), ptr);
    l[5] = new flip_normals(new yz_rect(p0.y(), p1.y(), p0.z(), p1.z(), p0.x(), ptr));
    list_ptr = new hitable_list(l, 6);
}

rotate_y::rotate_y(hitable *p, float angle) : ptr(p) {   // hitable.h:98-126
    const float radians = (M_PI / 180.) * angle;
    sin_theta = std::sin(radians);
    cos_theta = std::cos(radians);
    hasbox = ptr->bounding_box(0, 1, bbox);
    vec3 lo(0x1.fffffep+127f, 0x1.fffffep+127f, 0x1.fffffep+127f);
    vec3 hi(-0x1.fffffep+127f, -0x1.fffffep+127f, -0x1.fffffep+127f);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                const float x = i * bbox.max().x() + (1 - i) * bbox.min().x();
                const float y = j * bbox.max().y() + (1 - j) * bbox.min().y();
                const float z = k * bbox.max().z() + (1 - k) * bbox.min().z();
                const vec3 corner(cos_theta * x + sin_theta * z, y, -sin_theta * x + cos_theta * z);
                for (int c = 0; c < 3; c++) {
                    if (corner[c] > hi[c]) hi[c] = corner[c];
                    if (corner[c] < lo[c]) lo[c] = corner[c];
                }
            }
    bbox = aabb(lo, hi);
}

// bvh.h:58-121.  The comparators return -1 when a's box minimum is lower on the
// axis and 1 otherwise, fed to libc qsort, so the element order matches.
template <int Axis>
static int box_compare(const void *a, const void *b) {
    aabb box_left, box_right;
    const hitable *ah = *(hitable *const *)a;
    const hitable *bh = *(hitable *const *)b;
    if (!ah->bounding_box(0, 0, box_left) || !bh->bounding_box(0, 0, box_right))
        std::cerr << "no bounding box in bvh_node constructor\n";
    return (box_left.min()[Axis] - box_right.min()[Axis] < 0.0) ? -1 : 1;
}

bvh_node::bvh_node(hitable **l, int n, float time0, float time1) {
    const int axis = int(3 * drand48());
    if (axis == 0) qsort(l, n, sizeof(hitable *), box_compare<0>);
    else if (axis == 1) qsort(l, n, sizeof(hitable *), box_compare<1>);
    else qsort(l, n, sizeof(hitable *), box_compare<2>);
    if (n == 1) {
        left = right = l[0];
    } else if (n == 2) {
        left = l[0];
        right = l[1];
    } else {
        left = new bvh_node(l, n / 2, time0, time1);
        right = new bvh_node(l + n / 2, n - n / 2, time0, time1);
    }
    aabb box_left, box_right;
    if (!left->bounding_box(time0, time1, box_left) || !right->bounding_box(time0, time1, box_right))
        std::cerr << "no bounding box in bvh_node constructor\n";
    box = surrounding_box(box_left, box_right);
}

// -------------------------------------------------------------------- camera
camera::camera(vec3 lookfrom, vec3 lookat, vec3 vup, float vfov, float aspect, float aperture, float focus_dist,
               float t0, float t1) {   // camera.h:21-39
    time0 = t0;
    time1 = t1;
    len_radius = aperture / 2;
    const float theta = vfov * M_PI / 180;
    const float half_height = std::tan(theta / 2);
    const float half_width = aspect * half_height;
    origin = lookfrom;
    w = unit_vector(lookfrom - lookat);
    u = unit_vector(cross(vup, w));
    v = cross(w, u);
    lower_left_corner = origin - half_width * focus_dist * u - half_height * focus_dist * v - focus_dist * w;
    horizontal = 2 * half_width * focus_dist * u;
    vertical = 2 * half_height * focus_dist * v;
}

rt_camera_desc camera::desc() const {
    rt_camera_desc d{};
    for (int i = 0; i < 3; i++) {
        d.origin[i] = origin[i];
        d.lower_left_corner[i] = lower_left_corner[i];
        d.horizontal[i] = horizontal[i];
        d.vertical[i] = vertical[i];
        d.u[i] = u[i];
        d.v[i] = v[i];
        d.w[i] = w[i];
    }
    d.lens_radius = len_radius;
    d.time0 = time0;
    d.time1 = time1;
    return d;
}

// ------------------------------------------------------------- scene builders
hitable *random_scene() {   // main.cpp:49-85
    const int n = 500;
    hitable **list = new hitable *[n + 1];
    texture *checker = new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)),
                                           new constant_texture(vec3(0.9, 0.9, 0.9)));
    list[0] = new sphere(vec3(0, -700, 0), 700, new lambertian(checker));
    int i = 1;
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            const float choose_mat = drand48();
            const double rx = drand48(), rz = drand48();
            vec3 center(a + 0.9 * rx, 0.2, b + 0.9 * rz);
            if ((center - vec3(4, 0.2, 0)).length() > 0.9) {
                if (choose_mat < 0.8) {
                    // diffuse spheres are commented out in the reference (main.cpp:66-68)
                } else if (choose_mat < 0.95) {
                    const double x = drand48(), y = drand48(), z = drand48(), f = drand48();
                    list[i++] = new sphere(center, 0.2,
                                           new metal(vec3(0.5 * (1 + x), 0.5 * (1 + y), 0.5 * (1 + z)), 0.5 * f));
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

hitable *random_scene_motion() {   // TNW/Chapter01:36-67, texture API of main.cpp:54-57
    hitable **list = new hitable *[501];
    texture *checker = new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)),
                                           new constant_texture(vec3(0.9, 0.9, 0.9)));
    list[0] = new sphere(vec3(0, -700, 0), 700, new lambertian(checker));
    int i = 1;
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            const float choose_mat = drand48();
            const double rx = drand48(), rz = drand48();
            vec3 center(a + 0.9 * rx, 0.2, b + 0.9 * rz);
            if ((center - vec3(4, 0.2, 0)).length() > 0.9) {
                if (choose_mat < 0.8) {
                    const double dy = drand48();
                    const vec3 c1 = center + vec3(0, 0.5 * dy, 0);
                    const double r0 = drand48(), r1 = drand48(), g0 = drand48(), g1 = drand48();
                    const double b0 = drand48(), b1 = drand48();
                    list[i++] = new moving_sphere(center, c1, 0.0, 1.0, 0.2,
                        new lambertian(new constant_texture(vec3(r0 * r1, g0 * g1, b0 * b1))));
                } else if (choose_mat < 0.95) {
                    const double x = drand48(), y = drand48(), z = drand48(), f = drand48();
                    list[i++] = new sphere(center, 0.2,
                                           new metal(vec3(0.5 * (1 + x), 0.5 * (1 + y), 0.5 * (1 + z)), 0.5 * f));
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

hitable *two_spheres() {   // main.cpp:99-110
    new diffuse_light(new constant_texture(vec3(15, 15, 15)));   // built but unused by the reference
    new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)), new constant_texture(vec3(0.9, 0.9, 0.9)));
    material *red = new lambertian(new constant_texture(vec3(0.65, 0.05, 0.05)));
    hitable **list = new hitable *[51];
    list[0] = new sphere(vec3(0, -10, 0), 10, red);
    list[1] = new yz_rect(0, 555, 0, 555, 0, red);
    return new hitable_list(list, 2);
}

hitable *simple_light() {   // main.cpp:122-133
    texture *pertext = new noise_texture(4);
    texture *checker = new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)),
                                           new constant_texture(vec3(0.9, 0.9, 0.9)));
    hitable **list = new hitable *[4];
    int i = 0;
    list[i++] = new sphere(vec3(0, 2, 0), 2, new lambertian(pertext));
    list[i++] = new sphere(vec3(0, -700, 0), 700, new lambertian(checker));
    list[i++] = new sphere(vec3(0, 7, 0), 2, new diffuse_light(new constant_texture(vec3(4, 4, 4))));
    list[i++] = new xy_rect(3, 5, 1, 3, -2, new diffuse_light(new constant_texture(vec3(4, 4, 4))));
    return new hitable_list(list, i);
}

hitable *test_scene() {   // main.cpp:135-145
    texture *pertext = new noise_texture(4);
    texture *checker = new checker_texture(new constant_texture(vec3(0.2, 0.3, 0.1)),
                                           new constant_texture(vec3(0.9, 0.9, 0.9)));
    hitable **list = new hitable *[4];
    list[0] = new sphere(vec3(0, -700, 0), 700, new lambertian(checker));
    list[1] = new sphere(vec3(0, 2, 0), 2, new lambertian(pertext));
    list[2] = new sphere(vec3(0, 7, 0), 2, new diffuse_light(new constant_texture(vec3(11, 11, 11))));
    return new hitable_list(list, 3);
}

static hitable *cornell(bool smoke) {   // main.cpp:148-188
    hitable **list = new hitable *[8];
    int i = 0;
    material *red = new lambertian(new constant_texture(vec3(0.65, 0.05, 0.05)));
    material *white = new lambertian(new constant_texture(vec3(0.73, 0.73, 0.73)));
    material *green = new lambertian(new constant_texture(vec3(0.12, 0.45, 0.15)));
    material *light = new diffuse_light(new constant_texture(smoke ? vec3(4, 4, 4) : vec3(15, 15, 15)));
    list[i++] = new flip_normals(new yz_rect(0, 555, 0, 555, 555, green));
    list[i++] = new yz_rect(0, 555, 0, 555, 0, red);
    if (smoke) list[i++] = new xz_rect(113, 443, 127, 432, 554, light);
    else list[i++] = new xz_rect(213, 343, 227, 332, 554, light);
    list[i++] = new flip_normals(new xz_rect(0, 555, 0, 555, 555, white));
    list[i++] = new xz_rect(0, 555, 0, 555, 0, white);
    list[i++] = new flip_normals(new xy_rect(0, 555, 0, 555, 555, white));
    hitable *b1 = new translate(new rotate_y(new box(vec3(0, 0, 0), vec3(165, 165, 165), white), -18), vec3(130, 0, 65));
    hitable *b2 = new translate(new rotate_y(new box(vec3(0, 0, 0), vec3(165, 330, 165), white), 15), vec3(265, 0, 295));
    if (smoke) {
        list[i++] = new constant_medium(b1, 0.01, new constant_texture(vec3(1.0, 1.0, 1.0)));
        list[i++] = new constant_medium(b2, 0.01, new constant_texture(vec3(0.0, 0.0, 0.0)));
    } else {
        list[i++] = b1;
        list[i++] = b2;
    }
    return new hitable_list(list, i);
}
hitable *cornell_box() { return cornell(false); }
hitable *cornell_smoke() { return cornell(true); }

hitable *final_scene() {   // main.cpp:190-230
    const int nb = 10;
    hitable **list = new hitable *[3000];
    material *white = new lambertian(new constant_texture(vec3(0.73, 0.73, 0.73)));
    material *ground = new lambertian(new constant_texture(vec3(0.48, 0.83, 0.53)));
    int l = 0;
    for (int i = 0; i < nb; i++) {
        for (int j = 0; j < nb; j++) {
            const float w = 100;
            const float x0 = i * w, z0 = j * w, y0 = 0;
            const float x1 = x0 + w;
            const float y1 = 100 * (drand48() + 0.01);
            const float z1 = z0 + w;
            list[l++] = new box(vec3(x0, y0, z0), vec3(x1, y1, z1), ground);
        }
    }
    material *light = new diffuse_light(new constant_texture(vec3(7, 7, 7)));
    list[l++] = new xz_rect(123, 423, 147, 412, 554, light);
    const vec3 center(400, 400, 200);
    list[l++] = new moving_sphere(center, center + vec3(30, 0, 0), 0, 1, 50,
                                  new lambertian(new constant_texture(vec3(0.7, 0.3, 0.1))));
    list[l++] = new sphere(vec3(260, 150, 45), 50, new dielectric(1.5));
    list[l++] = new sphere(vec3(0, 150, 145), 50, new metal(vec3(0.8, 0.8, 0.9), 10.0));
    hitable *boundary = new sphere(vec3(360, 150, 145), 70, new dielectric(1.5));
    list[l++] = boundary;
    list[l++] = new constant_medium(boundary, 0.2, new constant_texture(vec3(0.2, 0.4, 0.9)));
    boundary = new sphere(vec3(0, 0, 0), 5000, new dielectric(1.5));
    list[l++] = new constant_medium(boundary, 0.0001, new constant_texture(vec3(1.0, 1.0, 1.0)));
    texture *pertext = new noise_texture(0.1);
    list[l++] = new sphere(vec3(220, 280, 300), 80, new lambertian(pertext));
    for (int j = 0; j < 1000; j++) {
        const double x = drand48(), y = drand48(), z = drand48();
        list[l++] = new sphere(vec3(165 * x - 100, 165 * y + 270, 165 * z + 395), 10, white);
    }
    return new hitable_list(list, l);
}

hitable *earth(const char *png_path) {   // main.cpp:87-97
    hitable **list = new hitable *[2];
    material *light = new diffuse_light(new constant_texture(vec3(7, 7, 7)));
    list[0] = new xz_rect(63, 483, 55, 482, 554, light);
    int nx, ny, nn;
    unsigned char *tex_data = stbi_load(png_path, &nx, &ny, &nn, 0);
    material *mat = new lambertian(new image_texture(tex_data, nx, ny));
    list[1] = new sphere(vec3(360, 250, 150), 100, mat);
    return new hitable_list(list, 2);
}

// Edge scenes of the tests (not in the reference's main.cpp), the same objects as
// oracle/ref_harness.cpp edge_* builds from the reference's classes: no objects;
// one sphere (a BVH that is a single leaf); degenerate geometry.
hitable *edge_empty() { return new hitable_list(new hitable *[1], 0); }

hitable *edge_single() {
    hitable **l = new hitable *[1];
    l[0] = new sphere(vec3(0, 1, 0), 1, new lambertian(new constant_texture(vec3(0.5, 0.5, 0.5))));
    return new hitable_list(l, 1);
}

hitable *edge_degenerate() {
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

hitable *build_named_scene(const std::string &name, float *time0, float *time1) {
    reset_reference_rng();
    *time0 = 0.0f;
    *time1 = 1.0f;
    if (name == "random_scene") return random_scene();
    if (name == "random_motion") return random_scene_motion();
    if (name == "cornell_box") return cornell_box();
    if (name == "cornell_smoke") return cornell_smoke();
    if (name == "final") return final_scene();
    if (name == "simple_light") return simple_light();
    if (name == "two_spheres") return two_spheres();
    if (name == "test") return test_scene();
    if (name == "edge_empty") return edge_empty();
    if (name == "edge_single") return edge_single();
    if (name == "edge_degenerate") return edge_degenerate();
    if (name == "earth") {
        const char *png = std::getenv("RTNW_EARTH_PNG");
        return earth(png ? png : "picture.png");
    }
    return nullptr;
}

}  // namespace rtnw
