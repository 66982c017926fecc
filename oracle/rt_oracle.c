/* oracle/rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 * A plain-C restatement of the reference's per-pixel sample loop.  Every
 * function cites the reference line it follows; arithmetic is written with the
 * exact float/double promotions the reference's C++ produces (float overloads
 * of sqrt/sin/atan2/asin/floor/fabs/tan, double pow/log, double literals), and
 * the library is compiled with -ffp-contract=off so no FMA is introduced.
 *
 * Two RNG sources:
 *   canonical  — the glibc drand48 LCG from state 0 (what an unseeded reference
 *                run uses; glibc stdlib/drand48-iter.c: a=0x5DEECE66D, c=0xB).
 *   counter    — one keyed stream per camera sample + keyed medium draws (the
 *                stream spec shared with the GPU kernel).
 * Scene construction always uses the canonical stream, after the 1533 draws of
 * the Perlin static initialisers (perlin.h:108-111), as the reference does.
 */
#define _GNU_SOURCE
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#define RT_MAXFLOAT 0x1.fffffep+127f /* MAXFLOAT / FLT_MAX (hitable.h:8) */

/* ------------------------------------------------------------------ vec3 */
typedef struct { float e[3]; } v3;                        /* vec3.h:12-41 */
static inline v3 V(float a, float b, float c) { v3 r; r.e[0] = a; r.e[1] = b; r.e[2] = c; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }   /* vec3.h:60 */
static inline v3 vsub(v3 a, v3 b) { return V(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }   /* vec3.h:64 */
static inline v3 vmul(v3 a, v3 b) { return V(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }   /* vec3.h:68 */
static inline v3 vscale(float t, v3 v) { return V(t * v.e[0], t * v.e[1], t * v.e[2]); }              /* vec3.h:76,84 */
static inline v3 vdivs(v3 v, float t) { return V(v.e[0] / t, v.e[1] / t, v.e[2] / t); }              /* vec3.h:80 */
static inline v3 vneg(v3 v) { return V(-v.e[0], -v.e[1], -v.e[2]); }                                 /* vec3.h:24 */
static inline float vdot(v3 a, v3 b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; } /* vec3.h:88 */
static inline v3 vcross(v3 a, v3 b) {                                                                /* vec3.h:92 */
    return V(a.e[1] * b.e[2] - a.e[2] * b.e[1], -(a.e[0] * b.e[2] - a.e[2] * b.e[0]), a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
static inline float vlen(v3 v) { return sqrtf(v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]); } /* vec3.h:35 */
static inline v3 vunit(v3 v) { return vdivs(v, vlen(v)); }                                           /* vec3.h:143 */

typedef struct { v3 A, B; float time; } ray_t;                                                        /* ray.h:11-25 */
static inline ray_t R(v3 a, v3 b, float t) { ray_t r; r.A = a; r.B = b; r.time = t; return r; }
static inline v3 ray_at(const ray_t *r, float t) { return vadd(r->A, vscale(t, r->B)); }             /* ray.h:18 */

/* ------------------------------------------------------------------- RNG */
#define LCG_A 0x5DEECE66Dull
#define LCG_C 0xBull
#define LCG_M 0xFFFFFFFFFFFFull

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t sample_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return mix64(mix64(seed ^ 0x5851F42D4C957F2Dull) ^ (((uint64_t)pixel << 32) | sample));
}

typedef struct {
    int counter;
    uint64_t x;      /* canonical LCG state */
    uint64_t key;    /* counter: sample key (the medium stream's seed) */
    uint64_t n;      /* unused */
    int nmedia;      /* counter: the scene's constant_media (the medium stream's stride per segment) */
} rng_t;

/* drand48's step (x = a x + c mod 2^48, draw = x / 2^48) in both modes: canonical is
 * one stream for the whole run; counter restarts it per sample at x = key mod 2^48
 * (rng_seed_sample), so a sample's draws do not depend on which other samples ran. */
static inline double rng_next(rng_t *g) {
    g->x = (LCG_A * g->x + LCG_C) & LCG_M;
    return (double)g->x * 0x1p-48;
}
static inline void rng_seed_sample(rng_t *g, uint64_t key) {
    g->key = key;
    g->x = key & LCG_M;
    g->n = 0;
}
/* x advanced n drand48 steps at once: x_n = A^n x + C (A^(n-1) + ... + 1) mod 2^48,
 * by squaring (the kernel walks the same sequence one step per medium and segment). */
static inline uint64_t lcg_skip(uint64_t x, uint64_t n) {
    uint64_t a = LCG_A, c = LCG_C, A = 1, C = 0;
    for (; n; n >>= 1) {
        if (n & 1) { A = (A * a) & LCG_M; C = (C * a + c) & LCG_M; }
        c = (c * (a + 1)) & LCG_M;
        a = (a * a) & LCG_M;
    }
    return (A * x + C) & LCG_M;
}
/* The constant_medium draw of medium k (list order) at segment `bounce` of the sample:
 * the medium stream is drand48's generator started at mix64(key ^ 0xD1B5..) mod 2^48
 * and stepped once per medium per segment, whether or not the medium draws, so draw
 * (bounce, k) is the stream's (bounce * nmedia + k + 1)-th value. */
static inline double rng_medium(rng_t *g, int bounce, int k) {
    if (!g->counter) return rng_next(g);
    uint64_t x0 = mix64(g->key ^ 0xD1B54A32D192ED03ull) & LCG_M;
    return (double)lcg_skip(x0, (uint64_t)bounce * (uint64_t)g->nmedia + (uint64_t)k + 1) * 0x1p-48;
}

/* ---------------------------------------------------------------- Perlin */
static v3 g_ranvec[256];
static int g_perm[3][256];

static void perlin_generate(rng_t *g) {                                  /* perlin.h:82-111 */
    for (int i = 0; i < 256; ++i) {
        double x = -1 + 2 * rng_next(g);
        double y = -1 + 2 * rng_next(g);
        double z = -1 + 2 * rng_next(g);
        g_ranvec[i] = vunit(V((float)x, (float)y, (float)z));
    }
    for (int a = 0; a < 3; a++) {
        int *p = g_perm[a];
        for (int i = 0; i < 256; i++) p[i] = i;
        for (int i = 255; i > 0; i--) {                                  /* permute, perlin.h:90-97 */
            int target = (int)(rng_next(g) * (i + 1));
            int tmp = p[i]; p[i] = p[target]; p[target] = tmp;
        }
    }
}

static float perlin_noise(v3 p) {                                        /* perlin.h:43-61 */
    float u = p.e[0] - floorf(p.e[0]);
    float v = p.e[1] - floorf(p.e[1]);
    float w = p.e[2] - floorf(p.e[2]);
    u = u * u * (3 - 2 * u);
    v = v * v * (3 - 2 * v);
    w = w * w * (3 - 2 * w);
    int i = (int)floorf(p.e[0]);
    int j = (int)floorf(p.e[1]);
    int k = (int)floorf(p.e[2]);
    v3 c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++)
                c[di][dj][dk] = g_ranvec[g_perm[0][(i + di) & 255] ^ g_perm[1][(j + dj) & 255] ^ g_perm[2][(k + dk) & 255]];
    /* perlin_interp, perlin.h:25-39 (the Hermite smoothing is applied again) */
    float uu = u * u * (3 - 2 * u);
    float vv = v * v * (3 - 2 * v);
    float ww = w * w * (3 - 2 * w);
    float accum = 0;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int d = 0; d < 2; d++) {
                v3 weight_v = V(u - a, v - b, w - d);
                accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) *
                         (d * ww + (1 - d) * (1 - ww)) * vdot(c[a][b][d], weight_v);
            }
    return accum;
}

static float perlin_turb(v3 p) {                                         /* perlin.h:64-74 */
    float accum = 0;
    v3 temp_p = p;
    float weight = 1.0;
    for (int i = 0; i < 7; i++) {
        accum += weight * perlin_noise(temp_p);
        weight = (float)(weight * 0.5);
        temp_p = V(temp_p.e[0] * 2, temp_p.e[1] * 2, temp_p.e[2] * 2);
    }
    return fabsf(accum);
}

/* -------------------------------------------------------------- textures */
enum { TX_CONST, TX_CHECKER, TX_NOISE, TX_IMAGE };
typedef struct tex_s {
    int kind; v3 color; const struct tex_s *even, *odd; float scale;
    const unsigned char *data; int nx, ny;   /* image_texture, surface_texture.h:13-16 */
} tex_t;

static v3 tex_value(const tex_t *t, float u, float v, v3 p) {
    for (;;) {
        if (t->kind == TX_CONST) return t->color;                            /* texture.h:22-24 */
        if (t->kind == TX_CHECKER) {                                          /* texture.h:35-41 */
            float sines = sinf(10 * p.e[0]) * sinf(10 * p.e[1]) * sinf(10 * p.e[2]);
            t = (sines < 0) ? t->odd : t->even;
            continue;
        }
        if (t->kind == TX_IMAGE) {                                            /* surface_texture.h:19-30 */
            int i = (int)((1 - u) * t->nx);
            int j = (int)((double)((1 - v) * t->ny) - 0.001);
            if (i < 0) i = 0;
            if (j < 0) j = 0;
            if (i > t->nx - 1) i = t->nx - 1;
            if (j > t->ny - 1) j = t->ny - 1;
            float r = (float)((int)t->data[3 * i + 3 * t->nx * j] / 255.0);
            float g = (float)((int)t->data[3 * i + 3 * t->nx * j + 1] / 255.0);
            float b = (float)((int)t->data[3 * i + 3 * t->nx * j + 2] / 255.0);
            return V(r, g, b);
        }
        /* noise_texture, texture.h:52-56 */
        float s = 1 + sinf(t->scale * p.e[0] + 5 * perlin_turb(vscale(t->scale, p)));
        v3 half = V(0.5f * 1, 0.5f * 1, 0.5f * 1);
        return V(s * half.e[0], s * half.e[1], s * half.e[2]);
    }
}

/* ------------------------------------------------------------- materials */
enum { MT_LAMBERT, MT_METAL, MT_DIELECTRIC, MT_LIGHT, MT_ISOTROPIC };
typedef struct mat_s { int kind; const tex_t *tex; v3 albedo; float fuzz; float ri; } mat_t;

typedef struct { float t, u, v; v3 p, normal; const mat_t *mat; } hit_t;   /* hitable.h:21-29 */

static v3 random_in_unit_sphere(rng_t *g) {                               /* material.h:41-47 */
    v3 p;
    do {
        double x = rng_next(g), y = rng_next(g), z = rng_next(g);
        p = vsub(vscale(2.0f, V((float)x, (float)y, (float)z)), V(1, 1, 1));
    } while (vdot(p, p) >= 1.0);
    return p;
}
static v3 reflect(v3 v, v3 n) { return vsub(v, vscale(2 * vdot(v, n), n)); }   /* material.h:36-38 */
static int refract(v3 v, v3 n, float ni_over_nt, v3 *refracted) {              /* material.h:23-33 */
    v3 uv = vunit(v);
    float dt = vdot(uv, n);
    float discriminant = (float)(1.0 - (double)(ni_over_nt * ni_over_nt * (1 - dt * dt)));
    if (discriminant > 0) {
        *refracted = vsub(vscale(ni_over_nt, vsub(uv, vscale(dt, n))), vscale(sqrtf(discriminant), n));
        return 1;
    }
    return 0;
}
static float schlick(float cosine, float ref_idx) {                            /* material.h:16-20 */
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return (float)(r0 + (double)(1 - r0) * pow((double)(1 - cosine), 5.0));
}

static v3 mat_emitted(const mat_t *m, float u, float v, v3 p) {                 /* material.h:56,134 */
    if (m->kind == MT_LIGHT) return tex_value(m->tex, u, v, p);
    return V(0, 0, 0);
}

static int mat_scatter(const mat_t *m, const ray_t *r_in, const hit_t *rec, v3 *att, ray_t *scattered, rng_t *g) {
    switch (m->kind) {
    case MT_LAMBERT: {                                                          /* material.h:64-69 */
        v3 target = vadd(vadd(rec->p, rec->normal), random_in_unit_sphere(g));
        *scattered = R(rec->p, vsub(target, rec->p), r_in->time);
        *att = tex_value(m->tex, rec->u, rec->v, rec->p);
        return 1;
    }
    case MT_METAL: {                                                            /* material.h:77-82 */
        v3 reflected = reflect(vunit(r_in->B), rec->normal);
        *scattered = R(rec->p, vadd(reflected, vscale(m->fuzz, random_in_unit_sphere(g))), 0.0f);
        *att = m->albedo;
        return vdot(scattered->B, rec->normal) > 0;
    }
    case MT_DIELECTRIC: {                                                       /* material.h:90-120 */
        v3 outward_normal;
        v3 reflected = reflect(r_in->B, rec->normal);
        float ni_over_nt;
        *att = V(1.0f, 1.0f, 1.0f);
        v3 refracted = V(0, 0, 0);
        float reflect_prob, cosine;
        float ref_idx = m->ri;
        if (vdot(r_in->B, rec->normal) > 0) {
            outward_normal = vneg(rec->normal);
            ni_over_nt = ref_idx;
            cosine = vdot(r_in->B, rec->normal) / vlen(r_in->B);
            cosine = sqrtf(1 - ref_idx * ref_idx * (1 - cosine * cosine));
        } else {
            outward_normal = rec->normal;
            ni_over_nt = (float)(1.0 / (double)ref_idx);
            cosine = -vdot(r_in->B, rec->normal) / vlen(r_in->B);
        }
        if (refract(r_in->B, outward_normal, ni_over_nt, &refracted))
            reflect_prob = schlick(cosine, ref_idx);
        else
            reflect_prob = 1.0f;
        if (rng_next(g) < reflect_prob)
            *scattered = R(rec->p, reflected, 0.0f);
        else
            *scattered = R(rec->p, refracted, 0.0f);
        return 1;
    }
    case MT_ISOTROPIC:                                                          /* material.h:145-149 */
        *scattered = R(rec->p, random_in_unit_sphere(g), 0.0f);
        *att = tex_value(m->tex, rec->u, rec->v, rec->p);
        return 1;
    default:                                                                    /* diffuse_light, material.h:130-132 */
        return 0;
    }
}

/* ------------------------------------------------------------- geometry */
enum { OB_LIST, OB_SPHERE, OB_MSPHERE, OB_XY, OB_XZ, OB_YZ, OB_BOX, OB_FLIP, OB_TRANSLATE, OB_ROTY, OB_MEDIUM };
typedef struct obj_s {
    int kind;
    v3 c0, c1; float r, t0, t1;          /* spheres */
    float a0, a1, b0, b1, k;             /* rects: (x0,x1,y0,y1) / (x0,x1,z0,z1) / (y0,y1,z0,z1) */
    const mat_t *mat;
    struct obj_s **kids; int nkids;      /* list / box */
    struct obj_s *child;                 /* flip / translate / rotate / medium boundary */
    v3 offset; float sin_t, cos_t;       /* translate / rotate_y */
    float density; int ordinal;          /* medium */
} obj_t;

typedef struct {
    rng_t *g;
    int bounce;
    int skip_media;
} hctx_t;

static void sphere_uv(v3 p, float *u, float *v) {                       /* hitable.h:14-19 */
    float phi = atan2f(p.e[2], p.e[0]);
    float theta = asinf(p.e[1]);
    *u = (float)(1 - ((double)phi + M_PI) / (2 * M_PI));
    *v = (float)(((double)theta + M_PI / 2) / M_PI);
}

static inline v3 msphere_center(const obj_t *o, float time) {          /* sphere.h:81-83 */
    return vadd(o->c0, vscale((time - o->t0) / (o->t1 - o->t0), vsub(o->c1, o->c0)));
}

static int obj_hit(const obj_t *o, const ray_t *r, float tmin, float tmax, hit_t *rec, hctx_t *cx);

static int medium_hit(const obj_t *o, const ray_t *r, float t_min, float t_max, hit_t *rec, hctx_t *cx) {
    /* constant_medium::hit, constant_medium.h:26-50 */
    hit_t rec1, rec2;
    memset(&rec1, 0, sizeof rec1); memset(&rec2, 0, sizeof rec2);
    if (obj_hit(o->child, r, -FLT_MAX, FLT_MAX, &rec1, cx)) {
        if (obj_hit(o->child, r, (float)(rec1.t + 0.0001), FLT_MAX, &rec2, cx)) {
            if (rec1.t < t_min) rec1.t = t_min;
            if (rec2.t > t_max) rec2.t = t_max;
            if (rec1.t >= rec2.t) return 0;
            if (rec1.t < 0) rec1.t = 0;
            float distance_inside_boundary = (rec2.t - rec1.t) * vlen(r->B);
            float hit_distance = (float)(-(1 / o->density) * log(rng_medium(cx->g, cx->bounce, o->ordinal)));
            if (hit_distance < distance_inside_boundary) {
                rec->t = rec1.t + hit_distance / vlen(r->B);
                rec->p = ray_at(r, rec->t);
                rec->normal = V(1, 0, 0);
                rec->mat = o->mat;
                return 1;
            }
        }
    }
    return 0;
}

static int obj_hit(const obj_t *o, const ray_t *r, float tmin, float tmax, hit_t *rec, hctx_t *cx) {
    switch (o->kind) {
    case OB_LIST: {                                                       /* hitable_list.h:20-32 */
        hit_t temp_rec;
        memset(&temp_rec, 0, sizeof temp_rec);
        int hit_anything = 0;
        double closest_so_far = tmax;
        for (int i = 0; i < o->nkids; i++) {
            if (obj_hit(o->kids[i], r, tmin, (float)closest_so_far, &temp_rec, cx)) {
                hit_anything = 1;
                closest_so_far = temp_rec.t;
                *rec = temp_rec;
            }
        }
        return hit_anything;
    }
    case OB_SPHERE: {                                                     /* sphere.h:25-52 */
        v3 oc = vsub(r->A, o->c0);
        float a = vdot(r->B, r->B);
        float b = vdot(oc, r->B);
        float c = vdot(oc, oc) - o->r * o->r;
        float discriminant = b * b - a * c;
        if (discriminant > 0) {
            float temp = (-b - sqrtf(discriminant)) / a;
            if (!(temp < tmax && temp > tmin)) temp = (-b + sqrtf(discriminant)) / a;
            if (temp < tmax && temp > tmin) {
                rec->t = temp;
                rec->p = ray_at(r, rec->t);
                sphere_uv(vdivs(vsub(rec->p, o->c0), o->r), &rec->u, &rec->v);
                rec->normal = vdivs(vsub(rec->p, o->c0), o->r);
                rec->mat = o->mat;
                return 1;
            }
        }
        return 0;
    }
    case OB_MSPHERE: {                                                    /* sphere.h:92-118 */
        v3 oc = vsub(r->A, msphere_center(o, r->time));
        float a = vdot(r->B, r->B);
        float b = vdot(oc, r->B);
        float c = vdot(oc, oc) - o->r * o->r;
        float discriminant = b * b - a * c;
        if (discriminant > 0) {
            float temp = (-b - sqrtf(discriminant)) / a;
            if (!(temp < tmax && temp > tmin)) temp = (-b + sqrtf(discriminant)) / a;
            if (temp < tmax && temp > tmin) {
                rec->t = temp;
                rec->p = ray_at(r, rec->t);
                rec->normal = vdivs(vsub(rec->p, msphere_center(o, r->time)), o->r);
                rec->mat = o->mat;
                return 1;
            }
        }
        return 0;
    }
    case OB_XY: case OB_XZ: case OB_YZ: {                                  /* aarect.h:50-100 */
        int ax = o->kind == OB_XY ? 2 : (o->kind == OB_XZ ? 1 : 0);
        int ia = o->kind == OB_YZ ? 1 : 0;
        int ib = o->kind == OB_XY ? 1 : 2;
        float t = (o->k - r->A.e[ax]) / r->B.e[ax];
        if (t < tmin || t > tmax) return 0;
        float a = r->A.e[ia] + t * r->B.e[ia];
        float b = r->A.e[ib] + t * r->B.e[ib];
        if (a < o->a0 || a > o->a1 || b < o->b0 || b > o->b1) return 0;
        rec->u = (a - o->a0) / (o->a1 - o->a0);
        rec->v = (b - o->b0) / (o->b1 - o->b0);
        rec->t = t;
        rec->mat = o->mat;
        rec->p = ray_at(r, t);
        rec->normal = V(ax == 0, ax == 1, ax == 2);
        return 1;
    }
    case OB_BOX:                                                          /* box.h:36-38 */
        return obj_hit(o->child, r, tmin, tmax, rec, cx);
    case OB_FLIP:                                                         /* hitable.h:42-49 */
        if (obj_hit(o->child, r, tmin, tmax, rec, cx)) { rec->normal = vneg(rec->normal); return 1; }
        return 0;
    case OB_TRANSLATE: {                                                  /* hitable.h:66-74 */
        ray_t moved = R(vsub(r->A, o->offset), r->B, r->time);
        if (obj_hit(o->child, &moved, tmin, tmax, rec, cx)) { rec->p = vadd(rec->p, o->offset); return 1; }
        return 0;
    }
    case OB_ROTY: {                                                       /* hitable.h:128-150 */
        v3 origin = r->A, direction = r->B;
        float c = o->cos_t, s = o->sin_t;
        origin.e[0] = c * r->A.e[0] - s * r->A.e[2];
        origin.e[2] = s * r->A.e[0] + c * r->A.e[2];
        direction.e[0] = c * r->B.e[0] - s * r->B.e[2];
        direction.e[2] = s * r->B.e[0] + c * r->B.e[2];
        ray_t rotated = R(origin, direction, r->time);
        if (obj_hit(o->child, &rotated, tmin, tmax, rec, cx)) {
            v3 p = rec->p, normal = rec->normal;
            p.e[0] = c * rec->p.e[0] + s * rec->p.e[2];
            p.e[2] = -s * rec->p.e[0] + c * rec->p.e[2];
            normal.e[0] = c * rec->normal.e[0] + s * rec->normal.e[2];
            normal.e[2] = -s * rec->normal.e[0] + c * rec->normal.e[2];
            rec->p = p;
            rec->normal = normal;
            return 1;
        }
        return 0;
    }
    case OB_MEDIUM:
        if (cx->skip_media) return 0;
        return medium_hit(o, r, tmin, tmax, rec, cx);
    }
    return 0;
}

/* ----------------------------------------------------------------- scene */
typedef struct {
    void **blocks; int nblocks, cap;
    obj_t *world;
    obj_t *media[64]; int nmedia;
} scene_t;

static void *arena_alloc(scene_t *s, size_t n) {
    void *p = calloc(1, n);
    if (s->nblocks == s->cap) { s->cap = s->cap ? 2 * s->cap : 256; s->blocks = realloc(s->blocks, s->cap * sizeof(void *)); }
    s->blocks[s->nblocks++] = p;
    return p;
}
static void scene_free(scene_t *s) {
    for (int i = 0; i < s->nblocks; i++) free(s->blocks[i]);
    free(s->blocks);
}

static tex_t *t_const(scene_t *s, double r, double g, double b) {
    tex_t *t = arena_alloc(s, sizeof *t); t->kind = TX_CONST; t->color = V((float)r, (float)g, (float)b); return t;
}
static tex_t *t_checker(scene_t *s, const tex_t *even, const tex_t *odd) {
    tex_t *t = arena_alloc(s, sizeof *t); t->kind = TX_CHECKER; t->even = even; t->odd = odd; return t;
}
static tex_t *t_noise(scene_t *s, double scale) {
    tex_t *t = arena_alloc(s, sizeof *t); t->kind = TX_NOISE; t->scale = (float)scale; return t;
}
static mat_t *m_lambert(scene_t *s, const tex_t *t) { mat_t *m = arena_alloc(s, sizeof *m); m->kind = MT_LAMBERT; m->tex = t; return m; }
static mat_t *m_light(scene_t *s, const tex_t *t) { mat_t *m = arena_alloc(s, sizeof *m); m->kind = MT_LIGHT; m->tex = t; return m; }
static mat_t *m_iso(scene_t *s, const tex_t *t) { mat_t *m = arena_alloc(s, sizeof *m); m->kind = MT_ISOTROPIC; m->tex = t; return m; }
static mat_t *m_dielectric(scene_t *s, double ri) { mat_t *m = arena_alloc(s, sizeof *m); m->kind = MT_DIELECTRIC; m->ri = (float)ri; return m; }
static mat_t *m_metal(scene_t *s, v3 a, float f) {                       /* material.h:76 */
    mat_t *m = arena_alloc(s, sizeof *m); m->kind = MT_METAL; m->albedo = a; m->fuzz = (f < 1) ? f : 1; return m;
}

static obj_t *o_new(scene_t *s, int kind) { obj_t *o = arena_alloc(s, sizeof *o); o->kind = kind; return o; }
static obj_t *o_sphere(scene_t *s, v3 c, float r, const mat_t *m) { obj_t *o = o_new(s, OB_SPHERE); o->c0 = c; o->r = r; o->mat = m; return o; }
static obj_t *o_msphere(scene_t *s, v3 c0, v3 c1, float t0, float t1, float r, const mat_t *m) {
    obj_t *o = o_new(s, OB_MSPHERE); o->c0 = c0; o->c1 = c1; o->t0 = t0; o->t1 = t1; o->r = r; o->mat = m; return o;
}
static obj_t *o_rect(scene_t *s, int kind, float a0, float a1, float b0, float b1, float k, const mat_t *m) {
    obj_t *o = o_new(s, kind); o->a0 = a0; o->a1 = a1; o->b0 = b0; o->b1 = b1; o->k = k; o->mat = m; return o;
}
static obj_t *o_flip(scene_t *s, obj_t *c) { obj_t *o = o_new(s, OB_FLIP); o->child = c; return o; }
static obj_t *o_list(scene_t *s, obj_t **kids, int n) { obj_t *o = o_new(s, OB_LIST); o->kids = kids; o->nkids = n; return o; }
static obj_t **o_array(scene_t *s, int n) { return arena_alloc(s, sizeof(obj_t *) * (size_t)n); }
static obj_t *o_box(scene_t *s, v3 p0, v3 p1, const mat_t *m) {         /* box.h:23-34 */
    obj_t **l = o_array(s, 6);
    l[0] = o_rect(s, OB_XY, p0.e[0], p1.e[0], p0.e[1], p1.e[1], p1.e[2], m);
    l[1] = o_flip(s, o_rect(s, OB_XY, p0.e[0], p1.e[0], p0.e[1], p1.e[1], p0.e[2], m));
    l[2] = o_rect(s, OB_XZ, p0.e[0], p1.e[0], p0.e[2], p1.e[2], p1.e[1], m);
    l[3] = o_flip(s, o_rect(s, OB_XZ, p0.e[0], p1.e[0], p0.e[2], p1.e[2], p0.e[1], m));
    l[4] = o_rect(s, OB_YZ, p0.e[1], p1.e[1], p0.e[2], p1.e[2], p1.e[0], m);
    l[5] = o_flip(s, o_rect(s, OB_YZ, p0.e[1], p1.e[1], p0.e[2], p1.e[2], p0.e[0], m));
    obj_t *o = o_new(s, OB_BOX);
    o->c0 = p0; o->c1 = p1;
    o->child = o_list(s, l, 6);
    return o;
}
static obj_t *o_translate(scene_t *s, obj_t *c, v3 off) { obj_t *o = o_new(s, OB_TRANSLATE); o->child = c; o->offset = off; return o; }
static obj_t *o_rotate_y(scene_t *s, obj_t *c, float angle) {            /* hitable.h:98-101 */
    obj_t *o = o_new(s, OB_ROTY); o->child = c;
    float radians = (float)((M_PI / 180.) * angle);
    o->sin_t = sinf(radians);
    o->cos_t = cosf(radians);
    return o;
}
static obj_t *o_medium(scene_t *s, obj_t *boundary, float d, const tex_t *a) {   /* constant_medium.h:16 */
    obj_t *o = o_new(s, OB_MEDIUM); o->child = boundary; o->density = d; o->mat = m_iso(s, a); return o;
}

static obj_t *build_random(scene_t *s, rng_t *g, int motion) {         /* main.cpp:49-85 / TNW Ch01:36-67 */
    obj_t **list = o_array(s, 501);
    tex_t *checker = t_checker(s, t_const(s, 0.2, 0.3, 0.1), t_const(s, 0.9, 0.9, 0.9));
    list[0] = o_sphere(s, V(0, -700, 0), 700, m_lambert(s, checker));
    int i = 1;
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            float choose_mat = (float)rng_next(g);
            double dx = rng_next(g), dz = rng_next(g);
            v3 center = V((float)(a + 0.9 * dx), 0.2f, (float)(b + 0.9 * dz));
            if (vlen(vsub(center, V(4, 0.2f, 0))) > 0.9) {
                if (choose_mat < 0.8) {
                    if (motion) {
                        double dy = rng_next(g);
                        v3 c1 = vadd(center, V(0, (float)(0.5 * dy), 0));
                        double r0 = rng_next(g), r1 = rng_next(g), g0 = rng_next(g), g1 = rng_next(g), b0 = rng_next(g), b1 = rng_next(g);
                        list[i++] = o_msphere(s, center, c1, 0.0f, 1.0f, 0.2f,
                                              m_lambert(s, t_const(s, r0 * r1, g0 * g1, b0 * b1)));
                    }
                } else if (choose_mat < 0.95) {
                    double x = rng_next(g), y = rng_next(g), z = rng_next(g);
                    double f = rng_next(g);
                    list[i++] = o_sphere(s, center, 0.2f,
                                         m_metal(s, V((float)(0.5 * (1 + x)), (float)(0.5 * (1 + y)), (float)(0.5 * (1 + z))), (float)(0.5 * f)));
                } else {
                    list[i++] = o_sphere(s, center, 0.2f, m_dielectric(s, 1.5));
                }
            }
        }
    }
    list[i++] = o_sphere(s, V(0, 1, 0), 1.0f, m_dielectric(s, 2.5));
    list[i++] = o_sphere(s, V(-4, 1, 0), 1.0f, m_lambert(s, t_const(s, 0.4, 0.2, 0.1)));
    list[i++] = o_sphere(s, V(4, 1, 0), 1.0f, m_metal(s, V(1, 1, 1), 0.0f));
    return o_list(s, list, i);
}

static obj_t *build_cornell(scene_t *s, int smoke) {                      /* main.cpp:148-188 */
    obj_t **list = o_array(s, 8);
    int i = 0;
    mat_t *red = m_lambert(s, t_const(s, 0.65, 0.05, 0.05));
    mat_t *white = m_lambert(s, t_const(s, 0.73, 0.73, 0.73));
    mat_t *green = m_lambert(s, t_const(s, 0.12, 0.45, 0.15));
    mat_t *light = m_light(s, smoke ? t_const(s, 4, 4, 4) : t_const(s, 15, 15, 15));
    list[i++] = o_flip(s, o_rect(s, OB_YZ, 0, 555, 0, 555, 555, green));
    list[i++] = o_rect(s, OB_YZ, 0, 555, 0, 555, 0, red);
    if (smoke) list[i++] = o_rect(s, OB_XZ, 113, 443, 127, 432, 554, light);
    else list[i++] = o_rect(s, OB_XZ, 213, 343, 227, 332, 554, light);
    list[i++] = o_flip(s, o_rect(s, OB_XZ, 0, 555, 0, 555, 555, white));
    list[i++] = o_rect(s, OB_XZ, 0, 555, 0, 555, 0, white);
    list[i++] = o_flip(s, o_rect(s, OB_XY, 0, 555, 0, 555, 555, white));
    obj_t *b1 = o_translate(s, o_rotate_y(s, o_box(s, V(0, 0, 0), V(165, 165, 165), white), -18), V(130, 0, 65));
    obj_t *b2 = o_translate(s, o_rotate_y(s, o_box(s, V(0, 0, 0), V(165, 330, 165), white), 15), V(265, 0, 295));
    if (smoke) {
        list[i++] = o_medium(s, b1, 0.01f, t_const(s, 1.0, 1.0, 1.0));
        list[i++] = o_medium(s, b2, 0.01f, t_const(s, 0.0, 0.0, 0.0));
    } else {
        list[i++] = b1;
        list[i++] = b2;
    }
    return o_list(s, list, i);
}

static obj_t *build_final(scene_t *s, rng_t *g) {                         /* main.cpp:190-230 */
    int nb = 10;
    obj_t **list = o_array(s, 3000);
    mat_t *white = m_lambert(s, t_const(s, 0.73, 0.73, 0.73));
    mat_t *ground = m_lambert(s, t_const(s, 0.48, 0.83, 0.53));
    int l = 0;
    for (int i = 0; i < nb; i++) {
        for (int j = 0; j < nb; j++) {
            float w = 100;
            float x0 = i * w, z0 = j * w, y0 = 0;
            float x1 = x0 + w;
            float y1 = (float)(100 * (rng_next(g) + 0.01));
            float z1 = z0 + w;
            list[l++] = o_box(s, V(x0, y0, z0), V(x1, y1, z1), ground);
        }
    }
    mat_t *light = m_light(s, t_const(s, 7, 7, 7));
    list[l++] = o_rect(s, OB_XZ, 123, 423, 147, 412, 554, light);
    v3 center = V(400, 400, 200);
    list[l++] = o_msphere(s, center, vadd(center, V(30, 0, 0)), 0, 1, 50, m_lambert(s, t_const(s, 0.7, 0.3, 0.1)));
    list[l++] = o_sphere(s, V(260, 150, 45), 50, m_dielectric(s, 1.5));
    list[l++] = o_sphere(s, V(0, 150, 145), 50, m_metal(s, V(0.8f, 0.8f, 0.9f), 10.0f));
    obj_t *boundary = o_sphere(s, V(360, 150, 145), 70, m_dielectric(s, 1.5));
    list[l++] = boundary;
    list[l++] = o_medium(s, boundary, 0.2f, t_const(s, 0.2, 0.4, 0.9));
    boundary = o_sphere(s, V(0, 0, 0), 5000, m_dielectric(s, 1.5));
    list[l++] = o_medium(s, boundary, 0.0001f, t_const(s, 1.0, 1.0, 1.0));
    tex_t *pertext = t_noise(s, 0.1);
    list[l++] = o_sphere(s, V(220, 280, 300), 80, m_lambert(s, pertext));
    for (int j = 0; j < 1000; j++) {
        double x = rng_next(g), y = rng_next(g), z = rng_next(g);
        list[l++] = o_sphere(s, V((float)(165 * x - 100), (float)(165 * y + 270), (float)(165 * z + 395)), 10, white);
    }
    return o_list(s, list, l);
}

static obj_t *build_simple_light(scene_t *s) {                            /* main.cpp:122-133 */
    tex_t *pertext = t_noise(s, 4);
    tex_t *checker = t_checker(s, t_const(s, 0.2, 0.3, 0.1), t_const(s, 0.9, 0.9, 0.9));
    obj_t **list = o_array(s, 4);
    int i = 0;
    list[i++] = o_sphere(s, V(0, 2, 0), 2, m_lambert(s, pertext));
    list[i++] = o_sphere(s, V(0, -700, 0), 700, m_lambert(s, checker));
    list[i++] = o_sphere(s, V(0, 7, 0), 2, m_light(s, t_const(s, 4, 4, 4)));
    list[i++] = o_rect(s, OB_XY, 3, 5, 1, 3, -2, m_light(s, t_const(s, 4, 4, 4)));
    return o_list(s, list, i);
}

static obj_t *build_two_spheres(scene_t *s) {                             /* main.cpp:99-110 */
    m_light(s, t_const(s, 15, 15, 15));
    t_checker(s, t_const(s, 0.2, 0.3, 0.1), t_const(s, 0.9, 0.9, 0.9));
    mat_t *red = m_lambert(s, t_const(s, 0.65, 0.05, 0.05));
    obj_t **list = o_array(s, 51);
    list[0] = o_sphere(s, V(0, -10, 0), 10, red);
    list[1] = o_rect(s, OB_YZ, 0, 555, 0, 555, 0, red);
    return o_list(s, list, 2);
}

static unsigned char *g_image;
static int g_image_nx, g_image_ny;

void oracle_set_image(const uint8_t *data, int nx, int ny, int nn) {
    free(g_image);
    g_image = malloc((size_t)nx * ny * nn);
    memcpy(g_image, data, (size_t)nx * ny * nn);
    g_image_nx = nx;
    g_image_ny = ny;
}

static obj_t *build_earth(scene_t *s) {                                   /* main.cpp:87-97 */
    obj_t **list = o_array(s, 2);
    mat_t *light = m_light(s, t_const(s, 7, 7, 7));
    list[0] = o_rect(s, OB_XZ, 63, 483, 55, 482, 554, light);
    tex_t *t = arena_alloc(s, sizeof *t);
    t->kind = TX_IMAGE; t->data = g_image; t->nx = g_image_nx; t->ny = g_image_ny;
    list[1] = o_sphere(s, V(360, 250, 150), 100, m_lambert(s, t));
    return o_list(s, list, 2);
}

static obj_t *build_test(scene_t *s) {                                    /* main.cpp:135-145 */
    tex_t *pertext = t_noise(s, 4);
    tex_t *checker = t_checker(s, t_const(s, 0.2, 0.3, 0.1), t_const(s, 0.9, 0.9, 0.9));
    obj_t **list = o_array(s, 4);
    list[0] = o_sphere(s, V(0, -700, 0), 700, m_lambert(s, checker));
    list[1] = o_sphere(s, V(0, 2, 0), 2, m_lambert(s, pertext));
    list[2] = o_sphere(s, V(0, 7, 0), 2, m_light(s, t_const(s, 11, 11, 11)));
    return o_list(s, list, 3);
}

/* Edge scenes of the tests, the same objects as oracle/ref_harness.cpp edge_*. */
static obj_t *build_edge_empty(scene_t *s) { return o_list(s, o_array(s, 1), 0); }
static obj_t *build_edge_single(scene_t *s) {
    obj_t **list = o_array(s, 1);
    list[0] = o_sphere(s, V(0, 1, 0), 1, m_lambert(s, t_const(s, 0.5, 0.5, 0.5)));
    return o_list(s, list, 1);
}
static obj_t *build_edge_degenerate(scene_t *s) {
    obj_t **list = o_array(s, 11);
    int i = 0;
    mat_t *glass = m_dielectric(s, 1.5);
    list[i++] = o_sphere(s, V(0, -1000, 0), 1000, m_lambert(s, t_const(s, 0.5, 0.5, 0.5)));
    list[i++] = o_sphere(s, V(0, 1, 0), 0, m_lambert(s, t_const(s, 0.8, 0.3, 0.3)));
    list[i++] = o_sphere(s, V(-2.5f, 1, 0), -1, glass);
    list[i++] = o_sphere(s, V(2.5f, 1, 0), 1, glass);
    list[i++] = o_sphere(s, V(2.5f, 1, 0), -0.9f, glass);
    list[i++] = o_rect(s, OB_XZ, -1, -1, -1, 1, 0.5f, m_light(s, t_const(s, 4, 4, 4)));
    list[i++] = o_msphere(s, V(1, 0.5f, 1.5f), V(1, 0.5f, 2), 0.5f, 0.5f, 0.5f, m_lambert(s, t_const(s, 0.2, 0.8, 0.2)));
    list[i++] = o_sphere(s, V(-1, 0.7f, 1.5f), 0.7f, m_metal(s, V(0.7f, 0.6f, 0.5f), 1.5f));
    list[i++] = o_medium(s, o_sphere(s, V(1, 0.5f, -1.5f), 0.5f, glass), 0, t_const(s, 1, 1, 1));
    list[i++] = o_medium(s, o_sphere(s, V(-1, 0.5f, -1.5f), 0.5f, glass), 1e30f, t_const(s, 0.9, 0.9, 0.9));
    list[i++] = o_flip(s, o_rect(s, OB_XY, -3, 3, 0, 3, -3, m_light(s, t_const(s, 2, 2, 2))));
    return o_list(s, list, i);
}

static void collect_media(scene_t *s, obj_t *o) {
    switch (o->kind) {
    case OB_LIST: for (int i = 0; i < o->nkids; i++) collect_media(s, o->kids[i]); break;
    case OB_BOX: case OB_FLIP: case OB_TRANSLATE: case OB_ROTY: collect_media(s, o->child); break;
    case OB_MEDIUM: o->ordinal = s->nmedia; s->media[s->nmedia++] = o; break;
    default: break;
    }
}

/* Fresh reference process: drand48 state 0, Perlin static init, then the scene.
 * *g_after receives the canonical stream state the reference's pixel loop starts from. */
static int scene_build(scene_t *s, int which, rng_t *g_after) {
    memset(s, 0, sizeof *s);
    rng_t g; memset(&g, 0, sizeof g);
    perlin_generate(&g);
    switch (which) {
    case ORACLE_SCENE_RANDOM: s->world = build_random(s, &g, 0); break;
    case ORACLE_SCENE_RANDOM_MOTION: s->world = build_random(s, &g, 1); break;
    case ORACLE_SCENE_CORNELL: s->world = build_cornell(s, 0); break;
    case ORACLE_SCENE_CORNELL_SMOKE: s->world = build_cornell(s, 1); break;
    case ORACLE_SCENE_FINAL: s->world = build_final(s, &g); break;
    case ORACLE_SCENE_SIMPLE_LIGHT: s->world = build_simple_light(s); break;
    case ORACLE_SCENE_TWO_SPHERES: s->world = build_two_spheres(s); break;
    case ORACLE_SCENE_TEST: s->world = build_test(s); break;
    case ORACLE_SCENE_EARTH: if (!g_image) return -1; s->world = build_earth(s); break;
    case ORACLE_SCENE_EDGE_EMPTY: s->world = build_edge_empty(s); break;
    case ORACLE_SCENE_EDGE_SINGLE: s->world = build_edge_single(s); break;
    case ORACLE_SCENE_EDGE_DEGENERATE: s->world = build_edge_degenerate(s); break;
    default: return -1;
    }
    collect_media(s, s->world);
    if (g_after) *g_after = g;
    return 0;
}

/* ---------------------------------------------------------------- camera */
typedef struct { v3 origin, u, v, w, horizontal, vertical, llc; float lens_radius, time0, time1; } cam_t;

static cam_t camera_make(v3 lookfrom, v3 lookat, v3 vup, float vfov, float aspect, float aperture, float focus_dist,
                         float t0, float t1) {                           /* camera.h:21-39 */
    cam_t c;
    c.time0 = t0; c.time1 = t1;
    c.lens_radius = aperture / 2;
    float theta = (float)(vfov * M_PI / 180);
    float half_height = tanf(theta / 2);
    float half_width = aspect * half_height;
    c.origin = lookfrom;
    c.w = vunit(vsub(lookfrom, lookat));
    c.u = vunit(vcross(vup, c.w));
    c.v = vcross(c.w, c.u);
    c.llc = vsub(vsub(vsub(c.origin, vscale(half_width * focus_dist, c.u)), vscale(half_height * focus_dist, c.v)),
                 vscale(focus_dist, c.w));
    c.horizontal = vscale(2 * half_width * focus_dist, c.u);
    c.vertical = vscale(2 * half_height * focus_dist, c.v);
    return c;
}

static cam_t camera_preset(int which, int nx, int ny) {
    float aspect = (float)nx / (float)ny;
    switch (which) {
    case ORACLE_CAM_RANDOM: return camera_make(V(13, 2, 3), V(0, 0, 0), V(0, 1, 0), 20, aspect, 0.1f, 10.0f, 0.0f, 1.0f);
    case ORACLE_CAM_FINAL_ALT: return camera_make(V(478, 278, -600), V(278, 278, 0), V(0, 1, 0), 20, aspect, 0.0f, 10.0f, 0.0f, 1.0f);
    default: return camera_make(V(228, 278, -800), V(278, 278, 0), V(0, 1, 0), 40.0f, aspect, 0.0f, 10.0f, 0.0f, 1.0f);
    }
}

static ray_t camera_get_ray(const cam_t *c, float s, float t, rng_t *g) {   /* camera.h:41-56 */
    v3 p;
    do {
        double a = rng_next(g), b = rng_next(g);
        p = vsub(vscale(2.0f, V((float)a, (float)b, 0)), V(1, 1, 0));
    } while (vdot(p, p) >= 1.0);
    v3 rd = vscale(c->lens_radius, p);
    v3 offset = vadd(vscale(rd.e[0], c->u), vscale(rd.e[1], c->v));
    float time = (float)(c->time0 + rng_next(g) * (double)(c->time1 - c->time0));
    return R(vadd(c->origin, offset),
             vsub(vsub(vadd(vadd(c->llc, vscale(s, c->horizontal)), vscale(t, c->vertical)), c->origin), offset), time);
}

/* ------------------------------------------------------------ integrator */
typedef struct {
    const scene_t *sc;
    const oracle_params *p;
    double segments;
} run_t;

static int world_hit(run_t *rn, const ray_t *r, hit_t *rec, rng_t *g, int depth) {
    hctx_t cx = { g, depth, rn->p->media_after };
    rn->segments += 1;
    int hit = obj_hit(rn->sc->world, r, rn->p->tmin, RT_MAXFLOAT, rec, &cx);
    if (rn->p->media_after) {               /* kernel order: media after the surface pass */
        float closest = hit ? rec->t : RT_MAXFLOAT;
        cx.skip_media = 0;
        for (int m = 0; m < rn->sc->nmedia; m++) {
            hit_t temp = *rec;
            if (medium_hit(rn->sc->media[m], r, rn->p->tmin, closest, &temp, &cx)) {
                hit = 1; closest = temp.t; *rec = temp;
            }
        }
    }
    return hit;
}

static v3 background(const oracle_params *p, const ray_t *r) {
    if (p->background == 1) {                                            /* TNW/Chapter03:29-31 */
        v3 unit_direction = vunit(r->B);
        float t = (float)(0.5 * (unit_direction.e[1] + 1.0));
        v3 a = vscale((float)(1.0 - t), V(1.0f, 1.0f, 1.0f));
        v3 b = vscale(t, V(0.5f, 0.7f, 1.0f));
        return vadd(a, b);
    }
    return V(0, 0, 0);                                                    /* main.cpp:44 */
}

static v3 color_right(run_t *rn, const ray_t *r, int depth, rng_t *g) {    /* main.cpp:25-46 */
    hit_t rec;
    memset(&rec, 0, sizeof rec);
    if (world_hit(rn, r, &rec, g, depth)) {
        ray_t scattered;
        v3 attenuation;
        v3 emitted = mat_emitted(rec.mat, rec.u, rec.v, rec.p);
        if (depth < rn->p->max_depth && mat_scatter(rec.mat, r, &rec, &attenuation, &scattered, g))
            return vadd(emitted, vmul(attenuation, color_right(rn, &scattered, depth + 1, g)));
        return emitted;
    }
    return background(rn->p, r);
}

static v3 color_forward(run_t *rn, ray_t r, rng_t *g) {   /* the kernel's iterative form of main.cpp:25-46 */
    v3 beta = V(1, 1, 1);
    for (int depth = 0;; depth++) {
        hit_t rec;
        memset(&rec, 0, sizeof rec);
        if (!world_hit(rn, &r, &rec, g, depth)) return vmul(beta, background(rn->p, &r));
        ray_t scattered;
        v3 attenuation;
        v3 emitted = mat_emitted(rec.mat, rec.u, rec.v, rec.p);
        if (depth < rn->p->max_depth && mat_scatter(rec.mat, &r, &rec, &attenuation, &scattered, g)) {
            beta = vmul(beta, attenuation);
            r = scattered;
            continue;
        }
        return vmul(beta, emitted);
    }
}

static inline v3 de_nan(v3 c) {                                         /* main.cpp:232-242 */
    for (int k = 0; k < 3; k++) if (!(c.e[k] == c.e[k])) c.e[k] = 0;
    return c;
}

static v3 render_pixel(run_t *rn, const cam_t *cam, int i, int j, rng_t *g) {
    const oracle_params *p = rn->p;
    int chunk = p->chunk > 0 ? p->chunk : p->ns;
    v3 col = V(0, 0, 0), part = V(0, 0, 0);
    for (int s = 0; s < p->ns; s++) {
        if (g->counter) {
            rng_seed_sample(g, sample_key(p->seed, (uint32_t)(j * p->nx + i), (uint32_t)s + p->sample_offset));
            g->nmedia = rn->sc->nmedia;
        }
        float u = (float)(i + rng_next(g)) / (float)p->nx;                /* main.cpp:305-306 */
        float v = (float)(j + rng_next(g)) / (float)p->ny;
        ray_t r = camera_get_ray(cam, u, v, g);
        v3 temp = p->forward ? color_forward(rn, r, g) : color_right(rn, &r, 0, g);
        temp = de_nan(temp);
        part = vadd(part, temp);
        if ((s + 1) % chunk == 0 || s + 1 == p->ns) { col = vadd(col, part); part = V(0, 0, 0); }
    }
    float k = (float)(1.0 / (double)(float)p->ns);                        /* vec3.h:134-141 */
    return V(col.e[0] * k, col.e[1] * k, col.e[2] * k);
}

int oracle_render(const oracle_params *p, float *out, oracle_stats *stats) {
    scene_t sc;
    if (p->nx <= 0 || p->ny <= 0 || p->ns <= 0) return -1;
    rng_t g_canon;
    if (scene_build(&sc, p->scene, &g_canon) != 0) return -2;
    int x0 = p->x0, y0 = p->y0, w = p->w, h = p->h;
    if (w <= 0) { x0 = 0; y0 = 0; w = p->nx; h = p->ny; }
    if (x0 < 0 || y0 < 0 || x0 + w > p->nx || y0 + h > p->ny) { scene_free(&sc); return -3; }
    cam_t cam = camera_preset(p->camera, p->nx, p->ny);
    struct timespec ta, tb;
    clock_gettime(CLOCK_MONOTONIC, &ta);
    double segments = 0;
    if (p->rng == 0) {
        /* canonical stream: the whole image in reference order (main.cpp:299-304) */
        rng_t g = g_canon;
        run_t rn = { &sc, p, 0 };
        for (int j = p->ny - 1; j >= 0; j--) {
            for (int i = 0; i < p->nx; i++) {
                v3 c = render_pixel(&rn, &cam, i, j, &g);
                int row = p->ny - 1 - j;
                if (row >= y0 && row < y0 + h && i >= x0 && i < x0 + w) {
                    float *o = &out[((size_t)(row - y0) * w + (i - x0)) * 3];
                    o[0] = c.e[0]; o[1] = c.e[1]; o[2] = c.e[2];
                }
            }
        }
        segments = rn.segments;
    } else {
        int nt = p->threads > 0 ? p->threads : 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt) reduction(+ : segments)
        for (int row = y0; row < y0 + h; row++) {
            rng_t g; memset(&g, 0, sizeof g); g.counter = 1;
            run_t rn = { &sc, p, 0 };
            int j = p->ny - 1 - row;
            for (int i = x0; i < x0 + w; i++) {
                v3 c = render_pixel(&rn, &cam, i, j, &g);
                float *o = &out[((size_t)(row - y0) * w + (i - x0)) * 3];
                o[0] = c.e[0]; o[1] = c.e[1]; o[2] = c.e[2];
            }
            segments += rn.segments;
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &tb);
    if (stats) {
        stats->samples = (double)w * h * p->ns;
        if (p->rng == 0) stats->samples = (double)p->nx * p->ny * p->ns;
        stats->segments = segments;
        stats->seconds = (tb.tv_sec - ta.tv_sec) + 1e-9 * (tb.tv_nsec - ta.tv_nsec);
    }
    scene_free(&sc);
    return 0;
}

void oracle_quantize(const float *mean, int n, uint8_t *rgb) {          /* main.cpp:316-325 */
    for (int q = 0; q < n; q++) {
        for (int k = 0; k < 3; k++) {
            float c = sqrtf(mean[3 * q + k]);
            int iv = (int)(255.99 * c);
            rgb[3 * q + k] = (uint8_t)(iv > 255 ? 255 : iv);
        }
    }
}

long oracle_ppm_text(const uint8_t *rgb, int nx, int ny, char *buf, long cap) {   /* main.cpp:297,327-330 */
    long n = 0;
    char line[64];
    int m = snprintf(line, sizeof line, "P3\n%d %d\n255\n", nx, ny);
    if (n + m <= cap && buf) memcpy(buf + n, line, (size_t)m);
    n += m;
    for (long q = 0; q < (long)nx * ny; q++) {
        m = snprintf(line, sizeof line, "%d %d %d\n", rgb[3 * q], rgb[3 * q + 1], rgb[3 * q + 2]);
        if (n + m <= cap && buf) memcpy(buf + n, line, (size_t)m);
        n += m;
    }
    return n;
}

void oracle_perlin_tables(float *ranvec, int32_t *perm) {
    rng_t g; memset(&g, 0, sizeof g);
    perlin_generate(&g);
    for (int i = 0; i < 256; i++) for (int k = 0; k < 3; k++) ranvec[3 * i + k] = g_ranvec[i].e[k];
    for (int a = 0; a < 3; a++) for (int i = 0; i < 256; i++) perm[256 * a + i] = g_perm[a][i];
}

void oracle_drand48(uint64_t x0, int n, double *out) {
    rng_t g; memset(&g, 0, sizeof g); g.x = x0 & LCG_M;
    for (int i = 0; i < n; i++) out[i] = rng_next(&g);
}

void oracle_counter_draws(uint64_t seed, uint32_t pixel, uint32_t sample, int n, double *out) {
    rng_t g; memset(&g, 0, sizeof g); g.counter = 1; rng_seed_sample(&g, sample_key(seed, pixel, sample));
    for (int i = 0; i < n; i++) out[i] = rng_next(&g);
}

double oracle_medium_draw(uint64_t seed, uint32_t pixel, uint32_t sample, int bounce, int medium, int nmedia) {
    rng_t g; memset(&g, 0, sizeof g); g.counter = 1; rng_seed_sample(&g, sample_key(seed, pixel, sample));
    g.nmedia = nmedia;
    return rng_medium(&g, bounce, medium);
}

/* ------------------------------------------------------------ scene dump */
typedef struct { char *buf; long cap, n; const void *ids[4096]; int nids; } dump_t;
static void dputs(dump_t *d, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void dputs(dump_t *d, const char *fmt, ...) {
    char tmp[512];
    va_list ap; va_start(ap, fmt);
    int m = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    if (d->buf && d->n + m <= d->cap) memcpy(d->buf + d->n, tmp, (size_t)m);
    d->n += m;
}
static int dump_id(dump_t *d, const void *p) {
    for (int i = 0; i < d->nids; i++) if (d->ids[i] == p) return i;
    d->ids[d->nids] = p;
    return d->nids++;
}
static void dump_tex(dump_t *d, const tex_t *t) {
    if (t->kind == TX_CONST) { dputs(d, "(const %a %a %a)", t->color.e[0], t->color.e[1], t->color.e[2]); return; }
    if (t->kind == TX_CHECKER) { dputs(d, "(checker even="); dump_tex(d, t->even); dputs(d, " odd="); dump_tex(d, t->odd); dputs(d, ")"); return; }
    if (t->kind == TX_NOISE) { dputs(d, "(noise %a)", t->scale); return; }
    uint32_t h = 2166136261u;   /* FNV-1a over the addressable texels */
    for (long b = 0; b < 3L * t->nx * t->ny; b++) h = (h ^ t->data[b]) * 16777619u;
    dputs(d, "(image %d %d %08x)", t->nx, t->ny, h);
}
static void dump_mat(dump_t *d, const mat_t *m) {
    dputs(d, " mat%d=", dump_id(d, m));
    switch (m->kind) {
    case MT_LAMBERT: dputs(d, "lambertian"); dump_tex(d, m->tex); break;
    case MT_METAL: dputs(d, "metal(%a %a %a fuzz %a)", m->albedo.e[0], m->albedo.e[1], m->albedo.e[2], m->fuzz); break;
    case MT_DIELECTRIC: dputs(d, "dielectric(%a)", m->ri); break;
    case MT_LIGHT: dputs(d, "light"); dump_tex(d, m->tex); break;
    case MT_ISOTROPIC: dputs(d, "isotropic"); dump_tex(d, m->tex); break;
    }
}
static void dump_node(dump_t *d, const obj_t *o, const char *wrap) {
    char w2[1024];
    switch (o->kind) {
    case OB_LIST: for (int i = 0; i < o->nkids; i++) dump_node(d, o->kids[i], wrap); return;
    case OB_BOX: dump_node(d, o->child, wrap); return;
    case OB_FLIP: snprintf(w2, sizeof w2, "%sflip ", wrap); dump_node(d, o->child, w2); return;
    case OB_TRANSLATE: snprintf(w2, sizeof w2, "%stranslate(%a %a %a) ", wrap, o->offset.e[0], o->offset.e[1], o->offset.e[2]); dump_node(d, o->child, w2); return;
    case OB_ROTY: snprintf(w2, sizeof w2, "%srotate_y(sin %a cos %a) ", wrap, o->sin_t, o->cos_t); dump_node(d, o->child, w2); return;
    case OB_MEDIUM:
        dputs(d, "%smedium density %a", wrap, o->density); dump_mat(d, o->mat);
        dputs(d, " boundary{\n"); dump_node(d, o->child, "  "); dputs(d, "}\n"); return;
    case OB_SPHERE: dputs(d, "%ssphere %a %a %a r %a", wrap, o->c0.e[0], o->c0.e[1], o->c0.e[2], o->r); dump_mat(d, o->mat); dputs(d, "\n"); return;
    case OB_MSPHERE:
        dputs(d, "%smoving_sphere %a %a %a -> %a %a %a t %a %a r %a", wrap, o->c0.e[0], o->c0.e[1], o->c0.e[2],
              o->c1.e[0], o->c1.e[1], o->c1.e[2], o->t0, o->t1, o->r);
        dump_mat(d, o->mat); dputs(d, "\n"); return;
    case OB_XY: dputs(d, "%sxy_rect %a %a %a %a k %a", wrap, o->a0, o->a1, o->b0, o->b1, o->k); dump_mat(d, o->mat); dputs(d, "\n"); return;
    case OB_XZ: dputs(d, "%sxz_rect %a %a %a %a k %a", wrap, o->a0, o->a1, o->b0, o->b1, o->k); dump_mat(d, o->mat); dputs(d, "\n"); return;
    case OB_YZ: dputs(d, "%syz_rect %a %a %a %a k %a", wrap, o->a0, o->a1, o->b0, o->b1, o->k); dump_mat(d, o->mat); dputs(d, "\n"); return;
    }
}

long oracle_scene_dump(int which, char *buf, long cap) {
    scene_t sc;
    if (scene_build(&sc, which, NULL) != 0) return -1;
    dump_t *d = calloc(1, sizeof *d);
    d->buf = buf; d->cap = cap;
    dump_node(d, sc.world, "");
    long n = d->n;
    free(d);
    scene_free(&sc);
    return n;
}
