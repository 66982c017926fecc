/* include/rt_hip.h — C ABI of librt_hip.so, the MI355X path tracer.
 *
 * Boundary being replaced (the reference has no FFI; its hot path is a C++ call
 * pair):
 *   vec3 color(const ray&, hitable *world, int depth)      main.cpp:25-46
 *   the per-pixel sample loop of main()                     main.cpp:299-332
 *   hitable::hit / material::scatter / texture::value       hitable.h:34, material.h:54, texture.h:13
 * The host keeps the reference's hitable/material/texture/camera classes (see
 * peter-shirley-ray-tracing-the-next-week_amd/csrc/host/rtnw.h); a world built
 * with them is flattened into an rt_scene_desc, uploaded once with
 * rt_scene_create, and rendered on the GPU with rt_render_tile / rt_render_tiles.
 *
 * Conventions: plain C types only; every function returns RT_OK (0) or a
 * negative rt_status; rt_last_error() returns a thread-local message.  A scene is
 * bound to one HIP device; calls on one scene are serialised on a stream.  There
 * is no CPU fallback: without a usable GPU every render entry point fails.
 */
#ifndef RT_HIP_H
#define RT_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rt_stats gained the shading-stage divergence fields (wave_shade_passes ...) */
#define RT_ABI_VERSION 2

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,      /* bad argument / malformed descriptor */
    RT_ERR_HIP = -2,          /* HIP runtime failure (no device, launch error, ...) */
    RT_ERR_NOMEM = -3,
    RT_ERR_UNSUPPORTED = -4   /* a scene feature the device path does not implement */
} rt_status;

/* ------------------------------------------------------------ scene descriptor
 * Flattened form of a hitable tree.  Leaves are listed in depth-first list order
 * (the order hitable_list::hit visits them, hitable_list.h:24); that order is the
 * tie-break order of the closest-hit search.                                   */
enum rt_prim_kind {
    RT_PRIM_SPHERE = 0,          /* sphere.h:10-52:  p = {cx, cy, cz, r}                      */
    RT_PRIM_MOVING_SPHERE = 1,   /* sphere.h:61-118: p = {c0x,c0y,c0z, c1x,c1y,c1z, t0, t1, r} */
    RT_PRIM_XY_RECT = 2,         /* aarect.h:11-65:  p = {x0, x1, y0, y1, k}                  */
    RT_PRIM_XZ_RECT = 3,         /* aarect.h:23-83:  p = {x0, x1, z0, z1, k}                  */
    RT_PRIM_YZ_RECT = 4          /* aarect.h:35-100: p = {y0, y1, z0, z1, k}                  */
};

typedef struct rt_prim {
    int32_t kind;        /* rt_prim_kind */
    int32_t material;    /* index into rt_scene_desc.materials */
    int32_t instance;    /* -1, or index into rt_scene_desc.instances (transform chain) */
    int32_t flip;        /* 1: a flip_normals wraps the primitive directly (hitable.h:39-54) */
    float p[12];
} rt_prim;               /* 64 bytes */

enum rt_xform_op {
    RT_OP_TRANSLATE = 1, /* hitable.h:57-83:  {ox, oy, oz}            */
    RT_OP_ROTATE_Y = 2,  /* hitable.h:85-150: {sin_theta, cos_theta}  */
    RT_OP_FLIP = 3       /* hitable.h:39-54 between two transforms    */
};

typedef struct rt_instance {
    int32_t nops;        /* <= 6; ops[0] is the outermost wrapper */
    int32_t pad[3];
    float ops[6][4];     /* {op, a, b, c} */
} rt_instance;

enum rt_material_kind {
    RT_MAT_LAMBERTIAN = 0,    /* material.h:61-72   texture        */
    RT_MAT_METAL = 1,         /* material.h:74-85   albedo, fuzz   */
    RT_MAT_DIELECTRIC = 2,    /* material.h:87-123  ref_idx        */
    RT_MAT_DIFFUSE_LIGHT = 3, /* material.h:126-139 texture        */
    RT_MAT_ISOTROPIC = 4      /* material.h:142-151 texture        */
};

typedef struct rt_material {
    int32_t kind;
    int32_t texture;     /* -1 when unused */
    float fuzz;          /* already clamped to <= 1 (material.h:76) */
    float ref_idx;
    float albedo[3];
    int32_t pad;
} rt_material;           /* 32 bytes */

enum rt_texture_kind {
    RT_TEX_CONSTANT = 0, /* texture.h:16-27 color                    */
    RT_TEX_CHECKER = 1,  /* texture.h:30-45 even, odd (texture idx)  */
    RT_TEX_NOISE = 2,    /* texture.h:48-59 scale                    */
    RT_TEX_IMAGE = 3     /* surface_texture.h:10-30 image (index into images)      */
};

typedef struct rt_texture {
    int32_t kind;
    int32_t even, odd;   /* checker children */
    float scale;         /* noise */
    float color[3];      /* constant */
    int32_t image;       /* image: index into rt_scene_desc.images */
} rt_texture;            /* 32 bytes */

typedef struct rt_image {    /* texels of one image_texture (surface_texture.h:13) */
    int64_t offset;          /* byte offset into rt_scene_desc.image_data */
    int32_t nx, ny;          /* image size; texel (i, j) channel c is at 3*i + 3*nx*j + c
                                (surface_texture.h:26-28 addresses with stride 3 whatever
                                the file's channel count) */
} rt_image;

typedef struct rt_medium {   /* constant_medium.h:14-50 */
    int32_t boundary_first;  /* range in rt_scene_desc.boundary_prims */
    int32_t boundary_count;
    float density;
    int32_t material;        /* the isotropic phase material */
    int32_t order;           /* number of surface prims before it in list order */
    int32_t pad[3];
} rt_medium;

typedef struct rt_scene_desc {
    uint32_t abi_version;         /* RT_ABI_VERSION */
    int32_t nprims, nboundary, nmedia, nmaterials, ntextures, ninstances;
    const rt_prim *prims;         /* surfaces, depth-first list order */
    const rt_prim *boundary_prims;/* leaves of media boundaries */
    const rt_medium *media;       /* in list order (= keyed-draw ordinal) */
    const rt_material *materials;
    const rt_texture *textures;
    const rt_instance *instances;
    const float *perlin_ranvec;   /* 256 x 3, perlin.h:82-87 */
    const int32_t *perlin_perm;   /* 3 x 256, perlin.h:99-111 */
    float time0, time1;           /* shutter span rays may carry (moving-sphere bounds) */
    int32_t nimages;
    const rt_image *images;
    const uint8_t *image_data;    /* texel bytes of all images */
    int64_t image_bytes;
} rt_scene_desc;

/* ------------------------------------------------------------------ camera */
typedef struct rt_camera_desc {   /* the state camera.h:21-39 computes */
    float origin[3], lower_left_corner[3], horizontal[3], vertical[3], u[3], v[3], w[3];
    float lens_radius, time0, time1;
} rt_camera_desc;

/* Same arithmetic as camera::camera (camera.h:21-39). */
int rt_camera_init(rt_camera_desc *out, const float lookfrom[3], const float lookat[3], const float vup[3],
                   float vfov, float aspect, float aperture, float focus_dist, float t0, float t1);

/* ------------------------------------------------------------------ render */
enum { RT_BG_BLACK = 0, RT_BG_SKY = 1 };
enum {
    RT_FLAG_COUNT = 1,            /* counting variant: fills the rt_stats visit counters */
    RT_FLAG_PROFILE = 2,          /* stamp variant: fills cycles_* (diagnostic; never timed) */
    /* Progressive rendering / checkpoint-resume: the output holds per-pixel
     * SUMS instead of means.  SUM_IN: on entry the output already holds the sums of
     * samples [0, sample_offset) (e.g. read back from rt_checkpoint_read); this call
     * adds samples [sample_offset, sample_offset + spp) to them one at a time, in
     * sample order, so a resumed render is bitwise the uninterrupted one.  SUM_OUT:
     * write the sums (to checkpoint or resume later); without it the output is the
     * mean, col * float(1.0 / ns) with ns = sample_offset + spp under SUM_IN, else spp. */
    RT_FLAG_SUM_IN = 4,
    RT_FLAG_SUM_OUT = 8
};

typedef struct rt_render_params {
    int32_t nx, ny;               /* full image (u,v normalisation and pixel keys) */
    int32_t spp;                  /* samples per pixel (main.cpp:251 ns) */
    int32_t max_depth;            /* scatter while depth < max_depth (main.cpp:34: 50) */
    float t_min;                  /* main.cpp:27: 0.001 */
    int32_t background;           /* RT_BG_* */
    int32_t chunk;                /* samples per work item (partial sum); <= 0 selects 1, the
                                     reference's one-add-per-sample order (main.cpp:311).  A job
                                     whose partial-sum slab (16 B x pixels x ceil(spp/chunk))
                                     would pass the slab budget (8 GiB, env RTNW_SLAB_BUDGET) runs
                                     as several launches over sample batches, each batch added
                                     to a per-pixel running sum in sample order: the image does
                                     not depend on the job's size or split (any rank count) */
    int32_t flags;                /* RT_FLAG_* */
    uint32_t sample_offset;       /* first sample index (progressive rendering) */
    uint32_t pad;
    uint64_t seed;                /* counter-RNG key */
} rt_render_params;

typedef struct rt_stats {
    double samples;               /* camera samples rendered */
    double segments;              /* rays traced = world hit calls (RT_FLAG_COUNT) */
    double node_visits;           /* BVH2 nodes fetched, each holding both child boxes (RT_FLAG_COUNT) */
    double sphere_tests;          /* sphere tests, BVH leaves + media boundaries (RT_FLAG_COUNT) */
    double moving_sphere_tests;   /* (RT_FLAG_COUNT) */
    double rect_tests;            /* xy/xz/yz rect tests (RT_FLAG_COUNT) */
    double instanced_tests;       /* tests through a translate/rotate_y chain (RT_FLAG_COUNT) */
    double medium_tests;          /* constant_medium evaluations (RT_FLAG_COUNT) */
    double shades;                /* material evaluations (RT_FLAG_COUNT) */
    double noise_evals;           /* Perlin turbulence evaluations (RT_FLAG_COUNT) */
    double algorithmic_bytes;     /* SURVEY §8d byte model for the launch (RT_FLAG_COUNT) */
    double kernel_ms;             /* megakernel time from HIP events on the render stream */
    double resolve_ms;            /* partial-sum resolve kernel time */
    double cycles_claim;          /* RT_FLAG_PROFILE: wave cycles in work claim + camera sampling */
    double cycles_traverse;       /*   ... in the BVH / primitive search */
    double cycles_media;          /*   ... in constant_medium evaluation + hit record */
    double cycles_shade;          /*   ... in material / texture evaluation */
    double grid;                  /* workgroups launched (persistent grid) */
    double wave_iterations;       /* RT_FLAG_COUNT: megakernel loop iterations, summed over waves */
    double wave_node_trips;       /*   wave-level BVH node steps (SIMD efficiency = node_visits / 64x this) */
    double wave_prim_trips;       /*   wave-level primitive-test steps */
    double wave_sphere_draw_trips;/*   wave-level random_in_unit_sphere rejection rounds */
    double lane_sphere_draw_trips;/*   lane-level rejection rounds */
    double chunk;                 /* samples per work item the launch used (rt_render_params.chunk or its default) */
    double batches;               /* megakernel launches (sample batches) the job took */
    double lds_level;             /* scene data in LDS: 0 none (HBM, L1/L2), 1 the BVH2 nodes */
    double stack_depth;           /* traversal stack entries per lane (LDS variants: the BVH depth + 1) */
    double scan_groups;           /* flat scan instead of a BVH (<= 64 primitives): its instance groups, else 0 */
    double prescan;               /* BVH scenes: largest primitives kept out of the BVH, tested first in lockstep */
    double wave_exhaust_first_us; /* RT_FLAG_PROFILE wave timeline of the job's last launch (s_memrealtime, us
                                     after its first wave started):
                                     the first wave to find the work pool empty */
    double wave_exhaust_last_us;  /*   the last wave to find it empty */
    double wave_end_first_us;     /*   the first wave to finish */
    double wave_end_mean_us;      /*   mean wave finish */
    double wave_end_last_us;      /*   the last wave to finish (the launch's end) */
    double wave_shade_passes;     /* RT_FLAG_COUNT: wave-level passes through the material scatter branches */
    double wave_shade_kinds;      /*   distinct scatter materials (lambertian/metal/dielectric/isotropic) summed
                                         over those passes: the branches each pass ran */
    double lane_scatters;         /*   lanes that scattered (SIMD efficiency = this / 64x wave_shade_passes) */
    double cycles_scatter;        /* RT_FLAG_PROFILE: wave cycles in the material scatter branches (part of
                                         cycles_shade) */
} rt_stats;

typedef struct rt_scene rt_scene; /* opaque; owns device copies */

/* Copies the descriptor into device memory (HBM) of `device` and builds the BVH.
 * The caller keeps ownership of d. */
int rt_scene_create(const rt_scene_desc *d, int device, rt_scene **out);
void rt_scene_destroy(rt_scene *s);

/* Renders the w x h rectangle at (x0, y0) (image coords, row 0 = top row of the
 * PPM, i.e. main.cpp's j = ny-1) into out_rgb (host memory, h*w*3 floats, linear
 * mean radiance = main.cpp's `col` after `col /= float(ns)`).  Synchronous. */
int rt_render_tile(rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p,
                   int x0, int y0, int w, int h, float *out_rgb, rt_stats *stats);

/* Renders ntiles rectangles (tiles[4k..4k+3] = x0, y0, w, h) into device memory:
 * out_dev receives the tiles packed back to back (tile k at offset sum_{i<k} w_i*h_i*3
 * floats, each row-major).  Enqueued on `stream` (a hipStream_t; NULL = default
 * stream).  When stats is non-NULL the call waits for completion to read the
 * HIP-event timings.  ntiles == 0 is a no-op (a rank without tiles). */
int rt_render_tiles(rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p,
                    const int32_t *tiles, int ntiles, float *out_dev, void *stream, rt_stats *stats);

/* Device buffer helpers, so callers without a HIP toolchain can drive the ABI. */
int rt_device_alloc(int device, uint64_t bytes, void **out);
int rt_device_free(void *ptr);
int rt_copy_to_host(void *dst, const void *src_dev, uint64_t bytes);
int rt_device_count(int *out);

/* Diagnostic: the device's float transcendentals of the path on n host inputs (out: n
 * floats) — fn 0 the megakernel's sinf (texture.h:36, 55), 2 its asinf and 4 its
 * atan2f(a, b) (hitable.h:15-16), all restated from glibc (rt_libm.h); 1, 3, 5 ocml's
 * sinf / asinf / atan2f for comparison.  For the parity tests; not on the render path. */
int rt_math_probe(int fn, const float *a, const float *b, float *out, int64_t n);

/* ------------------------------------------------ multi-GPU
 * One process per GPU.  The root calls rt_dist_unique_id and hands the 128 bytes to
 * every rank (any side channel); each rank calls rt_dist_init (ncclCommInitRank),
 * renders its share of the pixels — by default 8 x 8 pixel blocks dealt along a
 * Hilbert curve (rt_rank_tiles, RT_LAYOUT_BLOCKS), or the interleave of rt_rank_pixels:
 * with world = a x b, rank (ry, rx) renders x = rx (mod a), y = ry (mod b), a
 * sub-sampled copy of the whole view — and ONE ncclGather (rccl.h:745) brings the packed shares
 * to the root, which unpacks them.  The RNG is keyed by (pixel, sample), so the
 * image is bitwise the 1-GPU image for any rank count.                           */
#define RT_DIST_ID_BYTES 128
typedef struct rt_dist rt_dist;   /* one rank's RCCL communicator */
int rt_dist_unique_id(uint8_t id[RT_DIST_ID_BYTES]);             /* ncclGetUniqueId (root only) */
int rt_dist_init(const uint8_t id[RT_DIST_ID_BYTES], int rank, int world, int device, rt_dist **out);
void rt_dist_destroy(rt_dist *d);
/* ncclGather of `count` floats from every rank's send_dev into recv_dev on `root`
 * (world x count floats, rank-major); enqueued on `stream` (hipStream_t, NULL = default). */
int rt_dist_gather(rt_dist *d, const float *send_dev, uint64_t count, float *recv_dev, int root, void *stream);
/* world = a x b, a >= b, as square as possible (8 -> 4 x 2). */
void rt_interleave_factors(int world, int *a, int *b);
/* The pixels of `rank` as 1x1 tiles (4 int32 each) in claim order: bands of 8 rows of
 * the rank's lattice, column by column.  Returns the count (tiles == NULL: count only). */
int64_t rt_rank_pixels(int nx, int ny, int rank, int world, int32_t *tiles, int64_t cap);
/* How a job's pixels are split over the ranks (rt_rank_tiles, rt_dist_set_layout):
 *   RT_LAYOUT_BLOCKS       the image's block x block pixel blocks in Hilbert-curve order,
 *                          block k of the curve to rank k mod world (the default of
 *                          rt_dist_render and bench.py: every rank's blocks spread over
 *                          the view, and a wave's 64 work items stay one 8 x 8 block);
 *   RT_LAYOUT_INTERLEAVED  rt_rank_pixels' pixel interleave;
 *   RT_LAYOUT_LATTICE      the blocks on the interleave's a x b lattice, row-major.
 * The pixels come as 1x1 tiles in claim order (each block column by column).  Returns the
 * count (tiles == NULL: count only), RT_ERR_INVALID for a bad argument or a short buffer;
 * block <= 0 means RT_LAYOUT_BLOCK.  Replaces main.cpp:299-300's one pixel loop per job. */
#define RT_LAYOUT_BLOCKS 0
#define RT_LAYOUT_INTERLEAVED 1
#define RT_LAYOUT_LATTICE 2
#define RT_LAYOUT_BLOCK 8
int64_t rt_rank_tiles(int nx, int ny, int rank, int world, int layout, int block, int32_t *tiles, int64_t cap);
/* Scatters packed tiles (rt_render_tiles' output layout) into an nx x ny x 3 image. */
int rt_unpack_tiles(const float *packed, const int32_t *tiles, int64_t ntiles, int nx, int ny, float *image);
/* The whole rank job: this rank's pixels -> rt_render_tiles -> rt_dist_gather -> on the
 * root, the full nx x ny x 3 mean image in host memory (`image`; NULL on other ranks).
 * Mean images only: RT_FLAG_SUM_IN / RT_FLAG_SUM_OUT return RT_ERR_INVALID (on every
 * rank alike).  A rank whose render fails still joins the gather; one that cannot
 * allocate its buffers aborts the communicator (ncclCommAbort, later calls on it fail)
 * and its launcher must stop the peers waiting in the gather. */
int rt_dist_render(rt_dist *d, rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p, float *image,
                   rt_stats *stats);
/* The split rt_dist_render uses (RT_LAYOUT_*; RT_LAYOUT_BLOCKS unless set).  Every rank of
 * a job must set the same layout.  The gathered image is the same for every layout. */
int rt_dist_set_layout(rt_dist *d, int layout);

/* ----------------------------------------------------- resolve (main.cpp:314-330) */
/* sqrt gamma + int(255.99*c) + clamp to 255, per channel (main.cpp:316-325). */
void rt_quantize(const float *mean_rgb, int64_t n_pixels, uint8_t *rgb);
/* P3 text of main.cpp:297,327-330; returns the byte count (writes when buf != NULL and cap suffices). */
int64_t rt_ppm_text(const uint8_t *rgb, int nx, int ny, char *buf, int64_t cap);

/* ------------------------------------------- checkpoint / resume
 * A progressive render keeps per-pixel SUMS (RT_FLAG_SUM_OUT) and resumes from them
 * (RT_FLAG_SUM_IN with sample_offset = samples_done): bitwise the same image as an
 * uninterrupted render.  The file holds this header, `count` floats in the packed
 * tile layout of rt_render_tiles, and a checksum; it is replaced atomically.       */
#define RT_CHECKPOINT_MAGIC 0x4B435452u   /* "RTCK" */
#define RT_CHECKPOINT_VERSION 1u
typedef struct rt_checkpoint {
    uint32_t magic, version;      /* set by rt_checkpoint_write */
    int32_t nx, ny;               /* full image */
    uint32_t samples_done;        /* the sums hold samples [0, samples_done) of every pixel */
    int32_t max_depth, background;
    float t_min;
    uint64_t seed;                /* counter-RNG key of the render */
    uint64_t job_hash;            /* caller's identification of the scene / tiles */
    uint64_t count;               /* floats that follow (3 per pixel) */
} rt_checkpoint;
int rt_checkpoint_write(const char *path, const rt_checkpoint *hdr, const float *sums);
/* sums == NULL reads the header only; otherwise cap = capacity of sums in floats. */
int rt_checkpoint_read(const char *path, rt_checkpoint *hdr, float *sums, uint64_t cap);

/* ------------------------------------------------ host scene construction */
/* Builds one of the reference's scenes with the host API (random_scene, random_motion,
 * cornell_box, cornell_smoke, final, simple_light, two_spheres, test) exactly as a
 * fresh reference process would (drand48 state 0, Perlin static init first) and
 * returns its flattened descriptor (free with rt_scene_desc_free). */
int rt_builtin_scene_desc(const char *name, rt_scene_desc **out);
void rt_scene_desc_free(rt_scene_desc *d);
/* Leaf dump in the text format of oracle/ref_harness.cpp --dump (for parity tests). */
int64_t rt_scene_desc_dump(const rt_scene_desc *d, char *buf, int64_t cap);

const char *rt_last_error(void);
const char *rt_version(void);

#ifdef __cplusplus
}
#endif
#endif
