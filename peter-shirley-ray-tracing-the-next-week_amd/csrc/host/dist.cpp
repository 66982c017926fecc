// dist.cpp — the multi-GPU half of the C ABI (include/rt_hip.h, "multi-GPU"):
// one process per GPU, RCCL communicator (ncclCommInitRank), the pixel interleave
// that gives every rank a sub-sampled copy of the view, and ONE
// ncclGather (rccl.h:745) of the packed per-rank framebuffers to the root over xGMI.
// Replaces the reference's single-process pixel loop (main.cpp:299-332) for
// config 5 (final() 1000x1000x1000 over 8 GPUs); the RNG is keyed by (pixel,
// sample), so the gathered image is bitwise the 1-GPU image.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "rt_hip.h"

// error plumbing shared with capi.cpp (thread-local message)
int rt_internal_fail(int code, const std::string &msg);

namespace {
int fail(int code, const std::string &msg) { return rt_internal_fail(code, msg); }
int nccl_fail(ncclResult_t r, const char *what) {
    return fail(RT_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCL_TRY(expr)                                     \
    do {                                                   \
        ncclResult_t r_ = (expr);                          \
        if (r_ != ncclSuccess) return nccl_fail(r_, #expr); \
    } while (0)
#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
static_assert(sizeof(ncclUniqueId) == RT_DIST_ID_BYTES, "ncclUniqueId size");
}  // namespace

struct rt_dist {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
    bool aborted = false;   // ncclCommAbort after a local failure (rt_dist_render)
};

extern "C" {

int rt_dist_unique_id(uint8_t *id) {
    if (!id) return fail(RT_ERR_INVALID, "rt_dist_unique_id: null id");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, RT_DIST_ID_BYTES);
    return RT_OK;
}

int rt_dist_init(const uint8_t *id, int rank, int world, int device, rt_dist **out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return fail(RT_ERR_INVALID, "rt_dist_init: bad argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, RT_DIST_ID_BYTES);
    auto *d = new rt_dist();
    d->rank = rank;
    d->world = world;
    d->device = device;
    const ncclResult_t r = ncclCommInitRank(&d->comm, world, u, rank);
    if (r != ncclSuccess) {
        delete d;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = d;
    return RT_OK;
}

void rt_dist_destroy(rt_dist *d) {
    if (!d) return;
    if (d->comm && !d->aborted) (void)ncclCommDestroy(d->comm);
    delete d;
}

int rt_dist_gather(rt_dist *d, const float *send_dev, uint64_t count, float *recv_dev, int root, void *stream) {
    if (!d || !send_dev || root < 0 || root >= d->world || (d->rank == root && !recv_dev))
        return fail(RT_ERR_INVALID, "rt_dist_gather: bad argument");
    if (d->aborted) return fail(RT_ERR_HIP, "rt_dist_gather: the communicator was aborted after an earlier failure");
    HIP_TRY(hipSetDevice(d->device));
    NCCL_TRY(ncclGather(send_dev, recv_dev, (size_t)count, ncclFloat32, root, d->comm, (hipStream_t)stream));
    return RT_OK;
}

// world = a x b, a >= b, as close to square as possible (8 -> 4 x 2)
void rt_interleave_factors(int world, int *a, int *b) {
    int q = (int)std::sqrt((double)world);
    while (q > 1 && q * q > world) --q;
    while ((q + 1) * (q + 1) <= world) ++q;
    while (q > 1 && world % q) --q;
    if (q < 1) q = 1;
    *b = q;
    *a = world / q;
}

int64_t rt_rank_pixels(int nx, int ny, int rank, int world, int32_t *tiles, int64_t cap) {
    if (nx <= 0 || ny <= 0 || world < 1 || rank < 0 || rank >= world) return fail(RT_ERR_INVALID, "rt_rank_pixels: bad argument");
    int a = 1, b = 1;
    rt_interleave_factors(world, &a, &b);
    const int ry = rank / a, rx = rank % a;
    const int64_t nxs = rx < nx ? (nx - rx + a - 1) / a : 0, nys = ry < ny ? (ny - ry + b - 1) / b : 0;
    const int64_t n = nxs * nys;
    if (!tiles) return n;
    if (cap < n) return fail(RT_ERR_INVALID, "rt_rank_pixels: buffer too small");
    int64_t k = 0;
    for (int64_t band = 0; band < nys; band += 8)          // bands of 8 rows of the rank's lattice,
        for (int64_t i = 0; i < nxs; ++i)                 // column by column: any 64 consecutive
            for (int64_t j = band; j < std::min<int64_t>(band + 8, nys); ++j) {   // pixels = 8 columns
                tiles[4 * k + 0] = (int32_t)(rx + i * a);
                tiles[4 * k + 1] = (int32_t)(ry + j * b);
                tiles[4 * k + 2] = 1;
                tiles[4 * k + 3] = 1;
                ++k;
            }
    return n;
}

int rt_unpack_tiles(const float *packed, const int32_t *tiles, int64_t ntiles, int nx, int ny, float *image) {
    if ((!packed || !tiles || !image) && ntiles) return fail(RT_ERR_INVALID, "rt_unpack_tiles: null argument");
    int64_t off = 0;
    for (int64_t t = 0; t < ntiles; ++t) {
        const int x0 = tiles[4 * t], y0 = tiles[4 * t + 1], w = tiles[4 * t + 2], h = tiles[4 * t + 3];
        if (x0 < 0 || y0 < 0 || w <= 0 || h <= 0 || x0 + w > nx || y0 + h > ny)
            return fail(RT_ERR_INVALID, "rt_unpack_tiles: tile outside the image");
        for (int y = 0; y < h; ++y) {
            std::memcpy(image + 3 * ((int64_t)(y0 + y) * nx + x0), packed + off, sizeof(float) * 3 * (size_t)w);
            off += 3 * (int64_t)w;
        }
    }
    return RT_OK;
}

int rt_dist_render(rt_dist *d, rt_scene *s, const rt_camera_desc *cam, const rt_render_params *p, float *image,
                   rt_stats *stats) {
    // Argument errors below depend only on (nx, ny, world, flags), which every rank of
    // one job passes alike: all ranks return them before the gather, none is left
    // waiting in the collective.
    if (!d || !s || !cam || !p) return fail(RT_ERR_INVALID, "rt_dist_render: bad argument");
    if (d->aborted) return fail(RT_ERR_HIP, "rt_dist_render: the communicator was aborted after an earlier failure");
    // The shares are rendered into freshly zeroed buffers and gathered as means:
    // running sums in (RT_FLAG_SUM_IN) would start from zero but still be scaled by
    // 1/(sample_offset + spp), and sums out (RT_FLAG_SUM_OUT) would reach the root
    // labelled as a mean image.  Progressive multi-GPU renders use rt_render_tiles.
    if (p->flags & (RT_FLAG_SUM_IN | RT_FLAG_SUM_OUT))
        return fail(RT_ERR_INVALID, "rt_dist_render: RT_FLAG_SUM_IN / RT_FLAG_SUM_OUT are not supported (mean images only)");
    if (d->rank == 0 && !image) return fail(RT_ERR_INVALID, "rt_dist_render: the root needs an image buffer");
    // every rank's pixel count, so that the gather's per-rank count (the largest) is agreed
    int64_t nmax = 0;
    for (int r = 0; r < d->world; ++r) {
        const int64_t n = rt_rank_pixels(p->nx, p->ny, r, d->world, nullptr, 0);
        if (n < 0) return (int)n;
        nmax = std::max(nmax, n);
    }
    std::vector<int32_t> mine((size_t)rt_rank_pixels(p->nx, p->ny, d->rank, d->world, nullptr, 0) * 4);
    rt_rank_pixels(p->nx, p->ny, d->rank, d->world, mine.data(), (int64_t)mine.size() / 4);
    const uint64_t count = (uint64_t)nmax * 3;
    float *send = nullptr, *recv = nullptr;
    hipStream_t stream = nullptr;
    int rc = RT_OK;
    auto cleanup = [&]() {
        if (send) (void)hipFree(send);
        if (recv) (void)hipFree(recv);
        if (stream) (void)hipStreamDestroy(stream);
    };
    auto hip_ok = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
        return rc == RT_OK;
    };
    // A local resource failure (device, stream, buffers) cannot join the gather: the
    // communicator is aborted (ncclCommAbort) so that this rank does not leave a
    // half-open collective behind, and the error returned; the peers then block in
    // their gather until the job's launcher stops them (examples/render_dist.cpp and
    // bench.py's launch_ranks stop every rank once one exits with an error).
    if (!hip_ok(hipSetDevice(d->device), "hipSetDevice") ||
        !hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate") ||
        !hip_ok(hipMalloc(&send, count * sizeof(float)), "hipMalloc send") ||
        !hip_ok(hipMemsetAsync(send, 0, count * sizeof(float), stream), "hipMemset") ||
        (d->rank == 0 && !hip_ok(hipMalloc(&recv, count * d->world * sizeof(float)), "hipMalloc recv"))) {
        cleanup();
        (void)ncclCommAbort(d->comm);
        d->aborted = true;
        return rc;
    }
    // A rank whose render fails still joins the gather (with its zeroed buffer), so the
    // other ranks do not wait forever in the collective; its error is returned after.
    int render_rc = RT_OK;
    if (!mine.empty()) render_rc = rt_render_tiles(s, cam, p, mine.data(), (int)(mine.size() / 4), send, stream, stats);
    else if (stats) std::memset(stats, 0, sizeof *stats);
    const std::string render_err = render_rc == RT_OK ? std::string() : std::string(rt_last_error());
    rc = rt_dist_gather(d, send, count, recv, 0, stream);
    if (render_rc != RT_OK) rc = fail(render_rc, render_err);
    if (rc == RT_OK) hip_ok(hipStreamSynchronize(stream), "hipStreamSynchronize");
    if (rc == RT_OK && d->rank == 0) {
        std::vector<float> host(count * d->world);
        if (hip_ok(hipMemcpy(host.data(), recv, host.size() * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy")) {
            for (int r = 0; r < d->world && rc == RT_OK; ++r) {
                const int64_t n = rt_rank_pixels(p->nx, p->ny, r, d->world, nullptr, 0);
                std::vector<int32_t> t((size_t)n * 4);
                rt_rank_pixels(p->nx, p->ny, r, d->world, t.data(), n);
                rc = rt_unpack_tiles(host.data() + (size_t)r * count, t.data(), n, p->nx, p->ny, image);
            }
        }
    }
    cleanup();
    return rc;
}

}  // extern "C"
