// dist.cpp — the multi-GPU half of the C ABI (include/rt_hip.h, "multi-GPU"):
// one process per GPU, RCCL communicator (ncclCommInitRank), the rank shares (by default
// 8 x 8 pixel blocks dealt along a Hilbert curve; the pixel interleave and a block
// lattice on request: rt_rank_tiles), and ONE
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
    int layout = RT_LAYOUT_BLOCKS;   // how rt_dist_render splits the pixels (rt_dist_set_layout)
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

// Position of cell (x, y) on the Hilbert curve over an n x n grid (n a power of 2); the
// quadrant rotation reflects within the current sub-square (s - 1 - x), as rtnw.py's
// restatement in tests/test_layouts.py does, so both deal the same blocks.
static int64_t hilbert_index(int64_t n, int64_t x, int64_t y) {
    int64_t d = 0;
    for (int64_t s = n / 2; s > 0; s /= 2) {
        const int64_t rx = (x & s) > 0, ry = (y & s) > 0;
        d += s * s * ((3 * rx) ^ ry);
        if (!ry) {
            if (rx) {
                x = s - 1 - x;
                y = s - 1 - y;
            }
            std::swap(x, y);
        }
    }
    return d;
}

// One block's pixels as 1x1 tiles, column by column (any 64 consecutive items of a full
// 8 x 8 block are that block: one wave's claim, the 1-GPU render's coherence)
static void emit_block(int nx, int ny, int x0, int y0, int block, int32_t *tiles, int64_t &k) {
    for (int x = x0; x < std::min(x0 + block, nx); ++x)
        for (int y = y0; y < std::min(y0 + block, ny); ++y) {
            if (tiles) {
                tiles[4 * k + 0] = x;
                tiles[4 * k + 1] = y;
                tiles[4 * k + 2] = 1;
                tiles[4 * k + 3] = 1;
            }
            ++k;
        }
}

int64_t rt_rank_tiles(int nx, int ny, int rank, int world, int layout, int block, int32_t *tiles, int64_t cap) {
    if (nx <= 0 || ny <= 0 || world < 1 || rank < 0 || rank >= world || nx > 65535 || ny > 65535)
        return fail(RT_ERR_INVALID, "rt_rank_tiles: bad argument");
    if (layout == RT_LAYOUT_INTERLEAVED) return rt_rank_pixels(nx, ny, rank, world, tiles, cap);
    if (layout != RT_LAYOUT_BLOCKS && layout != RT_LAYOUT_LATTICE) return fail(RT_ERR_INVALID, "rt_rank_tiles: unknown layout");
    if (block <= 0) block = RT_LAYOUT_BLOCK;
    const int bx = (nx + block - 1) / block, by = (ny + block - 1) / block;
    // this rank's blocks, in claim order
    std::vector<int64_t> mine;
    if (layout == RT_LAYOUT_BLOCKS) {
        // every block's Hilbert position; block k of the curve goes to rank k mod world
        int64_t n = 1;
        while (n < std::max(bx, by)) n *= 2;
        std::vector<std::pair<int64_t, int64_t>> order((size_t)bx * by);
        for (int yb = 0; yb < by; ++yb)
            for (int xb = 0; xb < bx; ++xb) order[(size_t)yb * bx + xb] = {hilbert_index(n, xb, yb), (int64_t)yb * bx + xb};
        std::sort(order.begin(), order.end());   // positions are distinct: the order is the curve's
        for (size_t k = (size_t)rank; k < order.size(); k += (size_t)world) mine.push_back(order[k].second);
    } else {
        // the a x b interleave lattice at block granularity, row-major block order
        int a = 1, b = 1;
        rt_interleave_factors(world, &a, &b);
        const int ry = rank / a, rx = rank % a;
        for (int yb = ry; yb < by; yb += b)
            for (int xb = rx; xb < bx; xb += a) mine.push_back((int64_t)yb * bx + xb);
    }
    int64_t n = 0;
    for (const int64_t c : mine) emit_block(nx, ny, (int)(c % bx) * block, (int)(c / bx) * block, block, nullptr, n);
    if (!tiles) return n;
    if (cap < n) return fail(RT_ERR_INVALID, "rt_rank_tiles: buffer too small");
    int64_t k = 0;
    for (const int64_t c : mine) emit_block(nx, ny, (int)(c % bx) * block, (int)(c / bx) * block, block, tiles, k);
    return n;
}

int rt_dist_set_layout(rt_dist *d, int layout) {
    if (!d || (layout != RT_LAYOUT_BLOCKS && layout != RT_LAYOUT_INTERLEAVED && layout != RT_LAYOUT_LATTICE))
        return fail(RT_ERR_INVALID, "rt_dist_set_layout: bad argument");
    d->layout = layout;
    return RT_OK;
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
        const int64_t n = rt_rank_tiles(p->nx, p->ny, r, d->world, d->layout, RT_LAYOUT_BLOCK, nullptr, 0);
        if (n < 0) return (int)n;
        nmax = std::max(nmax, n);
    }
    std::vector<int32_t> mine((size_t)rt_rank_tiles(p->nx, p->ny, d->rank, d->world, d->layout, RT_LAYOUT_BLOCK, nullptr, 0) * 4);
    rt_rank_tiles(p->nx, p->ny, d->rank, d->world, d->layout, RT_LAYOUT_BLOCK, mine.data(), (int64_t)mine.size() / 4);
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
                const int64_t n = rt_rank_tiles(p->nx, p->ny, r, d->world, d->layout, RT_LAYOUT_BLOCK, nullptr, 0);
                std::vector<int32_t> t((size_t)n * 4);
                rt_rank_tiles(p->nx, p->ny, r, d->world, d->layout, RT_LAYOUT_BLOCK, t.data(), n);
                rc = rt_unpack_tiles(host.data() + (size_t)r * count, t.data(), n, p->nx, p->ny, image);
            }
        }
    }
    cleanup();
    return rc;
}

}  // extern "C"
