// tests/native/host_sanitize.cpp — drives the host side of librt_hip.so (scene
// builders, flattening, every BVH form, the PNG decoder, the C ABI's host-only
// helpers and its error paths) in a build whose host objects carry
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitizers.py; the
// device code object is linked in unsanitised, as the GPU sanitizer is not
// available).  Exit 0 = every call returned as expected and no sanitizer fired.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include <unistd.h>

#include "rt_hip.h"
#include "bvh.h"
#include "rtnw.h"

namespace {

int failures = 0;
#define EXPECT(c)                                                          \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::printf("FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, rt_last_error()); \
            failures++;                                                    \
        }                                                                  \
    } while (0)

void scenes() {
    const char *names[] = {"final", "random_scene", "cornell_box", "cornell_smoke", "random_motion", "simple_light",
                           "two_spheres", "test", "earth", "edge_empty", "edge_single", "edge_degenerate"};
    for (const char *nm : names) {
        rt_scene_desc *d = nullptr;
        EXPECT(rt_builtin_scene_desc(nm, &d) == RT_OK);
        if (!d) continue;
        std::vector<char> buf(1 << 20);
        const int64_t need = rt_scene_desc_dump(d, buf.data(), (int64_t)buf.size());
        EXPECT(need > 0 || d->nprims == 0);
        EXPECT(rt_scene_desc_dump(d, buf.data(), 16) == need);   // truncated: same length, no overrun
        for (const char *w : {"2", "4", "8", "8q"}) {
            setenv("RTNW_BVH_WIDTH", w, 1);
            const rtnw::BvhResult r = rtnw::build_bvh(d->prims, d->nprims, d->instances, d->time0, d->time1);
            EXPECT((int)r.order.size() == d->nprims);
        }
        unsetenv("RTNW_BVH_WIDTH");
        // no GPU in the sanitizer run: the upload must fail cleanly (RT_ERR_HIP), not crash
        rt_scene *s = nullptr;
        const int rc = rt_scene_create(d, 0, &s);
        EXPECT(rc == RT_OK || rc == RT_ERR_HIP);
        if (s) rt_scene_destroy(s);
        rt_scene_desc_free(d);
    }
    rt_scene_desc *d = nullptr;
    EXPECT(rt_builtin_scene_desc("no_such_scene", &d) == RT_ERR_INVALID);
    EXPECT(rt_builtin_scene_desc(nullptr, &d) == RT_ERR_INVALID);
}

void png(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::vector<unsigned char> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    EXPECT(!file.empty());
    int x = 0, y = 0, comp = 0;
    std::string err;
    unsigned char *img = rtnw::png_decode(file.data(), file.size(), &x, &y, &comp, &err);
    EXPECT(img != nullptr && x > 0 && y > 0 && comp >= 3);
    std::free(img);
    // every truncation and single-byte corruptions must fail (or decode) without a fault
    for (size_t n = 0; n < file.size(); n += 1 + n / 8) {
        unsigned char *p = rtnw::png_decode(file.data(), n, &x, &y, &comp, &err);
        std::free(p);
    }
    std::vector<unsigned char> bad = file;
    for (size_t i = 8; i < bad.size(); i += 97) {
        const unsigned char keep = bad[i];
        bad[i] ^= 0x5A;
        unsigned char *p = rtnw::png_decode(bad.data(), bad.size(), &x, &y, &comp, &err);
        std::free(p);
        bad[i] = keep;
    }
}

void abi_helpers() {
    rt_camera_desc cam;
    const float from[3] = {478, 278, -600}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
    EXPECT(rt_camera_init(&cam, from, at, up, 40, 1.0f, 0.0f, 10.0f, 0.0f, 1.0f) == RT_OK);
    const int nx = 37, ny = 23;
    std::vector<float> mean(3 * nx * ny);
    for (size_t i = 0; i < mean.size(); i++) mean[i] = (float)std::fmod(i * 0.37, 1.7) - 0.2f;
    mean[5] = NAN;
    mean[7] = INFINITY;
    std::vector<uint8_t> rgb(3 * nx * ny);
    rt_quantize(mean.data(), nx * ny, rgb.data());
    const int64_t need = rt_ppm_text(rgb.data(), nx, ny, nullptr, 0);
    std::vector<char> text(need + 1);
    EXPECT(rt_ppm_text(rgb.data(), nx, ny, text.data(), (int64_t)text.size()) == need);
    EXPECT(rt_ppm_text(rgb.data(), nx, ny, text.data(), 10) == need);
    // pixel interleave + unpack for every world size up to 8
    for (int world = 1; world <= 8; world++) {
        std::vector<float> image(3 * nx * ny, -1.0f);
        int64_t total = 0;
        for (int r = 0; r < world; r++) {
            const int64_t n = rt_rank_pixels(nx, ny, r, world, nullptr, 0);
            std::vector<int32_t> tiles(4 * n);
            EXPECT(rt_rank_pixels(nx, ny, r, world, tiles.data(), n) == n);
            std::vector<float> packed(3 * n, (float)r);
            EXPECT(rt_unpack_tiles(packed.data(), tiles.data(), n, nx, ny, image.data()) == RT_OK);
            total += n;
        }
        EXPECT(total == (int64_t)nx * ny);
        for (float v : image) EXPECT(v >= 0.0f);
    }
    // checkpoint round trip and the damaged-file paths
    char path[] = "/tmp/rt_sanitize_ckpt_XXXXXX";
    const int fd = mkstemp(path);
    EXPECT(fd >= 0);
    if (fd >= 0) close(fd);
    rt_checkpoint h{};
    h.nx = nx; h.ny = ny; h.samples_done = 7; h.max_depth = 50; h.t_min = 0.001f; h.seed = 99; h.count = mean.size();
    EXPECT(rt_checkpoint_write(path, &h, mean.data()) == RT_OK);
    rt_checkpoint g{};
    std::vector<float> back(mean.size());
    EXPECT(rt_checkpoint_read(path, &g, back.data(), back.size()) == RT_OK);
    EXPECT(std::memcmp(back.data(), mean.data(), back.size() * 4) == 0);
    EXPECT(rt_checkpoint_read(path, &g, back.data(), 3) != RT_OK);   // capacity too small
    {
        std::fstream f(path, std::ios::in | std::ios::out | std::ios::binary);
        f.seekp(sizeof(rt_checkpoint) + 40);
        f.put('\x7f');
    }
    EXPECT(rt_checkpoint_read(path, &g, back.data(), back.size()) != RT_OK);   // checksum
    {
        std::ofstream f(path, std::ios::binary | std::ios::trunc);
        f.write("RTCK", 4);
    }
    EXPECT(rt_checkpoint_read(path, &g, nullptr, 0) != RT_OK);   // truncated header
    std::remove(path);
    EXPECT(rt_checkpoint_read("/nonexistent/dir/x.ckpt", &g, nullptr, 0) != RT_OK);
    EXPECT(rt_version() != nullptr);
}

}  // namespace

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    if (argc > 1) setenv("RTNW_EARTH_PNG", argv[1], 1);
    scenes();
    if (argc > 1) png(argv[1]);
    abi_helpers();
    std::printf(failures ? "FAILED %d\n" : "OK\n", failures);
    return failures ? 1 : 0;
}
