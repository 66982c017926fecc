// examples/render_main.cpp — the reference's main() (main.cpp:244-336) with its
// pixel loop replaced by the MI355X path.  Scene and camera
// construction are the reference's; only the rendering moved to librt_hip.so.
//
//   render_main [scene] [nx] [ny] [ns] [out.ppm]
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "rt_hip.h"
#include "rtnw_compat.h"

int main(int argc, char **argv) {
    const std::string name = argc > 1 ? argv[1] : "final";
    const int nx = argc > 2 ? std::atoi(argv[2]) : 1000;   // main.cpp:248-251
    const int ny = argc > 3 ? std::atoi(argv[3]) : 1000;
    const int ns = argc > 4 ? std::atoi(argv[4]) : 100;
    const char *out = argc > 5 ? argv[5] : "Test.ppm";

    // cornell-box view, main.cpp:254-259 (the camera main() uses with final())
    vec3 lookfrom(228, 278, -800), lookat(278, 278, 0);
    camera cam(lookfrom, lookat, vec3(0, 1, 0), 40.0, float(nx) / float(ny), 0.0, 10.0, 0.0, 1.0);

    float t0, t1;
    hitable *world = rtnw::build_named_scene(name, &t0, &t1);   // the reference's builders
    if (!world) { std::fprintf(stderr, "unknown scene %s\n", name.c_str()); return 2; }
    auto flat = rtnw::flatten_world(world, t0, t1);

    rt_scene *scene = nullptr;
    if (rt_scene_create(&flat->desc, 0, &scene) != RT_OK) {
        std::fprintf(stderr, "rt_scene_create: %s\n", rt_last_error());
        return 1;
    }
    rt_camera_desc c = cam.desc();
    rt_render_params p = {};
    p.nx = nx; p.ny = ny; p.spp = ns;
    p.max_depth = 50;             // main.cpp:34
    p.t_min = 0.001f;             // main.cpp:27
    p.background = RT_BG_BLACK;   // main.cpp:44
    p.seed = 1;
    std::vector<float> mean(size_t(nx) * ny * 3);
    rt_stats st;
    if (rt_render_tile(scene, &c, &p, 0, 0, nx, ny, mean.data(), &st) != RT_OK) {
        std::fprintf(stderr, "rt_render_tile: %s\n", rt_last_error());
        return 1;
    }
    std::vector<uint8_t> rgb(mean.size());
    rt_quantize(mean.data(), int64_t(nx) * ny, rgb.data());                 // main.cpp:315-325
    std::string ppm(size_t(rt_ppm_text(rgb.data(), nx, ny, nullptr, 0)), '\0');
    rt_ppm_text(rgb.data(), nx, ny, &ppm[0], int64_t(ppm.size()));           // main.cpp:297, 327-330
    std::ofstream(out) << ppm;
    std::printf("%s %dx%dx%d: kernel %.3f ms (%.1f Msamples/s)\n", name.c_str(), nx, ny, ns, st.kernel_ms,
                double(nx) * ny * ns / (st.kernel_ms * 1e3));
    rt_scene_destroy(scene);
    return 0;
}
