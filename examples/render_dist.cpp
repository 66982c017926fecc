// examples/render_dist.cpp — the reference's main() (main.cpp:244-336) as a
// multi-GPU job without PyTorch: one process per GPU, an RCCL communicator
// (ncclCommInitRank through rt_dist_init), each rank renders its share of the pixels
// (8 x 8 blocks dealt along a Hilbert curve, rt_rank_tiles, as bench.py splits config 5)
// and ONE ncclGather brings them to rank 0, which writes the PPM
// (config 5: final() 1000x1000x1000 over 8 GPUs).
//
//   render_dist [--ranks N] [--scene final] [--nx 1000] [--ny 1000] [--ns 1000] [--seed S] [--ppm out.ppm]
//               [--layout blocks|interleaved|lattice]
//
// The launcher forks the N rank processes BEFORE anything touches the GPU (no exec);
// rank 0 creates the RCCL unique id and passes it to the others through a pipe.
// N defaults to the number of GPUs (RCCL needs one GPU per rank).
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "rt_hip.h"

namespace {

struct Options {
    int ranks = 0;
    std::string scene = "final", ppm = "Test.ppm";
    int nx = 1000, ny = 1000, ns = 1000;   // main.cpp:248-251 (ns as config 5)
    unsigned long long seed = 1;
    int layout = RT_LAYOUT_BLOCKS;   // rt_dist_set_layout
};

int run_rank(const Options &o, int rank, int rfd, int wfd) {
    uint8_t id[RT_DIST_ID_BYTES];
    if (rank == 0) {   // each side closes the pipe end it does not use, so a failed root means EOF, not a hang
        close(rfd);
        const int ok = rt_dist_unique_id(id) == RT_OK;
        if (!ok) std::fprintf(stderr, "rt_dist_unique_id: %s\n", rt_last_error());
        for (int r = 1; ok && r < o.ranks; ++r)
            if (write(wfd, id, sizeof id) != (ssize_t)sizeof id) { std::perror("write"); return 1; }
        close(wfd);
        if (!ok) return 1;
    } else {
        close(wfd);
        const ssize_t got = read(rfd, id, sizeof id);
        close(rfd);
        if (got != (ssize_t)sizeof id) { std::fprintf(stderr, "[rank %d] no communicator id from rank 0\n", rank); return 1; }
    }
    int ndev = 0;
    if (rt_device_count(&ndev) != RT_OK || ndev == 0) { std::fprintf(stderr, "no HIP device\n"); return 1; }
    const int device = rank % ndev;

    // tests: a rank that fails after the id exchange but before joining the
    // communicator, as a failed scene build would; its peers wait in ncclCommInitRank
    // until the launcher stops them
    const char *fail_rank = std::getenv("RTNW_DIST_FAIL_RANK");
    if (fail_rank && std::atoi(fail_rank) == rank) {
        std::fprintf(stderr, "[rank %d] RTNW_DIST_FAIL_RANK: exiting before rt_dist_init\n", rank);
        return 3;
    }
    rt_scene_desc *desc = nullptr;   // the reference's builder, as a fresh process would run it
    if (rt_builtin_scene_desc(o.scene.c_str(), &desc) != RT_OK) { std::fprintf(stderr, "%s\n", rt_last_error()); return 2; }
    rt_scene *scene = nullptr;
    if (rt_scene_create(desc, device, &scene) != RT_OK) { std::fprintf(stderr, "rt_scene_create: %s\n", rt_last_error()); return 1; }
    // cornell-box view, main.cpp:254-259 (the camera main() uses with final())
    const float from[3] = {228, 278, -800}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
    rt_camera_desc cam;
    rt_camera_init(&cam, from, at, up, 40.0f, float(o.nx) / float(o.ny), 0.0f, 10.0f, 0.0f, 1.0f);
    rt_render_params p = {};
    p.nx = o.nx; p.ny = o.ny; p.spp = o.ns;
    p.max_depth = 50;             // main.cpp:34
    p.t_min = 0.001f;             // main.cpp:27
    p.background = RT_BG_BLACK;   // main.cpp:44
    p.seed = o.seed;

    rt_dist *comm = nullptr;
    if (rt_dist_init(id, rank, o.ranks, device, &comm) != RT_OK) { std::fprintf(stderr, "rt_dist_init: %s\n", rt_last_error()); return 1; }
    if (rt_dist_set_layout(comm, o.layout) != RT_OK) { std::fprintf(stderr, "rt_dist_set_layout: %s\n", rt_last_error()); return 1; }
    std::vector<float> image(rank == 0 ? size_t(o.nx) * o.ny * 3 : 0);
    rt_stats st;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = rt_dist_render(comm, scene, &cam, &p, rank == 0 ? image.data() : nullptr, &st);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc != RT_OK) std::fprintf(stderr, "[rank %d] rt_dist_render: %s\n", rank, rt_last_error());
    std::fprintf(stderr, "[rank %d/%d] GPU %d: %.0f samples, kernel %.3f ms\n", rank, o.ranks, device, st.samples, st.kernel_ms);
    if (rc == RT_OK && rank == 0) {
        std::vector<uint8_t> rgb(image.size());
        rt_quantize(image.data(), int64_t(o.nx) * o.ny, rgb.data());   // main.cpp:315-325
        std::string text(size_t(rt_ppm_text(rgb.data(), o.nx, o.ny, nullptr, 0)), '\0');
        rt_ppm_text(rgb.data(), o.nx, o.ny, &text[0], int64_t(text.size()));   // main.cpp:297, 327-330
        std::ofstream(o.ppm) << text;
        std::printf("%s %dx%dx%d on %d GPU(s): %.3f s render + gather (%.1f Msamples/s)\n", o.scene.c_str(), o.nx, o.ny,
                    o.ns, o.ranks, secs, double(o.nx) * o.ny * o.ns / secs / 1e6);
    }
    rt_dist_destroy(comm);
    rt_scene_destroy(scene);
    rt_scene_desc_free(desc);
    return rc == RT_OK ? 0 : 1;
}

}  // namespace

int main(int argc, char **argv) {
    Options o;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--ranks") o.ranks = std::atoi(v.c_str());
        else if (k == "--scene") o.scene = v;
        else if (k == "--nx") o.nx = std::atoi(v.c_str());
        else if (k == "--ny") o.ny = std::atoi(v.c_str());
        else if (k == "--ns") o.ns = std::atoi(v.c_str());
        else if (k == "--seed") o.seed = std::strtoull(v.c_str(), nullptr, 0);
        else if (k == "--ppm") o.ppm = v;
        else if (k == "--layout" && (v == "blocks" || v == "interleaved" || v == "lattice"))
            o.layout = v == "blocks" ? RT_LAYOUT_BLOCKS : v == "interleaved" ? RT_LAYOUT_INTERLEAVED : RT_LAYOUT_LATTICE;
        else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }
    if (o.ranks <= 0) {   // one rank per GPU, counted in a child so that this launcher never initialises HIP
        const pid_t probe = fork();
        if (probe == 0) {
            int n = 0;
            _exit(rt_device_count(&n) == RT_OK ? (n > 100 ? 100 : n) : 0);
        }
        int status = 0;
        waitpid(probe, &status, 0);
        o.ranks = WIFEXITED(status) ? WEXITSTATUS(status) : 0;
        if (o.ranks == 0) { std::fprintf(stderr, "no HIP device\n"); return 1; }
    }
    int fds[2];
    if (pipe(fds) != 0) { std::perror("pipe"); return 1; }
    std::vector<pid_t> kids;
    for (int r = 0; r < o.ranks; ++r) {
        const pid_t pid = fork();
        if (pid < 0) { std::perror("fork"); return 1; }
        if (pid == 0) _exit(run_rank(o, r, fds[0], fds[1]));
        kids.push_back(pid);
    }
    close(fds[0]);
    close(fds[1]);
    // The first rank to fail stops the others: a peer of a rank that died before the
    // communicator existed, or before the gather, would otherwise wait forever in
    // ncclCommInitRank / ncclGather.  Returns the first failure's code.
    int first = 0;
    size_t left = kids.size();
    while (left > 0) {
        int status = 0;
        const pid_t k = waitpid(-1, &status, 0);
        if (k < 0) break;
        --left;
        for (pid_t &kid : kids)
            if (kid == k) kid = 0;
        const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
        if (code != 0 && first == 0) {
            first = code;
            std::fprintf(stderr, "[launcher] a rank exited with %d: stopping the other ranks\n", code);
            for (pid_t kid : kids)
                if (kid > 0) kill(kid, SIGTERM);
        }
    }
    return first;
}
