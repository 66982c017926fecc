#!/usr/bin/env python3
"""bench.py — Msamples/s of the final() path-tracing workload on MI355X.

Workload (BASELINE.json configs[3], the metric's config): final() (main.cpp:190-230),
camera main.cpp:254-259, 1000 spp, depth 50, black background, 500x500 pixels per
GPU.  One step = one full render of the job: every pixel x every sample, camera
ray -> path -> BVH/primitive/medium hits -> scatter, through the C ABI's
persistent HIP megakernel, plus (N > 1) the RCCL gather of the packed tiles to
rank 0.  Scene upload and BVH build happen before the timed region (inputs
resident in HBM); the PPM write is not part of a step.

Multi-GPU (torchrun, one process per GPU): weak scaling — N ranks render the same
view at N x 250,000 pixels (square, side round(500 sqrt(N)): 500, 707, 1000 =
config 5's image, 1414).  The pixels are interleaved over the ranks (N = a x b,
rank (ry, rx) renders x = rx mod a, y = ry mod b: a sub-sampled copy of the whole
view, so every rank's expected cost is the same), then one torch.distributed
gather (backend "nccl" = RCCL over xGMI) of the packed float pixels to rank 0.  `--dist-backend gloo` gathers through host memory instead, so the
multi-rank path can be rehearsed with several ranks on one GPU.

Prints ONE JSON line (rank 0) with roofline (algorithmic bytes / kernel time vs
8 TB/s HBM) and cpu_baseline (the reference binary on host cores, bounded sample).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd")
ORACLE = os.path.join(ROOT, "oracle")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rtnw  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
TILE = 8                       # unused by the interleaved layout
METRIC = "Msamples/s (pixels×spp/s) + achieved HBM GB/s, final() 500×500×1000spp"   # BASELINE.json
LAYOUT = "interleaved"         # rtnw.pixels_for_rank: rank (ry, rx) of a x b renders x = rx mod a, y = ry mod b


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs on one GPU: scene, image, spp (depth / background / camera:
# rtnw.SCENE_DEFAULTS).  c4 is the metric's config and the default; c2 and c3 are
# reported with --config for DESIGN.md, never as the headline.
CONFIGS = {
    "c2": ("cornell_box", 400, 400, 200),
    "c3": ("random_motion", 800, 400, 500),
    "c4": ("final", 500, 500, 1000),
}


def image_for(n, w=500, h=500):
    """N x (w x h) pixels at the 1-GPU image's aspect and view: sides scaled by sqrt(N)
    (final(): 500, 707, 1000 = config 5's image, 1414).  A wider image would show more
    of the dark ground and cost ~18% less per sample (tools/scaling_probe.py
    --fullres), so per-GPU work would shrink with N."""
    k = n ** 0.5
    return round(w * k), round(h * k)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(budget_procs, scene_name, nx, ny, target_s=8.0):
    """Reference renderer (oracle/_ref/ref_render, compiled from the reference's own
    sources) on host cores, rows split over P processes: a 1-spp pass calibrates the
    sample count so the timed pass takes about `target_s` seconds."""
    ref = os.path.join(ORACLE, "_ref", "ref_render")
    P = budget_procs
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        def run(ns):
            bands = [(ny * i // P, ny * (i + 1) // P) for i in range(P)]
            t0 = time.perf_counter()
            procs = [subprocess.Popen([ref, "--scene", scene_name, "--nx", str(nx), "--ny", str(ny), "--ns", str(ns),
                                       "--depth", str(depth), "--bg", "sky" if bg == rtnw.RT_BG_SKY else "black",
                                       "--cam", cam_name, "--rows", f"{a}:{b}"],
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd="/tmp")
                     for a, b in bands]
            ok = all(p.wait() == 0 for p in procs)
            return ok, time.perf_counter() - t0
        ok, dt1 = run(1)
        if ok:
            ns = max(1, min(1000, round(target_s / max(dt1, 1e-3))))
            ok, dt = run(ns)
            if ok:
                return {"value": nx * ny * ns / dt / 1e6, "unit": "Msamples/s", "cores": P, "kind": "reference",
                        "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                        "sample": f"{scene_name}() {nx}x{ny}x{ns}spp (spp sized by a 1-spp pass), the reference's "
                                  f"own accelerator choice (final(): flat list as shipped, main.cpp:291), rows split "
                                  f"over {P} processes of oracle/_ref/ref_render (clang++ -O2), wall {dt:.2f}s"}
    sys.path.insert(0, ORACLE)
    import oracle as O
    ns = 2
    spec = O.kernel_spec(scene_name, nx, ny, ns, seed=0, threads=P)
    _, st = O.render(spec)
    return {"value": st["samples"] / st["seconds"] / 1e6, "unit": "Msamples/s", "cores": P, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{scene_name}() {nx}x{ny}x{ns}spp, oracle/rt_oracle.c, OpenMP {P} threads, "
                      f"{st['seconds']:.2f}s"}


def read_traffic(samples_per_launch):
    """HBM bytes per launch from the latest committed PMC measurement
    (profiles/r<NN>/traffic.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this workload, FETCH_SIZE doubled per
    the gfx950 correction), scaled to this launch's sample count."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "traffic.json")))
    if not found:
        return None
    try:
        with open(found[-1]) as f:
            t = json.load(f)
        return t["hbm_bytes_per_sample"] * samples_per_launch
    except Exception:
        return None


def end_to_end(scene_name, cam, params, nx, ny, dev):
    """SURVEY §8d's second reading of the metric: one more render of the same
    workload timed from scene creation (flatten, SAH build, upload to HBM) through
    the render to the framebuffer in host memory.  Reported beside `value`, never as
    it (`value` starts with the scene resident)."""
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    scene = rtnw.Scene.builtin(scene_name, device=dev.index)
    t1 = time.perf_counter()
    out = torch.empty(nx * ny * 3, dtype=torch.float32, device=dev)
    scene.render_tiles(cam, params, [(0, 0, nx, ny)], out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    host = out.cpu()
    t3 = time.perf_counter()
    scene.close()
    del host
    return {"value": nx * ny * params.spp / (t3 - t0) / 1e6, "unit": "Msamples/s",
            "includes": "scene create (flatten + SAH BVH + HBM upload) + render + framebuffer readback",
            "scene_create_ms": (t1 - t0) * 1e3, "render_ms": (t2 - t1) * 1e3, "readback_ms": (t3 - t2) * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--chunk", type=int, default=0, help="samples per work item; 0 = the C ABI's default (1 here)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ppm", default="")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)
    if world > 1:
        torch.cuda.set_device(gpu)
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", gpu)

    scene_name, w1, h1, spp = CONFIGS[args.config]
    spp = args.spp or spp
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    nx, ny = image_for(world, w1, h1)
    if world > 1:
        all_tiles, all_counts = rtnw.rank_layout(nx, ny, TILE, world, LAYOUT)
    else:
        all_tiles, all_counts = [[(0, 0, nx, ny)]], [nx * ny * 3]
    tiles = all_tiles[rank]
    n_max = max(all_counts)

    scene = rtnw.Scene.builtin(scene_name, device=gpu)
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    params = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, chunk=args.chunk, seed=2024)
    out = torch.zeros(n_max, dtype=torch.float32, device=dev)
    gdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    gather_list = [torch.empty(n_max, dtype=torch.float32, device=gdev) for _ in range(world)] \
        if (world > 1 and rank == 0) else None

    def step():
        stream = torch.cuda.current_stream(dev).cuda_stream
        st = scene.render_tiles(cam, params, tiles, out.data_ptr(), stream, stats=True)
        if world > 1:
            dist.gather(out if args.dist_backend == "nccl" else out.cpu(), gather_list, dst=0)
        return st

    workload = f"{args.config}: {scene_name}() {nx}x{ny} pixels x {spp} spp, depth {depth}" + \
        (f" over {world} GPUs" if world > 1 else "")
    for i in range(args.warmup):
        st = step()
        log(f"[rank {rank}] warmup {i}: kernel {st['kernel_ms']:.1f} ms")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    kms = []
    for i in range(args.steps):
        st = step()
        kms.append(st["kernel_ms"])
        log(f"[rank {rank}] step {i}: kernel {st['kernel_ms']:.1f} ms")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = nx * ny * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # roofline of the megakernel: algorithmic bytes (counting launch, same RNG -> same
    # paths) over the average HIP-event duration of the timed launches on this rank
    cnt = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, chunk=args.chunk, seed=2024,
                            flags=rtnw.RT_FLAG_COUNT)
    cst = scene.render_tiles(cam, cnt, tiles, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream, stats=True)
    avg_kernel_s = float(np.mean(kms)) / 1e3
    alg = cst["algorithmic_bytes"]
    achieved = alg / avg_kernel_s / 1e9

    if rank == 0 and args.ppm:
        if world == 1:
            img = out[: nx * ny * 3].cpu().numpy().reshape(ny, nx, 3)
        else:   # the last timed step's gathered tiles, unpacked on the root
            img = np.zeros((ny, nx, 3), np.float32)
            for r in range(world):
                rtnw.unpack_tiles(gather_list[r][: all_counts[r]].cpu().numpy(), all_tiles[r], img)
        with open(args.ppm, "wb") as f:
            f.write(rtnw.ppm_text(rtnw.quantize(img)))

    if rank == 0:
        res = {
            "metric": METRIC if args.config == "c4" else
            f"Msamples/s (pixels×spp/s) + achieved HBM GB/s, {scene_name}() {w1}×{h1}×{CONFIGS[args.config][3]}spp",
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: procedural {scene_name}() scene built by the host API (main.cpp builders), "
                    f"counter-RNG samples, seed 2024",
            "config": {"workload": workload, "image": [nx, ny], "spp": spp, "pixels_per_gpu": nx * ny // world,
                       "rank_layout": ("pixel interleave %dx%d" % rtnw.interleave_factors(world)) if world > 1 else None,
                       "chunk": int(cst["chunk"]),
                       "parallelism": f"pixels x{world}" + (" + RCCL gather" if world > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": read_traffic(nx * ny // world * spp) if args.config == "c4" else None,
                         "kernel_ms_avg": avg_kernel_s * 1e3,
                         "algorithmic_bytes_per_launch": alg,
                         "rays_per_sample": cst["segments"] / max(1.0, cst["samples"]),
                         "node_visits_per_ray": cst["node_visits"] / max(1.0, cst["segments"]),
                         "prim_tests_per_ray": (cst["sphere_tests"] + cst["moving_sphere_tests"] + cst["rect_tests"])
                         / max(1.0, cst["segments"]),
                         "algorithmic_bytes_per_sample": alg / max(1.0, cst["samples"]),
                         "note": "algorithmic bytes count every node/primitive fetch; the scene is L2-resident, so "
                                 "frac > 1 is possible and the kernel is VALU-issue bound (DESIGN.md 5c); "
                                 "traffic = PMC HBM bytes per launch (profiles/r01/traffic.json)"},
            "cpu_baseline": None,
        }
        if world == 1:
            res["end_to_end"] = end_to_end(scene_name, cam, params, nx, ny, dev)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(min(16, os.cpu_count() or 1), scene_name, w1, h1)
        print(json.dumps(res), flush=True)
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
