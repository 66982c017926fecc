#!/usr/bin/env python3
"""bench.py — Msamples/s of the final() path-tracing workload on MI355X.

One step = one full render of the job: every pixel x every sample, camera ray ->
path -> BVH/primitive/medium hits -> scatter, through the C ABI's persistent HIP
megakernel (rt_render_tiles, output left in HBM), plus for N > 1 the gather of the
ranks' packed framebuffers to rank 0.  Scene upload and BVH build happen before the
timed region (inputs resident in HBM); the PPM write is not part of a step.

Workloads (BASELINE.json configs):
  N = 1 (default c4, the metric's config): final() (main.cpp:190-230), camera
      main.cpp:254-259, 500 x 500 x 1000 spp, depth 50, black background.
  N > 1 (default c5): final() 1000 x 1000 x 1000 spp split over the N ranks —
      strong scaling, total work fixed (the config BASELINE quotes for 8 GPUs).
      The image's 8 x 8 pixel blocks are dealt to the ranks in turn along a Hilbert
      curve (rtnw.blocks_for_rank: every rank's blocks spread evenly over the view,
      and a wave's 64 items stay one coherent block; RTNW_LAYOUT=interleaved selects
      the pixel interleave, =lattice the block lattice), then ONE
      gather to rank 0: by default the
      C ABI's rt_dist_gather (ncclGather on its own RCCL communicator, rccl.h:745,
      over xGMI), or `--gather torch` (torch.distributed.gather).  `--dist-backend
      gloo` gathers through host memory so the multi-rank path can be rehearsed with
      several ranks on one GPU.
  --config c2 / c3 / c4 with N > 1: weak scaling, N x the 1-GPU pixels.

Launch: under torchrun (WORLD_SIZE set; --gpus must equal it), or plain
`python bench.py --gpus N`, which starts the N rank processes itself (launch_ranks).


Prints ONE JSON line (rank 0) with
  roofline: the megakernel is bound by VALU instruction issue.
    achieved = the wave-level VALU instructions of one launch (SQ_INSTS_VALU per
    sample from the committed rocprofv3 pass, profiles/r<NN>/traffic.json, for this
    very library build) over the kernel's live HIP-event time; peak = the hardware
    ceiling, 1,024 SIMDs x 2.4 GHz (peak engine clock) / 2 cycles per wave64 VALU
    instruction on SIMD-32 (MI355X_MICROARCH.md), independent of the kernel's own
    mix; frac = achieved / peak, useful_frac = frac x lane_utilisation.
    valu_busy_frac = the share of SIMD cycles that issued VALU, at
    the issue cycles per instruction the same build's PMC pass measured: 4 x
    (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU (one quad-cycle per
    wave64 instruction, two instructions in one quad-cycle when they dual-issue:
    tools/lanes_summary.py) — rounds 4-5 reported it as frac.
    hbm_frac = PMC-measured HBM bytes per launch over the same time vs 8 TB/s;
    cache_served_bytes = SURVEY §8d's byte model.
  cpu_baseline: the reference binary (oracle/_ref/ref_render, compiled from the
    reference's own sources) on this job's CPU cores, bounded sample; the flat list
    as shipped (main.cpp:291) and with a corrected BVH (bvh.h:29-54, slab fixed).
"""
import argparse
import glob
import hashlib
import json
import os
import socket
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
SIMDS = 1024                   # 256 CUs x 4 SIMD-32 (MI355X_MICROARCH.md)
CLOCK_GHZ = 2.4                # max engine clock (spec)
VALU_CYCLES = 2                # a wave64 VALU instruction issues over 2 cycles on SIMD-32
VALU_PEAK = SIMDS * CLOCK_GHZ * 1e9 / VALU_CYCLES   # wave-level VALU instructions / s
METRIC = "Msamples/s (pixels×spp/s) + achieved HBM GB/s, final() 500×500×1000spp"   # BASELINE.json
# rtnw.blocks_for_rank (blocks, the default: 8 x 8 pixel blocks dealt along a Hilbert curve),
# rtnw.pixels_for_rank (interleaved: rank (ry, rx) of a x b renders x = rx mod a, y = ry mod b)
# or rtnw.lattice_blocks_for_rank (lattice: the 8 x 8 blocks on that a x b lattice).  Per-share
# probe of the final kernel at N = 8: 0.936-0.939 / 0.929-0.932 / 0.929 predicted efficiency
# (profiles/r05/layouts/)
LAYOUT = os.environ.get("RTNW_LAYOUT", "blocks")


def layout_name(world):
    if LAYOUT == "interleaved":
        return "pixel interleave %dx%d" % rtnw.interleave_factors(world)
    if LAYOUT == "lattice":
        return "8x8 block lattice %dx%d" % rtnw.interleave_factors(world)
    return "8x8 blocks dealt along a Hilbert curve"


def rank_pixels(nx, ny, rank, world):
    fn = {"blocks": rtnw.blocks_for_rank, "lattice": rtnw.lattice_blocks_for_rank}.get(LAYOUT, rtnw.pixels_for_rank)
    return fn(nx, ny, rank, world)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs: scene, image, spp, scaling over N (depth / background /
# camera: rtnw.SCENE_DEFAULTS).  c4 is the metric's config and the 1-GPU default; c5
# the multi-GPU default; c2 and c3 are reported with --config for DESIGN.md.
CONFIGS = {
    "c2": ("cornell_box", 400, 400, 200, "weak"),
    "c3": ("random_motion", 800, 400, 500, "weak"),
    "c4": ("final", 500, 500, 1000, "weak"),
    "c5": ("final", 1000, 1000, 1000, "strong"),
}


def image_for(n, w=500, h=500):
    """Weak scaling: N x (w x h) pixels at the 1-GPU image's aspect and view, sides
    scaled by sqrt(N) (a wider image would show more of the dark ground and cost ~18%
    less per sample, tools/scaling_probe.py --fullres)."""
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


def usable_cores():
    """CPUs this job may use: the affinity mask, capped by the cgroup's CPU quota (the
    GPU box gives a one-GPU job a 16-CPU quota on a 256-CPU host)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return n


def ref_rate(scene_name, nx, ny, procs, accel, target_s):
    """The reference binary on `procs` processes (row bands), a 1-spp pass sizing the
    timed pass to about target_s seconds; returns (Msamples/s, spp, wall s)."""
    ref = os.path.join(ORACLE, "_ref", "ref_render")
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]

    def run(ns):
        bands = [(ny * i // procs, ny * (i + 1) // procs) for i in range(procs)]
        t0 = time.perf_counter()
        ps = [subprocess.Popen([ref, "--scene", scene_name, "--nx", str(nx), "--ny", str(ny), "--ns", str(ns),
                                "--depth", str(depth), "--bg", "sky" if bg == rtnw.RT_BG_SKY else "black",
                               "--cam", cam_name, "--rows", f"{a}:{b}", "--accel", accel],
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd="/tmp")
              for a, b in bands if b > a]
        ok = all(p.wait() == 0 for p in ps)
        return ok, time.perf_counter() - t0

    ok, dt1 = run(1)
    if not ok:
        return None
    ns = max(1, min(1000, round(target_s / max(dt1, 1e-3))))
    ok, dt = run(ns)
    return (nx * ny * ns / dt / 1e6, ns, dt) if ok else None


def cpu_baseline(scene_name, nx, ny, target_s=10.0):
    """Reference renderer on every CPU this job may use: the flat list as shipped
    (main.cpp:291) is `value`; the reference's own bvh_node with the slab test fixed
    (--accel bvh, oracle/ref_harness.cpp fixed_bvh) is reported beside it."""
    ref = os.path.join(ORACLE, "_ref", "ref_render")
    P = usable_cores()
    host = os.cpu_count()
    if os.path.exists(ref) and os.access(ref, os.X_OK):
        flat = ref_rate(scene_name, nx, ny, P, "flat", target_s)
        bvh = ref_rate(scene_name, nx, ny, P, "bvh", target_s)
        if flat:
            res = {"value": flat[0], "unit": "Msamples/s", "cores": P, "kind": "reference",
                   "cpu_model": cpu_model(), "host_cpus": host,
                   "sample": f"{scene_name}() {nx}x{ny}x{flat[1]}spp (spp sized by a 1-spp pass), the reference as "
                             f"shipped (final(): flat list, main.cpp:291), rows split over {P} processes of "
                             f"oracle/_ref/ref_render (clang++ -O2) = this job's CPU quota, wall {flat[2]:.2f}s"}
            if bvh:
                res["corrected_bvh"] = {"value": bvh[0], "unit": "Msamples/s", "cores": P,
                                        "sample": f"{scene_name}() {nx}x{ny}x{bvh[1]}spp, the reference's bvh_node "
                                                  f"(bvh.h:29-54, 97-121) with aabb::hit's slab fixed, wall {bvh[2]:.2f}s"}
            if host and host > P:
                res["all_host_cpus_extrapolated"] = {
                    "cpus": host, "flat": flat[0] * host / P, "corrected_bvh": bvh[0] * host / P if bvh else None,
                    "note": "linear per-core extrapolation; this job may use only its quota"}
            return res
    sys.path.insert(0, ORACLE)
    import oracle as O
    ns = 2
    _, st = O.render(O.kernel_spec(scene_name, nx, ny, ns, seed=0, threads=P))
    return {"value": st["samples"] / st["seconds"] / 1e6, "unit": "Msamples/s", "cores": P, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": host,
            "sample": f"{scene_name}() {nx}x{ny}x{ns}spp, oracle/rt_oracle.c, OpenMP {P} threads, {st['seconds']:.2f}s"}


def lib_sha16():
    with open(rtnw.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def kernel_sha16(path=None):
    """SHA-256 (16 hex) of the library's device code object (its `.hip_fatbin`
    section): the PMC counters of a committed profile depend on the kernels only, so a
    profile stays this build's when only host code changed."""
    import struct
    with open(path or rtnw.LIB_PATH, "rb") as f:
        b = f.read()
    if b[:4] != b"\x7fELF" or b[4] != 2:
        return None
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    for sec in secs:
        name = b[names + sec[0]: b.index(b"\0", names + sec[0])]
        if name == b".hip_fatbin":
            return hashlib.sha256(b[sec[4]: sec[4] + sec[5]]).hexdigest()[:16]
    return None


def read_profile(workload_key, sha=None):
    """The committed PMC summary (profiles/r<NN>/traffic.json, tools/pmc_traffic.py
    from separate rocprofv3 passes of this workload): HBM bytes and VALU instructions
    per sample of the timed megakernel, and the kernels they were measured on.  The
    summary of these very kernels (kernel_sha16 == sha, the device code object) if one
    is committed, else the latest round's (profile_matches_library then says false)."""
    found = []
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "**", "traffic.json"), recursive=True)):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("config", "c4") == workload_key:
            t["path"] = os.path.relpath(path, ROOT)
            found.append(t)
    if not found:
        return None
    same = [t for t in found if sha and (t.get("kernel_sha16") == sha or t.get("lib_sha16") == sha)]
    return (same or found)[-1]


def read_lanes(workload_key, sha):
    """VALU lane utilisation (SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)) and the
    measured issue cycles per VALU instruction (4 (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2)
    / SQ_INSTS_VALU, None in passes without the dual-issue counter) of this workload from the
    committed rocprofv3 pass of these very kernels (profiles/r<NN>/lanes.json,
    tools/lanes_summary.py, matched by kernel_sha16), or None when no pass of this build is
    committed."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "**", "lanes.json"), recursive=True),
                       reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        c = t.get("configs", {}).get(workload_key)
        if sha and t.get("kernel_sha16") == sha and c and c.get("lane_utilisation"):
            return c["lane_utilisation"], os.path.relpath(path, ROOT), c.get("issue_cycles_per_instr"), \
                c.get("dual_issue_share")
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` with no launcher around it: start N FRESH rank processes
    (this interpreter has not touched the GPU: nothing before this call initialises
    HIP) with the rendezvous environment torchrun would give them — the pattern of
    examples/render_dist.cpp's fork-before-HIP launcher, as child processes, never an
    exec of this one.  Rank 0's stdout is this process's stdout (the JSON line).  When
    a rank fails, the others are terminated (a peer stuck in the rendezvous or in the
    gather would otherwise wait forever) and the first failure's code is returned."""
    port = _free_port()
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env))
        rc, live = 0, set(range(n))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    log(f"[launcher] rank {r} exited with {code}: stopping the other ranks")
                    for q in live:
                        procs[q].terminate()
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher (WORLD_SIZE unset) bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="", choices=[""] + sorted(CONFIGS),
                    help="default: c4 on one GPU, c5 (final() 1000^2 x 1000 spp, strong scaling) on several")
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp")
    ap.add_argument("--chunk", type=int, default=0, help="samples per work item; 0 = the C ABI's default (1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ppm", default="")
    ap.add_argument("--dump", default="", help="rank 0 saves the last step's float image (.npy) here")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo rehearses several ranks on one GPU")
    ap.add_argument("--share-of", type=int, default=0,
                    help="profiling: one process renders rank 0's share of config 5 split over N ranks "
                         "(the PMC profile key c5_nN that an N-GPU run's roofline reads)")
    ap.add_argument("--gather", default="auto", choices=["auto", "torch", "native"],
                    help="the C ABI's rt_dist_gather (ncclGather on its own RCCL comm; auto with nccl), or "
                         "torch.distributed.gather (auto with gloo)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RTNW_BENCH_FAIL_RANK") == str(rank):   # tests: a rank that dies before the rendezvous
        log(f"[rank {rank}] RTNW_BENCH_FAIL_RANK: exiting")
        sys.exit(3)
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)
    if world > 1:
        if args.dist_backend == "nccl":
            if world > ndev:
                log(f"bench.py: {world} ranks on {ndev} GPU(s): RCCL needs one GPU per rank "
                    "(--dist-backend gloo rehearses several ranks on one GPU)")
                sys.exit(2)
            torch.cuda.set_device(gpu)
        dist.init_process_group(args.dist_backend)
    if args.gather == "auto":
        args.gather = "native" if args.dist_backend == "nccl" else "torch"
    if args.gather == "native" and args.dist_backend != "nccl" and world > 1:
        log("bench.py: --gather native is an RCCL gather: it needs --dist-backend nccl")
        sys.exit(2)
    dev = torch.device("cuda", gpu)

    share = args.share_of if world == 1 and args.share_of > 1 else 0
    cfg = "c5" if share else (args.config or ("c4" if world == 1 else "c5"))
    scene_name, w1, h1, spp, scaling = CONFIGS[cfg]
    spp = args.spp or spp
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    nx, ny = (w1, h1) if scaling == "strong" else image_for(world, w1, h1)
    if world > 1:
        all_tiles = [rank_pixels(nx, ny, r, world) for r in range(world)]
    elif share:   # a rank's share alone (profiling; its image is that share's pixels)
        all_tiles = [rank_pixels(nx, ny, 0, share)]
    else:
        all_tiles = [[(0, 0, nx, ny)]]
    all_counts = [int(np.asarray(t).reshape(-1, 4)[:, 2:].prod(axis=1).sum()) * 3 for t in all_tiles]
    tiles = all_tiles[rank]
    n_max = max(all_counts)

    scene = rtnw.Scene.builtin(scene_name, device=gpu)
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    params = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, chunk=args.chunk, seed=2024)
    out = torch.zeros(n_max, dtype=torch.float32, device=dev)
    native = world > 1 and args.gather == "native"
    comm = None
    if native:   # the C ABI's own RCCL communicator; the unique id travels over the torch process group
        obj = [rtnw.dist_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = rtnw.Dist(obj[0], rank, world, gpu)
        recv = torch.empty(world * n_max if rank == 0 else 1, dtype=torch.float32, device=dev)
        gather_list = None
    else:
        gdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        gather_list = [torch.empty(n_max, dtype=torch.float32, device=gdev) for _ in range(world)] \
            if (world > 1 and rank == 0) else None

    def step():
        stream = torch.cuda.current_stream(dev).cuda_stream
        st = scene.render_tiles(cam, params, tiles, out.data_ptr(), stream, stats=True)
        if native:
            comm.gather(out.data_ptr(), n_max, recv.data_ptr(), 0, stream)
        elif world > 1:
            dist.gather(out if args.dist_backend == "nccl" else out.cpu(), gather_list, dst=0)
        return st

    workload = f"{cfg}: {scene_name}() {nx}x{ny} pixels x {spp} spp, depth {depth}" + \
        (f", split over {world} GPUs" if world > 1 and scaling == "strong" else
         (f", {world} GPUs x {nx * ny // world} pixels" if world > 1 else "")) + \
        (f", rank 0's share of {share} (profiling)" if share else "")
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
        log(f"[rank {rank}] step {i}: kernel {st['kernel_ms']:.1f} ms ({int(st['batches'])} launch(es))")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = nx * ny * spp if not share else all_counts[0] // 3 * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # roofline of this rank's megakernel launches (HIP events on the render stream)
    rank_samples = all_counts[rank] // 3 * spp
    avg_kernel_s = float(np.mean(kms)) / 1e3
    cnt = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, chunk=args.chunk, seed=2024,
                            flags=rtnw.RT_FLAG_COUNT)
    cst = scene.render_tiles(cam, cnt, tiles, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream, stats=True)
    cache_bytes = cst["algorithmic_bytes"]
    sha = kernel_sha16() or lib_sha16()
    # the PMC profile of this config (c5 on several GPUs: c4's, whose per-sample wave
    # coherence is the closer one — an interleaved rank's 8x8 work block spans 32x16
    # pixels of the 1000^2 view, against 8x8 of c4's 500^2 and 8x8 of c5's on one GPU)
    # the PMC profile of this config; c5 on N GPUs: the profile of one rank's share
    # (bench.py --share-of N on one GPU, key c5_nN: an interleaved rank's work blocks
    # span a4 x 8b pixels of the view, so its coherence is its own)
    nshare = world if world > 1 else share
    prof = read_profile(f"c5_n{nshare}" if cfg == "c5" and nshare > 1 else cfg, sha)
    roof = {"bound": "valu_issue", "achieved": None, "peak": None, "unit": "G wave-VALU-instr/s",
            "frac": None, "traffic": None, "hbm_frac": None, "kernel_ms_avg": avg_kernel_s * 1e3,
            "frac_uniform_2cyc": None, "valu_busy_frac": None, "valu_issue_cycles_per_instr": None,
            "lane_utilisation": None, "useful_frac": None, "useful_frac_uniform_2cyc": None, "lane_profile": None,
            "lds_level": int(st["lds_level"]), "stack_depth": int(st["stack_depth"]), "scan_groups": int(st["scan_groups"]), "prescan": int(st["prescan"]),
            "batches_per_step": int(st["batches"]),
            "valu_insts_per_sample": None, "profile": None, "profile_matches_library": None,
            "cache_served_bytes_per_launch": cache_bytes,
            "cache_served_bytes_per_sample": cache_bytes / max(1.0, cst["samples"]),
            "cache_served_GBps": cache_bytes / avg_kernel_s / 1e9,
            "rays_per_sample": cst["segments"] / max(1.0, cst["samples"]),
            "node_visits_per_ray": cst["node_visits"] / max(1.0, cst["segments"]),
            "prim_tests_per_ray": (cst["sphere_tests"] + cst["moving_sphere_tests"] + cst["rect_tests"])
            / max(1.0, cst["segments"]),
            # SIMD efficiency per stage from the counting run: lane-level events over 64 x
            # the wave-level trips that ran them (node steps, primitive tests, the
            # cooperative rejection rounds' candidates)
            "lane_efficiency": {
                "node_steps": cst["node_visits"] / max(1.0, 64 * cst["wave_node_trips"]),
                # leaf tests: every test minus one boundary-sphere test per medium
                # evaluation (exact when each medium's boundary is one sphere: final())
                "prim_tests": (cst["sphere_tests"] + cst["moving_sphere_tests"] + cst["rect_tests"]
                               - cst["medium_tests"]) / max(1.0, 64 * cst["wave_prim_trips"]),
                "coop_candidates": cst["lane_sphere_draw_trips"] / max(1.0, 64 * cst["wave_sphere_draw_trips"]),
                # material scatter branches (shade_finish): lanes that scattered per wave pass,
                # and the distinct materials a pass ran (branches executed one after another)
                "scatter": cst["lane_scatters"] / max(1.0, 64 * cst["wave_shade_passes"]),
                "scatter_materials_per_pass": cst["wave_shade_kinds"] / max(1.0, cst["wave_shade_passes"]),
                "segments_per_wave_iteration": cst["segments"] / max(1.0, cst["wave_iterations"])},
            "note": "the scene is L2/L1-resident: HBM carries ~1% of peak, the kernel is VALU-issue bound "
                    "(DESIGN.md §5c).  achieved = SQ_INSTS_VALU per sample (committed rocprofv3 pass of this "
                    "library build) x samples / live kernel time; peak = the hardware ceiling, 1024 SIMDs x "
                    "2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md), so frac does not "
                    "depend on how well the kernel issues (since round 6; rounds 4-5 divided by the kernel's "
                    "own issue cycles per instruction, which is valu_busy_frac now); useful_frac = frac x "
                    "lane_utilisation (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU); valu_busy_frac = "
                    "achieved x 4 (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU / (1024 x 2.4 GHz), "
                    "the share of SIMD cycles issuing VALU (SURVEY §8d(iii)); traffic = PMC HBM bytes per "
                    "launch (FETCH_SIZE x 2 + WRITE_SIZE); cache_served = SURVEY §8d byte model (node/primitive "
                    "fetches, mostly L1/L2 hits)"}
    if prof:
        roof["profile"] = prof["path"]
        roof["profile_matches_library"] = sha in (prof.get("kernel_sha16"), prof.get("lib_sha16"))
        if prof.get("valu_insts_per_sample"):
            vi = prof["valu_insts_per_sample"] * rank_samples
            roof["valu_insts_per_sample"] = prof["valu_insts_per_sample"]
            roof["achieved"] = vi / avg_kernel_s / 1e9
            # the hardware ceiling (MI355X_MICROARCH.md): one wave64 VALU instruction per 2
            # cycles per SIMD-32 at the 2.4 GHz peak clock, whatever the kernel's own mix
            # (the fastest opcode measured, v_add_f32 / distinct-source
            # v_fma_f32, issues in 2.3 cycles: profiles/r06/valu_rates.log)
            roof["peak"] = VALU_PEAK / 1e9
            roof["frac"] = vi / avg_kernel_s / VALU_PEAK
            roof["frac_uniform_2cyc"] = roof["frac"]
        # the share of the issued VALU slots' 64 lanes doing work (committed PMC pass of
        # this build): frac says how full the issue roof is, useful_frac how much of it
        # computes for a lane (the headroom is idle lanes, not issue)
        lanes = read_lanes(f"c5_n{nshare}" if cfg == "c5" and nshare > 1 else cfg, sha)
        if lanes:
            roof["lane_utilisation"], roof["lane_profile"] = lanes[0], lanes[1]
            if lanes[2] and roof["achieved"] is not None:
                # VALU busy: the issue cycles the kernel's own instructions
                # took, 4 (ACTIVE - ACTIVE2) / INSTS per instruction (dual issue counted;
                # tools/lanes_summary.py), over the SIMDs' cycles — how often a SIMD issued
                # VALU at all, not a fraction of a hardware roof (until round 5 this was `frac`)
                roof["valu_issue_cycles_per_instr"] = lanes[2]
                roof["dual_issue_share"] = lanes[3]
                roof["valu_busy_frac"] = roof["achieved"] * 1e9 * lanes[2] / (SIMDS * CLOCK_GHZ * 1e9)
            if roof["frac"] is not None:
                roof["useful_frac"] = roof["frac"] * lanes[0]
                roof["useful_frac_uniform_2cyc"] = roof["useful_frac"]
        if prof.get("hbm_bytes_per_sample"):
            tr = prof["hbm_bytes_per_sample"] * rank_samples
            roof["traffic"] = tr
            roof["hbm_frac"] = tr / avg_kernel_s / (HBM_PEAK_GBS * 1e9)

    if rank == 0 and (args.ppm or args.dump) and not share:
        if world == 1:
            img = out[: nx * ny * 3].cpu().numpy().reshape(ny, nx, 3)
        else:   # the last timed step's gathered shares, unpacked on the root
            img = np.zeros((ny, nx, 3), np.float32)
            for r in range(world):
                src = recv[r * n_max:(r + 1) * n_max] if native else gather_list[r]
                rtnw.unpack_tiles(src[: all_counts[r]].cpu().numpy(), all_tiles[r], img)
        if args.ppm:
            with open(args.ppm, "wb") as f:
                f.write(rtnw.ppm_text(rtnw.quantize(img)))
        if args.dump:
            np.save(args.dump, img)

    if rank == 0:
        res = {
            "metric": METRIC if cfg == "c4" else
            f"Msamples/s (pixels×spp/s) + achieved HBM GB/s, {scene_name}() {w1}×{h1}×{spp}spp",
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: procedural {scene_name}() scene built by the host API (main.cpp builders), "
                    f"counter-RNG samples, seed 2024",
            "config": {"workload": workload, "image": [nx, ny], "spp": spp, "pixels_per_gpu": nx * ny // world,
                       "rank_layout": layout_name(world) if world > 1 else None,
                       "chunk": int(cst["chunk"]),
                       "gather": (("rt_dist_gather (ncclGather)" if native else
                                   f"torch.distributed.gather ({args.dist_backend})") if world > 1 else None),
                       "parallelism": f"pixels x{world}" + (" + one gather" if world > 1 else "")},
            "roofline": roof,
            "cpu_baseline": None,
        }
        if world == 1 and not share:
            res["end_to_end"] = end_to_end(scene_name, cam, params, nx, ny, dev)
        if world == 1 and not share and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(scene_name, w1, h1)
        print(json.dumps(res), flush=True)
    if comm is not None:
        comm.close()
    scene.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
