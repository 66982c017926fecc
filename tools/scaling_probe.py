#!/usr/bin/env python3
"""tools/scaling_probe.py — the multi-GPU bench's per-rank work, measured on ONE GPU.

For each N in --ranks, builds the image bench.py uses at N GPUs and the tile lists
rank_layout deals to the N ranks, then renders every rank's tile list on this GPU
one after the other (HIP-event kernel time each).  Reports, per N:
  * per-sample cost of the N-GPU image relative to the 1-GPU image (weak scaling
    holds per-GPU work fixed only if this stays ~1), and
  * max/mean of the per-rank kernel times (load imbalance: the bench's value is set
    by the slowest rank).
Diagnostic only; the 8-GPU run itself is the driver's."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import rtnw  # noqa: E402

def wide_image(n):
    w, h, k = 500, 500, 1
    while k < n:
        w, h, k = (w * 2, h, k * 2) if w <= h else (w, h * 2, k * 2)
    return w, h


ap = argparse.ArgumentParser()
ap.add_argument("--ranks", default="1,2,4,8")
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--tile", type=int, default=bench.TILE)
ap.add_argument("--wide", action="store_true", help="the earlier N-GPU images: 500x500, 1000x500, 1000x1000, 2000x1000")
ap.add_argument("--order", default=bench.LAYOUT, choices=["diagonal", "hashed", "interleaved"])
ap.add_argument("--reverse", action="store_true", help="render the ranks last to first")
ap.add_argument("--repeats", type=int, default=3, help="median of this many launches per rank")
ap.add_argument("--fullres", action="store_true",
                help="instead: whole images of side 500 sqrt(N) and 2:1 ones at spp / N (equal sample counts)")
args = ap.parse_args()

dev = torch.device("cuda", 0)
scene = rtnw.Scene.builtin("final", device=0)
if args.fullres:
    dev = torch.device("cuda", 0)
    scene = rtnw.Scene.builtin("final", device=0)
    for n in [int(x) for x in args.ranks.split(",")]:
        for nx, ny in ({bench.image_for(n), wide_image(n)}):
            spp = args.spp // n
            cam = rtnw.Camera.preset("cornell", nx, ny)
            params = rtnw.RenderParams(nx, ny, spp, max_depth=50, seed=2024)
            out = torch.zeros(nx * ny * 3, dtype=torch.float32, device=dev)
            stream = torch.cuda.current_stream(dev).cuda_stream
            t = sorted(scene.render_tiles(cam, params, [(0, 0, nx, ny)], out.data_ptr(), stream)["kernel_ms"]
                       for _ in range(args.repeats + 1))[: args.repeats]
            print(json.dumps({"image": [nx, ny], "spp": spp, "ns_per_sample": t[len(t) // 2] * 1e6 / (nx * ny * spp)}),
                  flush=True)
    sys.exit(0)
res = {"spp": args.spp, "tile": args.tile, "order": args.order, "wide": args.wide, "runs": []}
base = None
for n in [int(x) for x in args.ranks.split(",")]:
    nx, ny = wide_image(n) if args.wide else bench.image_for(n)
    cam = rtnw.Camera.preset("cornell", nx, ny)
    params = rtnw.RenderParams(nx, ny, args.spp, max_depth=50, seed=2024)
    tiles, counts = rtnw.rank_layout(nx, ny, args.tile, n, args.order) if n > 1 else ([[(0, 0, nx, ny)]], [nx * ny * 3])
    out = torch.zeros(max(counts), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    scene.render_tiles(cam, params, tiles[0], out.data_ptr(), stream, stats=True)   # warm
    ms = [0.0] * n
    for r in (reversed(range(n)) if args.reverse else range(n)):
        t = sorted(scene.render_tiles(cam, params, tiles[r], out.data_ptr(), stream, stats=True)["kernel_ms"]
                   for _ in range(args.repeats))
        ms[r] = t[len(t) // 2]
    ns_per_sample = sum(ms) * 1e6 / (nx * ny * args.spp)
    if base is None:
        base = ns_per_sample
    row = {"n": n, "image": [nx, ny], "rank_ms": ms, "ns_per_sample": ns_per_sample,
           "cost_vs_1gpu_image": ns_per_sample / base, "imbalance_max_over_mean": max(ms) / (sum(ms) / n)}
    res["runs"].append(row)
    print(json.dumps(row), flush=True)
scene.close()
print(json.dumps(res))
