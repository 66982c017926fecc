#!/usr/bin/env python3
"""tools/scaling_probe.py — the multi-GPU bench's per-rank work, measured on ONE GPU.

`bench.py --gpus N` renders config 5 (final() 1000 x 1000 x 1000 spp, strong
scaling) as N interleaved pixel shares (rtnw.pixels_for_rank: rank (ry, rx) of
a x b renders x = rx mod a, y = ry mod b), one per GPU, then one gather.  For each N
this renders every share of that job on this GPU, one after the other (median
HIP-event kernel time of --repeats launches each), and reports per N:
  * rank_ms and imbalance = max/mean (the N-GPU step is set by the slowest rank);
  * ns_per_sample of the shares against the whole image on one GPU (an interleaved
    share is a sub-sampled view: its wave claims span a x b times the pixels);
  * predicted_msamples_per_s = the job's samples / the slowest share's time, i.e.
    the N-GPU value if the gather (12 MB) and the rendezvous cost nothing.
Diagnostic only; the 8-GPU run itself is the driver's.

    python tools/scaling_probe.py [--ranks 1,2,4,8] [--spp 1000] [--repeats 3] [--out probe.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import rtnw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5", choices=sorted(bench.CONFIGS))
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--spp", type=int, default=0, help="default: the config's (c5: 1000)")
    ap.add_argument("--repeats", type=int, default=3, help="median of this many launches per share")
    ap.add_argument("--out", default="")
    ap.add_argument("--layout", default="interleaved", choices=["interleaved", "blocks", "lattice", "diagonal", "hashed"],
                    help="interleaved: rtnw.pixels_for_rank; blocks: rtnw.blocks_for_rank (8 x 8 blocks dealt along "
                         "a Hilbert curve); diagonal / hashed: --tile blocks (rtnw.tiles_for_rank)")
    ap.add_argument("--tile", type=int, default=8)
    args = ap.parse_args()

    scene_name, nx, ny, spp, _ = bench.CONFIGS[args.config]
    spp = args.spp or spp
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    dev = torch.device("cuda", 0)
    scene = rtnw.Scene.builtin(scene_name, device=0)
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    params = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, seed=2024)
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = torch.zeros(nx * ny * 3, dtype=torch.float32, device=dev)
    res = {"config": args.config, "image": [nx, ny], "spp": spp, "layout": args.layout,
           "tile": args.tile if args.layout != "interleaved" else 1, "kernel_sha16": bench.kernel_sha16(), "runs": []}
    base = None
    for n in [int(x) for x in args.ranks.split(",")]:
        if n == 1:
            shares = [[(0, 0, nx, ny)]]
        elif args.layout == "interleaved":
            shares = [rtnw.pixels_for_rank(nx, ny, r, n) for r in range(n)]
        elif args.layout == "blocks":
            shares = [rtnw.blocks_for_rank(nx, ny, r, n, args.tile) for r in range(n)]
        elif args.layout == "lattice":
            shares = [rtnw.lattice_blocks_for_rank(nx, ny, r, n, args.tile) for r in range(n)]
        else:
            shares = [rtnw.tiles_for_rank(nx, ny, args.tile, r, n, args.layout) for r in range(n)]
        scene.render_tiles(cam, params, shares[0], out.data_ptr(), stream)   # warm
        ms, batches = [], []
        for r in range(n):
            runs = [scene.render_tiles(cam, params, shares[r], out.data_ptr(), stream) for _ in range(args.repeats)]
            ms.append(float(np.median([s["kernel_ms"] for s in runs])))
            batches.append(int(runs[0]["batches"]))
        ns = sum(ms) * 1e6 / (nx * ny * spp)
        base = base or ns
        row = {"n": n, "interleave": list(rtnw.interleave_factors(n)), "rank_ms": ms, "batches": batches,
               "max_ms": max(ms), "mean_ms": sum(ms) / n, "imbalance_max_over_mean": max(ms) / (sum(ms) / n),
               "ns_per_sample": ns, "cost_vs_1gpu_image": ns / base,
               "predicted_msamples_per_s": nx * ny * spp / (max(ms) / 1e3) / 1e6,
               "predicted_strong_scaling_efficiency": base * nx * ny * spp / 1e6 / (n * max(ms))}
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    scene.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
