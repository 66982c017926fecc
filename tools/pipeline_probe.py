#!/usr/bin/env python3
"""tools/pipeline_probe.py [--config c4] [--share-of N] [--steps K] — time K back-to-back
renders of one bench workload issued (a) on one stream, each launch after the previous
one's drain, and (b) alternately on two streams with a scene context each, so that a
launch's workgroups take the CUs its predecessor's drain frees.  Prints ms per step of
both.  Diagnostic for the bench's two-deep render queue."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import rtnw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--share-of", type=int, default=0)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    cfg = "c5" if args.share_of else args.config
    scene_name, nx, ny, spp, _ = bench.CONFIGS[cfg]
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    tiles = bench.rank_pixels(nx, ny, 0, args.share_of) if args.share_of else [(0, 0, nx, ny)]
    dev = torch.device("cuda", 0)
    scenes = [rtnw.Scene.builtin(scene_name, device=0) for _ in range(2)]
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    params = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, seed=2024)
    outs = [torch.zeros(nx * ny * 3, dtype=torch.float32, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for i in range(2):   # warm both contexts (slab, job list)
        scenes[i].render_tiles(cam, params, tiles, outs[i].data_ptr(), streams[i].cuda_stream, stats=False)
    torch.cuda.synchronize(dev)
    label = f"{cfg}" + (f" share of {args.share_of}" if args.share_of else "")
    for r in range(args.rounds):
        res = {}
        for mode in ("serial", "two_streams"):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(args.steps):
                j = k % 2 if mode == "two_streams" else 0
                scenes[j].render_tiles(cam, params, tiles, outs[j].data_ptr(), streams[j].cuda_stream, stats=False)
            torch.cuda.synchronize(dev)
            res[mode] = (time.perf_counter() - t0) / args.steps * 1e3
        print(f"{label} round {r}: ms/step serial {res['serial']:.2f}  two streams {res['two_streams']:.2f}  "
              f"({res['two_streams'] / res['serial'] - 1:+.2%})", flush=True)
    a = outs[0].cpu()
    b = outs[1].cpu()
    print("images of both contexts bitwise equal:", bool(torch.equal(a.view(torch.int32), b.view(torch.int32))))


if __name__ == "__main__":
    main()
