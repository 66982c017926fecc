#!/usr/bin/env python3
"""tools/tail_probe.py — the megakernel's fixed cost per launch (the tail of a
persistent launch: claimed-but-unfinished work items and the last long paths of the
slowest wave), measured as the intercept of kernel time against spp on one image.

    python tools/tail_probe.py [--config c4] [--spps 62,125,250,500,1000] [--claims 0,1,2,4]

claims: RTNW_CLAIM values (x 64 items per wave-level claim; 0 = the C ABI's default).
Prints per claim setting the kernel ms per spp and the least-squares fit
ms = a + b * samples (a = the per-launch fixed cost).  Diagnostic only."""
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
    ap.add_argument("--config", default="c4", choices=sorted(bench.CONFIGS))
    ap.add_argument("--spps", default="62,125,250,500,1000")
    ap.add_argument("--claims", default="0,1,2,4")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    scene_name, nx, ny, _, _ = bench.CONFIGS[args.config]
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = torch.zeros(nx * ny * 3, dtype=torch.float32, device=dev)
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    res = {"config": args.config, "image": [nx, ny], "rows": []}
    for claim in [int(c) for c in args.claims.split(",")]:
        if claim:
            os.environ["RTNW_CLAIM"] = str(claim)
        else:
            os.environ.pop("RTNW_CLAIM", None)
        scene = rtnw.Scene.builtin(scene_name, device=0)
        xs, ys = [], []
        for spp in [int(s) for s in args.spps.split(",")]:
            p = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, seed=2024)
            scene.render_tiles(cam, p, [(0, 0, nx, ny)], out.data_ptr(), stream)
            ms = float(np.median([scene.render_tiles(cam, p, [(0, 0, nx, ny)], out.data_ptr(), stream)["kernel_ms"]
                                  for _ in range(args.repeats)]))
            xs.append(nx * ny * spp)
            ys.append(ms)
        b, a = np.polyfit(np.array(xs, float), np.array(ys, float), 1)
        # the wave timeline of the largest spp (RT_FLAG_PROFILE variant: s_memrealtime per wave)
        pp = rtnw.RenderParams(nx, ny, int(args.spps.split(",")[-1]), max_depth=depth, background=bg, seed=2024,
                               flags=rtnw.RT_FLAG_PROFILE)
        st = scene.render_tiles(cam, pp, [(0, 0, nx, ny)], out.data_ptr(), stream)
        timeline = {k: st[k] for k in ("wave_exhaust_first_us", "wave_exhaust_last_us", "wave_end_first_us",
                                       "wave_end_mean_us", "wave_end_last_us")}
        timeline["profile_kernel_ms"] = st["kernel_ms"]
        row = {"claim": claim, "spp": [int(s) for s in args.spps.split(",")], "kernel_ms": ys,
               "fit_fixed_ms": float(a), "fit_ns_per_sample": float(b * 1e6), "timeline": timeline}
        res["rows"].append(row)
        print(json.dumps(row), flush=True)
        scene.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
