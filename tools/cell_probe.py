#!/usr/bin/env python3
"""tools/cell_probe.py [SCENE] [SPP] — what the medium cell (capi.cpp rt_scene_create,
rt_kernel.hip stage 3) does on a scene: primitives near the cell's ball, the share of ray
segments whose closest hit it decides without a descent, node visits per segment, and the
kernel time with the cell and without it (RTNW_CELL=0), plus whether both images agree
bit for bit.  Diagnostic only."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import rtnw  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "final"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
nx, ny = (500, 500) if scene_name == "final" else (400, 400)
cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
cam = rtnw.Camera.preset(cam_name, nx, ny)
out = {"scene": scene_name, "image": [nx, ny], "spp": spp}
imgs = {}
for cell in ("1", "0"):
    os.environ["RTNW_CELL"] = cell
    sc = rtnw.Scene.builtin(scene_name)
    row = {}
    for label, flags in (("plain", 0), ("count", rtnw.RT_FLAG_COUNT)):
        p = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, flags=flags, seed=7)
        img, st = sc.render_tile(cam, p, 0, 0, nx, ny, stats=True)
        if label == "plain":
            imgs[cell] = img
            row["kernel_ms"] = st["kernel_ms"]
        else:
            seg = max(1.0, st["segments"])
            row.update({"cell_prims": st["cell_prims"], "cell_segment_share": st["cell_segments"] / seg,
                        "segments_per_sample": seg / st["samples"], "node_visits_per_segment": st["node_visits"] / seg,
                        "prim_tests_per_segment": (st["sphere_tests"] + st["rect_tests"] + st["moving_sphere_tests"]) / seg,
                        "wave_iterations": st["wave_iterations"]})
    out["cell" if cell == "1" else "no_cell"] = row
out["bitwise_equal"] = bool(np.array_equal(imgs["1"].view(np.uint32), imgs["0"].view(np.uint32)))
print(json.dumps(out, indent=1))
