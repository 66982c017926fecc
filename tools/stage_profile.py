#!/usr/bin/env python3
"""tools/stage_profile.py — where the engine's wave-cycles go (RT_FLAG_PROFILE
build: s_memtime stamps at the stage boundaries, summed over waves): claim /
traverse / media / shade.  Diagnostic only: shares, never timings."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import rtnw  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "final"
nx, ny, spp = (500, 500, 256) if scene_name == "final" else (400, 400, 64)
cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
sc = rtnw.Scene.builtin(scene_name)
cam = rtnw.Camera.preset(cam_name, nx, ny)
out = {}
for label, flags in (("plain", 0), ("profile", rtnw.RT_FLAG_PROFILE), ("count", rtnw.RT_FLAG_COUNT)):
    p = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, flags=flags, seed=7,
                          chunk=int(os.environ.get("RT_CHUNK", "0")))
    _, st = sc.render_tile(cam, p, 0, 0, nx, ny, stats=True)
    out[label] = st
pr = out["profile"]
tot = sum(pr[k] for k in ("cycles_claim", "cycles_traverse", "cycles_media", "cycles_shade"))
shares = {k: pr[k] / tot for k in ("cycles_claim", "cycles_traverse", "cycles_media", "cycles_shade")}
c = out["count"]
scatter_share = pr["cycles_scatter"] / tot
scatter_eff = c["lane_scatters"] / (64 * max(1, c["wave_shade_passes"]))
kinds = c["wave_shade_kinds"] / max(1, c["wave_shade_passes"])
print(json.dumps({"scene": scene_name, "image": [nx, ny], "spp": spp, "plain_kernel_ms": out["plain"]["kernel_ms"],
                  "profile_kernel_ms": pr["kernel_ms"], "stage_share": shares,
                  "per_ray": {k: c[k] / max(1, c["segments"]) for k in
                              ("node_visits", "sphere_tests", "moving_sphere_tests", "rect_tests", "instanced_tests",
                               "medium_tests", "shades", "noise_evals")},
                  "rays_per_sample": c["segments"] / c["samples"], "grid": out["plain"]["grid"],
                  "simd_efficiency": {
                      "iterations_per_lane_segment": c["wave_iterations"] * 64 / c["segments"],
                      "node_steps": c["node_visits"] / (64 * max(1, c["wave_node_trips"])),
                      "prim_steps": (c["sphere_tests"] + c["rect_tests"] + c["moving_sphere_tests"]
                                     - c["medium_tests"]) / (64 * max(1, c["wave_prim_trips"])),
                      "sphere_draw_rounds": c["lane_sphere_draw_trips"] / (64 * max(1, c["wave_sphere_draw_trips"])),
                      "wave_node_steps_per_iteration": c["wave_node_trips"] / max(1, c["wave_iterations"]),
                      "wave_prim_steps_per_iteration": c["wave_prim_trips"] / max(1, c["wave_iterations"]),
                      "wave_sphere_draw_rounds_per_iteration": c["wave_sphere_draw_trips"] / max(1, c["wave_iterations"]),
                      "scatter_lanes": scatter_eff,
                      "scatter_materials_per_pass": kinds},
                  # material scatter branches (shade_finish, part of cycles_shade): their share of
                  # the wave cycles, and what a free, perfect material sort could remove — every
                  # pass one material with all 64 lanes scattering: share x (1 - efficiency / kinds)
                  "scatter_share": scatter_share,
                  "material_sort_bound": scatter_share * (1 - scatter_eff / max(1e-9, kinds))},
                 indent=1))
