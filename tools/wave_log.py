#!/usr/bin/env python3
"""tools/wave_log.py — how the waves of one megakernel launch end (RTNW_WAVE_LOG).

Renders c4 once with the profile variant and RTNW_WAVE_LOG set, then reads the
per-wave records (start, pool dry, end: s_memrealtime 100 MHz ticks; xcc << 32 |
HW_ID; items claimed) and prints the distribution of the wave end times, by XCD, by
SIMD and by the wave's slot on its SIMD, and items claimed vs end time.  Diagnostic.

    python tools/wave_log.py [--config c4] [--spp 1000] [--out summary.json]
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import rtnw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=sorted(bench.CONFIGS))
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    scene_name, nx, ny, spp, _ = bench.CONFIGS[args.config]
    spp = args.spp or spp
    cam_name, bg, depth = rtnw.SCENE_DEFAULTS[scene_name]
    path = os.path.join(tempfile.mkdtemp(), "waves.bin")
    os.environ["RTNW_WAVE_LOG"] = path
    sc = rtnw.Scene.builtin(scene_name)
    cam = rtnw.Camera.preset(cam_name, nx, ny)
    p = rtnw.RenderParams(nx, ny, spp, max_depth=depth, background=bg, seed=2024, flags=rtnw.RT_FLAG_PROFILE)
    sc.render_tile(cam, p, 0, 0, 8, 8)   # warm (a small job; its log is discarded)
    os.remove(path)
    _, st = sc.render_tile(cam, p, 0, 0, nx, ny, stats=True)
    raw = np.fromfile(path, dtype=np.uint64)
    if args.out:
        raw.tofile(os.path.splitext(args.out)[0] + ".bin")
    w = raw.reshape(-1, 12)   # RT_WAVE_LOG_WORDS (rt_kernel.h)
    print("records", len(w), "zero starts", int((w[:, 0] == 0).sum()), "first", w[:3].tolist(), file=sys.stderr)
    t0 = w[:, 0].min()
    start, dry, end = [(w[:, k] - t0).astype(np.float64) * 0.01 for k in range(3)]   # us
    xcc = (w[:, 3] >> np.uint64(32)).astype(np.int64) & 0xF
    hw = (w[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    slot, simd, cu = hw & 0xF, (hw >> 4) & 0x3, (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    items = w[:, 4].astype(np.float64)
    # after the wave's dry point: iterations, live lanes summed over them, pooled paths taken
    d_it, d_live, d_taken = (w[:, k].astype(np.float64) for k in (5, 6, 7))
    ball = (np.arange(len(w)) % 16) >= 16 - 3   # the ball waves (RT_BALL_WAVES, the LDS mode's 16-wave groups)
    dcyc = w[:, 8:12].astype(np.float64)   # stage cycles after the dry point
    dshare = lambda m: [float(x) for x in (dcyc[m].sum(0) / max(dcyc[m].sum(), 1))]   # noqa: E731
    q = lambda a: {f"p{k}": float(np.percentile(a, k)) for k in (0, 10, 50, 90, 99, 100)}   # noqa: E731
    res = {"config": args.config, "spp": spp, "waves": int(len(w)), "kernel_ms": st["kernel_ms"],
           "end_us": q(end), "dry_us": q(dry), "end_minus_dry_us": q(end - dry), "items": q(items),
           "end_by_xcc": {int(x): float(end[xcc == x].mean()) for x in np.unique(xcc)},
           "dry_by_xcc": {int(x): float(dry[xcc == x].mean()) for x in np.unique(xcc)},
           "items_by_xcc": {int(x): float(items[xcc == x].mean()) for x in np.unique(xcc)},
           "end_by_simd": {int(x): float(end[simd == x].mean()) for x in np.unique(simd)},
           "items_by_slot": {int(x): float(items[slot == x].mean()) for x in np.unique(slot)},
           "end_by_slot": {int(x): float(end[slot == x].mean()) for x in np.unique(slot)},
           "items_by_se": {int(x): float(items[se == x].mean()) for x in np.unique(se)},
           "items_by_cu_p": q(np.bincount(cu + 16 * (se + 8 * xcc), weights=items)[np.bincount(cu + 16 * (se + 8 * xcc)) > 0]),
           "corr_items_end": float(np.corrcoef(items, end)[0, 1]),
           # the drain: how long an iteration takes once the claims are exhausted, at how many lanes
           "drain_iters": q(d_it), "drain_us_per_iter": q((end - dry) / np.maximum(d_it, 1)),
           "drain_live_per_iter": q(d_live / np.maximum(d_it, 1)), "drain_taken": q(d_taken),
           "drain_us_per_iter_ball": float(((end - dry) / np.maximum(d_it, 1))[ball].mean()),
           "drain_us_per_iter_norm": float(((end - dry) / np.maximum(d_it, 1))[~ball].mean()),
           "end_ball_vs_norm": [float(end[ball].mean()), float(end[~ball].mean())],
           # where a drain iteration's cycles go (claim, traverse, media, shade), and its cycles
           "drain_stage_share_norm": dshare(~ball), "drain_stage_share_ball": dshare(ball),
           "drain_cycles_per_iter_norm": float(dcyc[~ball].sum() / max(d_it[~ball].sum(), 1)),
           "drain_cycles_per_iter_ball": float(dcyc[ball].sum() / max(d_it[ball].sum(), 1)),
           # wave-time idle between a wave's end and the launch's last end, over waves x (last end - first dry)
           "drain_idle_frac": float((end.max() - end).sum() / (len(end) * (end.max() - dry.min()))),
           "last_10_waves": [{"end": float(end[i]), "dry": float(dry[i]), "items": float(items[i]), "xcc": int(xcc[i]),
                              "se": int(se[i]), "cu": int(cu[i]), "simd": int(simd[i]), "slot": int(slot[i]),
                              "ball": bool(ball[i]), "drain_iters": int(d_it[i]), "drain_live": float(d_live[i] / max(d_it[i], 1)),
                              "drain_taken": int(d_taken[i])}
                             for i in np.argsort(end)[-10:]]}
    text = json.dumps(res, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
