#!/usr/bin/env python3
"""tools/ball_probe.py [--spp N] — the ball waves' counters (rt_kernel.hip stage 6) on c4:
one RT_FLAG_COUNT render of final() 500x500 with RTNW_TRACE set (the library prints the
ball-wave line on stderr) per RTNW_BALL_WAVES value given in --waves."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--waves", default="0,2,3,4")
args = ap.parse_args()
code = f"""
import sys; sys.path.insert(0, {os.path.join(ROOT, 'peter-shirley-ray-tracing-the-next-week_amd')!r})
import rtnw
sc = rtnw.Scene.builtin('final', device=0)
cam = rtnw.Camera.preset('cornell', 500, 500)
p = rtnw.RenderParams(500, 500, {args.spp}, seed=2024, flags=rtnw.RT_FLAG_COUNT)
img, st = sc.render_tile(cam, p, 0, 0, 500, 500, stats=True)
print('segments/sample %.3f node visits/segment %.3f kernel %.2f ms' % (st['segments'] / st['samples'],
      st['node_visits'] / st['segments'], st['kernel_ms']))
p = rtnw.RenderParams(500, 500, {args.spp}, seed=2024, flags=rtnw.RT_FLAG_PROFILE)
img, st = sc.render_tile(cam, p, 0, 0, 500, 500, stats=True)
"""
for w in args.waves.split(","):
    env = dict(os.environ, RTNW_BALL_WAVES=w, RTNW_TRACE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"RTNW_BALL_WAVES={w}:", r.stdout.strip(), [l for l in r.stderr.splitlines() if "ball" in l], flush=True)
    if r.returncode:
        print(r.stderr[-2000:])
