#!/usr/bin/env python3
"""tools/scaling_decomp.py — splits the per-sample cost growth of a rank's share of config 5
 into a fixed per-launch cost and a steady per-sample cost.

For the 1-GPU c5 image and rank 0's share of it at N ranks (`bench.py --share-of N`), the
kernel time of one launch is measured at several spp (each share and spp renders in one
launch); a least-squares line T(spp) = F + c * samples gives the fixed cost F (prologue:
LDS node copy, jump table, first claims; and the launch-end drain) and the steady cost c per
sample (which carries any change of ray coherence from the interleaved pixel lattice).  The
share's cost per sample at 1000 spp, relative to the 1-GPU image's, then splits into
  (c_share - c_c5) / (T_c5 / S_c5)                   the steady-state growth, and
  (F_share / S_share - F_c5 / S_c5) / (T_c5 / S_c5)  the fixed-cost growth,
whose sum is the measured ratio - 1 up to the fits' residuals.

    python tools/scaling_decomp.py --shares 8 [4 2] [--lib L] [--out json]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_ms(extra, lib):
    env = dict(os.environ)
    if lib:
        env["RTNW_LIB"] = os.path.abspath(lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--no-cpu-baseline"] + extra, env=env, capture_output=True, text=True, timeout=900)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    if not line:
        raise RuntimeError(out.stderr[-2000:])
    j = json.loads(line[-1])
    assert j["roofline"]["batches_per_step"] == 1, j["roofline"]["batches_per_step"]
    samples = j["value"] * 1e6 * j["ms_per_step"] / 1e3   # samples per step
    return j["roofline"]["kernel_ms_avg"], samples


def fit(points):
    s = np.array([p[1] for p in points])
    t = np.array([p[0] for p in points])
    c, f = np.polyfit(s, t, 1)   # ms per sample, ms
    return float(f), float(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shares", type=int, nargs="+", default=[8])
    ap.add_argument("--lib", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    res = {}
    c5 = [kernel_ms(["--config", "c5", "--spp", str(spp)], args.lib) for spp in (250, 500, 1000)]
    f1, k1 = fit(c5)
    t1, s1 = c5[-1]
    res["c5"] = {"points_ms_samples": c5, "fixed_ms": f1, "steady_ns_per_sample": k1 * 1e6}
    print(f"c5 1 GPU: fixed {f1:.3f} ms, steady {k1 * 1e6:.4f} ns/sample, 1000 spp {t1:.2f} ms", flush=True)
    for n in args.shares:
        # three spp from 1000 up to what one launch holds (the 16 GiB slab: 12 B per sample)
        top = min(4000, (16 << 30) // (12 * (1000 * 1000 // n)) // 500 * 500)
        pts = [kernel_ms(["--share-of", str(n), "--spp", str(spp)], args.lib) for spp in (1000, (1000 + top) // 2, top)]
        f, k = fit(pts)
        t, s = pts[0]
        base = t1 / s1   # the 1-GPU image's measured cost per sample
        ratio = (t / s) / base
        steady = (k - k1) / base         # growth from the steady per-sample cost
        fixed = (f / s - f1 / s1) / base  # growth from the fixed per-launch cost over fewer samples
        res[f"c5_n{n}"] = {"points_ms_samples": pts, "fixed_ms": f, "steady_ns_per_sample": k * 1e6,
                            "cost_per_sample_vs_c5": ratio, "growth_steady": steady, "growth_fixed": fixed,
                            "growth_fit_residual": ratio - 1 - steady - fixed, "predicted_efficiency": 1 / ratio}
        print(f"share of {n}: fixed {f:.3f} ms, steady {k * 1e6:.4f} ns/sample; cost/sample vs c5 {ratio:.4f} = "
              f"1 + steady {steady:+.4f} + fixed {fixed:+.4f} (fit residual {ratio - 1 - steady - fixed:+.4f})",
              flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
