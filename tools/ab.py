#!/usr/bin/env python3
"""tools/ab.py LIB... — A/B the megakernel variants on the c4 workload.

Each variant runs in its own process (RTNW_LIB selects the library), interleaved
over `--rounds` rounds so clock drift hits every variant alike; prints the median
kernel time and Msamples/s per variant.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+", help="LIB or LIB:VAR=VAL,VAR=VAL (extra environment), optionally followed by "
                                      "@ and extra bench.py arguments separated by '+' (LIB@--chunk+32)")
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--spp", type=int, default=1000)
args = ap.parse_args()
res = {lib: [] for lib in args.libs}
for r in range(args.rounds):
    for lib in args.libs:
        spec, _, bargs = lib.partition("@")
        path, _, extra = spec.partition(":")
        env = dict(os.environ, RTNW_LIB=os.path.abspath(path))
        for kv in filter(None, extra.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                              "--spp", str(args.spp), "--no-cpu-baseline"] + list(filter(None, bargs.split("+"))), env=env, capture_output=True, text=True,
                             timeout=int(os.environ.get("AB_RUN_TIMEOUT", "150")))
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(lib, "FAILED", out.stderr[-2000:], flush=True)
            continue
        j = json.loads(line[-1])
        res[lib].append((j["roofline"]["kernel_ms_avg"], j["value"]))
        print(f"round {r} {lib}: kernel {j['roofline']['kernel_ms_avg']:.2f} ms, {j['value']:.1f} Msamples/s", flush=True)
for lib, v in res.items():
    if v:
        ks = sorted(x[0] for x in v)
        print(f"SUMMARY {lib}: median kernel {ks[len(ks)//2]:.2f} ms  best {ks[0]:.2f} ms  "
              f"Msamples/s {max(x[1] for x in v):.1f}")
