"""tests/golden/make_golden.py — regenerates the golden fixtures from the REFERENCE.

Runs oracle/_ref/ref_render (the reference compiled from /root/reference by
oracle/Makefile) in this container and records its outputs as data:

  golden.json        PPM MD5s (canonical drand48 runs, the reference's own RNG),
                     scene-dump SHA-256s, Perlin table hash, drand48 / counter-stream
                     known answers, and the SURVEY §8c MD5s it re-measures;
  ref_<cfg>.npy      small float framebuffers from counter-RNG reference runs
                     (mean radiance after `col /= float(ns)`, rows top-down).

Usage (container only; the reference never travels to the GPU box):
    make -C oracle && python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

# canonical (reference RNG) PPM goldens: (scene, nx, ny, ns)
CANONICAL = [
    ("final", 40, 40, 4), ("final", 100, 100, 10), ("random_scene", 200, 100, 10), ("cornell_box", 40, 40, 8),
    ("cornell_smoke", 32, 32, 4), ("random_motion", 40, 20, 4), ("simple_light", 40, 20, 4),
    ("two_spheres", 20, 20, 4), ("test", 20, 20, 4), ("earth", 40, 40, 8),
    ("edge_empty", 20, 10, 2), ("edge_single", 40, 20, 4), ("edge_degenerate", 40, 20, 8),
]
# counter-RNG reference framebuffers: (name, scene, nx, ny, ns, seed)
COUNTER = [
    ("c1_random", "random_scene", 40, 20, 4, 1), ("c2_cornell", "cornell_box", 24, 24, 8, 2),
    ("c3_motion", "random_motion", 40, 20, 4, 3), ("c4_final", "final", 24, 24, 8, 4),
    ("smoke", "cornell_smoke", 24, 24, 8, 5), ("simple_light", "simple_light", 32, 16, 4, 6),
    ("earth", "earth", 32, 32, 8, 7),
    ("edge_empty", "edge_empty", 16, 8, 2, 12), ("edge_single", "edge_single", 32, 16, 8, 13),
    ("edge_degenerate", "edge_degenerate", 40, 20, 8, 14),
]


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_render missing: run `make -C oracle` in the container that has /root/reference")
    work = tempfile.mkdtemp()
    g = {"generator": "tests/golden/make_golden.py", "reference_binary": "oracle/_ref/ref_render (clang++ -O2)"}
    g["canonical_ppm_md5"] = {}
    for sc, nx, ny, ns in CANONICAL:
        _, ppm, _ = O.ref_render(O.RenderSpec(scene=sc, nx=nx, ny=ny, ns=ns), work)
        g["canonical_ppm_md5"][f"{sc}_{nx}x{ny}x{ns}"] = hashlib.md5(ppm).hexdigest()
    g["scene_dump_sha256"] = {sc: hashlib.sha256(O.ref_dump(sc, work).encode()).hexdigest() for sc in O.SCENES}
    g["counter_fb"] = {}
    for name, sc, nx, ny, ns, seed in COUNTER:
        mean, _, _ = O.ref_render(O.RenderSpec(scene=sc, nx=nx, ny=ny, ns=ns, rng="counter", seed=seed), work)
        np.save(os.path.join(HERE, f"ref_{name}.npy"), mean)
        g["counter_fb"][name] = dict(scene=sc, nx=nx, ny=ny, ns=ns, seed=seed,
                                     sha256=hashlib.sha256(mean.tobytes()).hexdigest())
    # Perlin tables of the reference's static initialisers
    perlin = os.path.join(work, "perlin.bin")
    import subprocess
    subprocess.run([O.REF_BIN, "--scene", "two_spheres", "--nx", "1", "--ny", "1", "--ns", "1", "--perlin", perlin],
                   check=True, capture_output=True)
    g["perlin_sha256"] = hashlib.sha256(open(perlin, "rb").read()).hexdigest()
    # glibc drand48 from an unseeded state (the first values; SURVEY §8c: first = 3.9e-14)
    g["drand48_first"] = [float(x) for x in O.drand48_stream(0, 8)]
    g["counter_draws_seed7_px5_s3"] = [float(x) for x in O.counter_draws(7, 5, 3, 6)]
    g["medium_draw_seed7_px5_s3_b2_k1_of2"] = float(O.medium_draw(7, 5, 3, 2, 1, 2))
    g["survey_clang_md5"] = {"final_40x40x4": "9e7ff7c4c3b8f54d2d59bde695c06e4f",
                             "final_100x100x10": "593c5e4075645c45dc3760d885c21e3b"}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
