"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes view of the plain-C restatement (liboracle.so, rt_oracle.h) and a runner
for the reference binary compiled from /root/reference (oracle/_ref/ref_render).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_render")

SCENES = {
    "random_scene": 0, "random_motion": 1, "cornell_box": 2, "cornell_smoke": 3,
    "final": 4, "simple_light": 5, "two_spheres": 6, "test": 7, "earth": 8,
    "edge_empty": 9, "edge_single": 10, "edge_degenerate": 11,   # the tests' edge cases (ref_harness.cpp edge_*)
}
EARTH_PNG = os.path.join(os.path.dirname(HERE), "tests", "golden", "picture.png")   # main.cpp:93's asset
CAMERAS = {"cornell": 0, "random": 1, "final_alt": 2}
# Per-scene defaults, as the reference driver pairs them (main.cpp:254-291) plus
# the chapter-1/3 sky background for the random scenes.
SCENE_DEFAULTS = {
    "random_scene": dict(camera="random", background="sky", max_depth=8),
    "random_motion": dict(camera="random", background="sky", max_depth=50),
    "cornell_box": dict(camera="cornell", background="black", max_depth=50),
    "cornell_smoke": dict(camera="cornell", background="black", max_depth=50),
    "final": dict(camera="cornell", background="black", max_depth=50),
    "simple_light": dict(camera="random", background="black", max_depth=50),
    "two_spheres": dict(camera="random", background="black", max_depth=50),
    "test": dict(camera="random", background="black", max_depth=50),
    "earth": dict(camera="cornell", background="black", max_depth=50),
    "edge_empty": dict(camera="random", background="sky", max_depth=50),
    "edge_single": dict(camera="random", background="sky", max_depth=50),
    "edge_degenerate": dict(camera="random", background="sky", max_depth=50),
}


def host_libm_pinned():
    """(pinned, why): whether this host's libm is the one csrc/hip/rt_libm.h restates —
    glibc 2.35 on an x86-64 CPU with FMA (its sinf ifunc then runs the FMA variant whose
    constants rt_libm.h was read from).  The oracle calls the host's sinf / asinf / atan2f
    (texture.h:36, 55; hitable.h:14-19), so a GPU image is the oracle's bit for bit only on
    such a host; on another the parity bar is north_star's RMS one and the exact-pixel
    share is reported, not asserted (tests/test_gpu_parity.py assert_exact, smoke())."""
    import platform
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.gnu_get_libc_version.restype = ctypes.c_char_p
        ver = libc.gnu_get_libc_version().decode()
    except (OSError, AttributeError):
        return False, "the host C library is not glibc"
    if ver != "2.35":
        return False, f"host glibc {ver}, rt_libm.h restates 2.35"
    if platform.machine() != "x86_64":
        return False, f"host {platform.machine()}, rt_libm.h restates the x86-64 FMA variant"
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False, "no /proc/cpuinfo to check for FMA"
    if " fma" not in flags:
        return False, "host CPU without FMA: glibc's sinf runs its non-FMA variant"
    return True, "glibc 2.35, x86-64 with FMA"


def png_rgba(path):
    """Minimal 8-bit non-interlaced PNG decode (test-side; independent of the product's)."""
    import struct
    import zlib
    d = open(path, "rb").read()
    assert d[:8] == b"\x89PNG\r\n\x1a\n"
    i, idat, w, h, ct = 8, b"", 0, 0, 0
    while i < len(d):
        n, = struct.unpack(">I", d[i:i + 4])
        t = d[i + 4:i + 8]
        if t == b"IHDR":
            w, h, bd, ct = struct.unpack(">IIBB", d[i + 8:i + 18])
            assert bd == 8
        elif t == b"IDAT":
            idat += d[i + 8:i + 8 + n]
        i += 12 + n
    ch = {0: 1, 2: 3, 4: 2, 6: 4}[ct]
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * ch + 1)
    out = np.zeros((h, w * ch), np.int32)
    for y in range(h):
        f, row = raw[y, 0], raw[y, 1:].astype(np.int32)
        up = out[y - 1] if y else np.zeros(w * ch, np.int32)
        cur = np.zeros(w * ch, np.int32)
        for x in range(w * ch):
            a = cur[x - ch] if x >= ch else 0
            b = up[x]
            c = up[x - ch] if x >= ch else 0
            if f == 0: v = row[x]
            elif f == 1: v = row[x] + a
            elif f == 2: v = row[x] + b
            elif f == 3: v = row[x] + ((a + b) >> 1)
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                v = row[x] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))
            cur[x] = v & 255
        out[y] = cur
    return out.astype(np.uint8).reshape(h, w, ch)


_image_loaded = False


def load_earth_image(path=None):
    """Hands earth()'s texels to the oracle (done once per process)."""
    global _image_loaded
    if _image_loaded:
        return
    img = np.ascontiguousarray(png_rgba(path or EARTH_PNG))
    h, w, ch = img.shape
    lib().oracle_set_image(img.ctypes.data, w, h, ch)
    _image_loaded = True


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("scene", ctypes.c_int32), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("ns", ctypes.c_int32),
        ("max_depth", ctypes.c_int32), ("background", ctypes.c_int32), ("tmin", ctypes.c_float),
        ("camera", ctypes.c_int32), ("rng", ctypes.c_int32), ("media_after", ctypes.c_int32),
        ("forward", ctypes.c_int32), ("chunk", ctypes.c_int32),
        ("x0", ctypes.c_int32), ("y0", ctypes.c_int32), ("w", ctypes.c_int32), ("h", ctypes.c_int32),
        ("threads", ctypes.c_int32), ("sample_offset", ctypes.c_uint32), ("pad_", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
    ]


class OracleStats(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_double), ("segments", ctypes.c_double), ("seconds", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_render.argtypes = [ctypes.POINTER(OracleParams), ctypes.c_void_p, ctypes.POINTER(OracleStats)]
        L.oracle_render.restype = ctypes.c_int
        L.oracle_quantize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.oracle_ppm_text.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_long]
        L.oracle_ppm_text.restype = ctypes.c_long
        L.oracle_perlin_tables.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_drand48.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        L.oracle_counter_draws.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.oracle_medium_draw.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int]
        L.oracle_medium_draw.restype = ctypes.c_double
        L.oracle_scene_dump.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_long]
        L.oracle_set_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_scene_dump.restype = ctypes.c_long
        _lib = L
    return _lib


@dataclass
class RenderSpec:
    scene: str = "final"
    nx: int = 40
    ny: int = 40
    ns: int = 4
    max_depth: int | None = None
    background: str | None = None
    camera: str | None = None
    tmin: float = 0.001
    rng: str = "canonical"          # or "counter"
    seed: int = 0
    sample_offset: int = 0
    media_after: bool = False       # kernel order
    forward: bool = False           # kernel accumulation
    chunk: int = 0
    rect: tuple | None = None       # (x0, y0, w, h) image coords
    threads: int = 1

    def resolved(self):
        d = SCENE_DEFAULTS[self.scene]
        return (self.max_depth if self.max_depth is not None else d["max_depth"],
                self.background or d["background"], self.camera or d["camera"])


def render(spec: RenderSpec):
    """Returns (mean float32 array [h, w, 3], stats dict)."""
    if spec.scene == "earth":
        load_earth_image()
    depth, bg, cam = spec.resolved()
    x0, y0, w, h = spec.rect if spec.rect else (0, 0, spec.nx, spec.ny)
    p = OracleParams(scene=SCENES[spec.scene], nx=spec.nx, ny=spec.ny, ns=spec.ns, max_depth=depth,
                     background=1 if bg == "sky" else 0, tmin=spec.tmin, camera=CAMERAS[cam],
                     rng=1 if spec.rng == "counter" else 0, media_after=int(spec.media_after),
                     forward=int(spec.forward), chunk=spec.chunk, x0=x0, y0=y0, w=w, h=h,
                     threads=spec.threads, sample_offset=spec.sample_offset, seed=spec.seed)
    out = np.zeros((h, w, 3), dtype=np.float32)
    st = OracleStats()
    rc = lib().oracle_render(ctypes.byref(p), out.ctypes.data, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return out, {"samples": st.samples, "segments": st.segments, "seconds": st.seconds}


def kernel_spec(scene: str, nx: int, ny: int, ns: int, *, seed: int = 0, chunk: int = 0, **kw) -> RenderSpec:
    """The CPU statement of exactly what the GPU kernel computes (counter RNG,
    media after surfaces, forward throughput, chunked partial sums)."""
    return RenderSpec(scene=scene, nx=nx, ny=ny, ns=ns, rng="counter", seed=seed, media_after=True,
                      forward=True, chunk=chunk, **kw)


def quantize(mean: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(mean, dtype=np.float32)
    n = m.size // 3
    rgb = np.zeros(n * 3, dtype=np.uint8)
    lib().oracle_quantize(m.ctypes.data, n, rgb.ctypes.data)
    return rgb.reshape(m.shape)


def ppm_text(rgb: np.ndarray) -> bytes:
    h, w, _ = rgb.shape
    r = np.ascontiguousarray(rgb, dtype=np.uint8)
    n = lib().oracle_ppm_text(r.ctypes.data, w, h, None, 0)
    buf = ctypes.create_string_buffer(n)
    lib().oracle_ppm_text(r.ctypes.data, w, h, buf, n)
    return buf.raw[:n]


def ppm_md5(mean: np.ndarray) -> str:
    return hashlib.md5(ppm_text(quantize(mean))).hexdigest()


def perlin_tables():
    rv = np.zeros(768, dtype=np.float32)
    pm = np.zeros(768, dtype=np.int32)
    lib().oracle_perlin_tables(rv.ctypes.data, pm.ctypes.data)
    return rv.reshape(256, 3), pm.reshape(3, 256)


def drand48_stream(x0: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.float64)
    lib().oracle_drand48(x0, n, out.ctypes.data)
    return out


def counter_draws(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.float64)
    lib().oracle_counter_draws(seed, pixel, sample, n, out.ctypes.data)
    return out


def medium_draw(seed: int, pixel: int, sample: int, bounce: int, medium: int, nmedia: int) -> float:
    """constant_medium draw of medium `medium` at segment `bounce` in a scene of `nmedia` media."""
    return lib().oracle_medium_draw(seed, pixel, sample, bounce, medium, nmedia)


def scene_dump(scene: str) -> str:
    if scene == "earth":
        load_earth_image()
    n = lib().oracle_scene_dump(SCENES[scene], None, 0)
    buf = ctypes.create_string_buffer(n)
    lib().oracle_scene_dump(SCENES[scene], buf, n)
    return buf.raw[:n].decode()


# ------------------------------------------------------------ reference binary
def have_ref() -> bool:
    return os.path.exists(REF_BIN) and os.access(REF_BIN, os.X_OK)


def ref_render(spec: RenderSpec, workdir: str, rows: tuple | None = None, timing: bool = False):
    """Runs the compiled reference; returns (mean [rows, nx, 3], ppm bytes, timing dict|None)."""
    depth, bg, cam = spec.resolved()
    fb = os.path.join(workdir, "ref_fb.f32")
    ppm = os.path.join(workdir, "ref.ppm")
    cmd = [REF_BIN, "--scene", spec.scene, "--nx", str(spec.nx), "--ny", str(spec.ny), "--ns", str(spec.ns),
           "--depth", str(depth), "--bg", bg, "--cam", cam, "--tmin", repr(spec.tmin),
           "--rng", spec.rng, "--seed", str(spec.seed), "--fb", fb, "--ppm", ppm,
           "--assets", os.path.dirname(EARTH_PNG)]
    if rows:
        cmd += ["--rows", f"{rows[0]}:{rows[1]}"]
    if timing:
        cmd += ["--time"]
    res = subprocess.run(cmd, capture_output=True, text=True, check=True)
    nrows = (rows[1] - rows[0]) if rows else spec.ny
    mean = np.fromfile(fb, dtype=np.float32).reshape(nrows, spec.nx, 3)
    with open(ppm, "rb") as f:
        text = f.read()
    tinfo = None
    if timing:
        import json
        tinfo = json.loads(res.stdout.strip().splitlines()[-1])
    return mean, text, tinfo


def ref_dump(scene: str, workdir: str) -> str:
    path = os.path.join(workdir, f"dump_{scene}.txt")
    subprocess.run([REF_BIN, "--scene", scene, "--nx", "1", "--ny", "1", "--ns", "1", "--dump", path,
                    "--assets", os.path.dirname(EARTH_PNG)],
                   capture_output=True, check=True)
    with open(path) as f:
        return f.read()
