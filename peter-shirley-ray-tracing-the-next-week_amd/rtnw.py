"""rtnw.py — Python view of librt_hip.so (include/rt_hip.h) via ctypes.

The path tracer's product is the C ABI; this module is the host-side mirror the
tests and bench.py drive it through, named after the reference's interface:

    scene  = Scene.builtin("final")             # main.cpp:190-230 built by the host API
    cam    = Camera.preset("cornell", nx, ny)   # camera.h:21-39 (main.cpp:254-259)
    mean   = scene.render_tile(cam, RenderParams(nx=.., ny=.., spp=..), 0, 0, nx, ny)
    ppm    = ppm_text(quantize(mean))           # main.cpp:314-330

There is no CPU fallback: every render goes through the HIP megakernel, and
loading fails loudly when librt_hip.so is missing.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTNW_LIB") or os.path.join(HERE, "librt_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "rt_hip.h")

RT_OK = 0
RT_BG_BLACK, RT_BG_SKY = 0, 1
RT_FLAG_COUNT = 1
RT_FLAG_PROFILE = 2
RT_FLAG_SUM_IN = 4      # the output holds the sums of samples [0, sample_offset) on entry
RT_FLAG_SUM_OUT = 8     # write per-pixel sums (checkpoints), not means
RT_CHECKPOINT_MAGIC = 0x4B435452


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt_hip error {code}: {msg}")
        self.code = code


class RtPrim(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("material", ctypes.c_int32), ("instance", ctypes.c_int32),
                ("flip", ctypes.c_int32), ("p", ctypes.c_float * 12)]


class RtInstance(ctypes.Structure):
    _fields_ = [("nops", ctypes.c_int32), ("pad", ctypes.c_int32 * 3), ("ops", (ctypes.c_float * 4) * 6)]


class RtMaterial(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("texture", ctypes.c_int32), ("fuzz", ctypes.c_float),
                ("ref_idx", ctypes.c_float), ("albedo", ctypes.c_float * 3), ("pad", ctypes.c_int32)]


class RtTexture(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("even", ctypes.c_int32), ("odd", ctypes.c_int32),
                ("scale", ctypes.c_float), ("color", ctypes.c_float * 3), ("image", ctypes.c_int32)]


class RtMedium(ctypes.Structure):
    _fields_ = [("boundary_first", ctypes.c_int32), ("boundary_count", ctypes.c_int32), ("density", ctypes.c_float),
                ("material", ctypes.c_int32), ("order", ctypes.c_int32), ("pad", ctypes.c_int32 * 3)]


class RtSceneDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("nprims", ctypes.c_int32), ("nboundary", ctypes.c_int32),
                ("nmedia", ctypes.c_int32), ("nmaterials", ctypes.c_int32), ("ntextures", ctypes.c_int32),
                ("ninstances", ctypes.c_int32),
                ("prims", ctypes.POINTER(RtPrim)), ("boundary_prims", ctypes.POINTER(RtPrim)),
                ("media", ctypes.POINTER(RtMedium)), ("materials", ctypes.POINTER(RtMaterial)),
                ("textures", ctypes.POINTER(RtTexture)), ("instances", ctypes.POINTER(RtInstance)),
                ("perlin_ranvec", ctypes.POINTER(ctypes.c_float)), ("perlin_perm", ctypes.POINTER(ctypes.c_int32)),
                ("time0", ctypes.c_float), ("time1", ctypes.c_float)]


class RtCameraDesc(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("lower_left_corner", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3), ("u", ctypes.c_float * 3),
                ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3), ("lens_radius", ctypes.c_float),
                ("time0", ctypes.c_float), ("time1", ctypes.c_float)]


class RtRenderParams(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("spp", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("t_min", ctypes.c_float), ("background", ctypes.c_int32), ("chunk", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("sample_offset", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("seed", ctypes.c_uint64)]


class RtStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "samples", "segments", "node_visits", "sphere_tests", "moving_sphere_tests", "rect_tests", "instanced_tests",
        "medium_tests", "shades", "noise_evals", "algorithmic_bytes", "kernel_ms", "resolve_ms",
        "cycles_claim", "cycles_traverse", "cycles_media", "cycles_shade", "grid", "wave_iterations",
        "wave_node_trips", "wave_prim_trips", "wave_sphere_draw_trips", "lane_sphere_draw_trips", "chunk",
        "batches", "lds_level", "stack_depth", "scan_groups", "prescan", "wave_exhaust_first_us",
        "wave_exhaust_last_us", "wave_end_first_us", "wave_end_mean_us", "wave_end_last_us",
        "wave_shade_passes", "wave_shade_kinds", "lane_scatters", "cycles_scatter")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class RtCheckpoint(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("version", ctypes.c_uint32), ("nx", ctypes.c_int32),
                ("ny", ctypes.c_int32), ("samples_done", ctypes.c_uint32), ("max_depth", ctypes.c_int32),
                ("background", ctypes.c_int32), ("t_min", ctypes.c_float), ("seed", ctypes.c_uint64),
                ("job_hash", ctypes.c_uint64), ("count", ctypes.c_uint64)]


_lib = None


def lib():
    """Loads librt_hip.so (torch first, so one HIP runtime serves both)."""
    global _lib
    if _lib is None:
        try:  # if torch is present, bind its HIP runtime (same SONAME) before ours
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {HERE}` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        sig = {
            "rt_camera_init": (ctypes.c_int, [P(RtCameraDesc), P(ctypes.c_float), P(ctypes.c_float), P(ctypes.c_float),
                                              ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                              ctypes.c_float, ctypes.c_float]),
            "rt_scene_create": (ctypes.c_int, [P(RtSceneDesc), ctypes.c_int, P(ctypes.c_void_p)]),
            "rt_scene_destroy": (None, [ctypes.c_void_p]),
            "rt_render_tile": (ctypes.c_int, [ctypes.c_void_p, P(RtCameraDesc), P(RtRenderParams), ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, P(RtStats)]),
            "rt_render_tiles": (ctypes.c_int, [ctypes.c_void_p, P(RtCameraDesc), P(RtRenderParams), ctypes.c_void_p,
                                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, P(RtStats)]),
            "rt_device_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, P(ctypes.c_void_p)]),
            "rt_device_free": (ctypes.c_int, [ctypes.c_void_p]),
            "rt_copy_to_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
            "rt_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
            "rt_quantize": (None, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
            "rt_ppm_text": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int64]),
            "rt_builtin_scene_desc": (ctypes.c_int, [ctypes.c_char_p, P(P(RtSceneDesc))]),
            "rt_scene_desc_free": (None, [P(RtSceneDesc)]),
            "rt_scene_desc_dump": (ctypes.c_int64, [P(RtSceneDesc), ctypes.c_char_p, ctypes.c_int64]),
            "rt_checkpoint_write": (ctypes.c_int, [ctypes.c_char_p, P(RtCheckpoint), ctypes.c_void_p]),
            "rt_checkpoint_read": (ctypes.c_int, [ctypes.c_char_p, P(RtCheckpoint), ctypes.c_void_p, ctypes.c_uint64]),
            "rt_dist_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
            "rt_dist_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, P(ctypes.c_void_p)]),
            "rt_dist_destroy": (None, [ctypes.c_void_p]),
            "rt_dist_gather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_void_p]),
            "rt_interleave_factors": (None, [ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int)]),
            "rt_rank_pixels": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_int64]),
            "rt_rank_tiles": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]),
            "rt_dist_set_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
            "rt_unpack_tiles": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p]),
            "rt_dist_render": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, P(RtCameraDesc), P(RtRenderParams),
                                              ctypes.c_void_p, P(RtStats)]),
            "rt_math_probe": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int64]),
            "rt_last_error": (ctypes.c_char_p, []),
            "rt_version": (ctypes.c_char_p, []),
        }
        optional = {"rt_math_probe"}   # diagnostics a library built before them lacks (A/B variants)
        for name, (res, args) in sig.items():
            if name in optional and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


MATH_PROBE = {"sinf": 0, "sinf_ocml": 1, "asinf": 2, "asinf_ocml": 3, "atan2f": 4, "atan2f_ocml": 5}


def math_probe(fn: str, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    """The device's float transcendentals on host inputs (rt_math_probe): `fn` one of
    MATH_PROBE (the megakernel's glibc restatements, rt_libm.h, or ocml's forms)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    bb = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
    out = np.empty_like(a)
    _check(lib().rt_math_probe(MATH_PROBE[fn], a.ctypes.data, bb.ctypes.data, out.ctypes.data, a.size))
    return out


def _check(rc):
    if rc != RT_OK:
        raise RtError(rc, lib().rt_last_error().decode())
    return rc


def header_symbols(path: str = HEADER):
    """Function names declared in include/rt_hip.h."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rt_\w+)\s*\(", text, flags=re.M)))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().rt_device_count(ctypes.byref(n))
    return n.value if rc == RT_OK else 0


# --------------------------------------------------------------------- camera
CAMERA_PRESETS = {   # main.cpp:254-276
    "cornell": dict(lookfrom=(228, 278, -800), lookat=(278, 278, 0), vfov=40.0, aperture=0.0),
    "random": dict(lookfrom=(13, 2, 3), lookat=(0, 0, 0), vfov=20.0, aperture=0.1),
    "final_alt": dict(lookfrom=(478, 278, -600), lookat=(278, 278, 0), vfov=20.0, aperture=0.0),
}


class Camera:
    def __init__(self, lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, t0=0.0, t1=1.0):
        f3 = ctypes.c_float * 3
        self.desc = RtCameraDesc()
        _check(lib().rt_camera_init(ctypes.byref(self.desc), f3(*lookfrom), f3(*lookat), f3(*vup), vfov, aspect,
                                    aperture, focus_dist, t0, t1))

    @classmethod
    def preset(cls, name, nx, ny):
        p = CAMERA_PRESETS[name]
        aspect = float(np.float32(nx) / np.float32(ny))
        return cls(p["lookfrom"], p["lookat"], (0, 1, 0), p["vfov"], aspect, p["aperture"], 10.0, 0.0, 1.0)

    def as_array(self):
        d = self.desc
        return np.array(list(d.origin) + list(d.lower_left_corner) + list(d.horizontal) + list(d.vertical) +
                        list(d.u) + list(d.v) + list(d.w) + [d.lens_radius, d.time0, d.time1], dtype=np.float32)


# ---------------------------------------------------------------------- scene
SCENE_DEFAULTS = {   # per-scene camera / background / depth pairing
    "random_scene": ("random", RT_BG_SKY, 8),
    "random_motion": ("random", RT_BG_SKY, 50),
    "cornell_box": ("cornell", RT_BG_BLACK, 50),
    "cornell_smoke": ("cornell", RT_BG_BLACK, 50),
    "final": ("cornell", RT_BG_BLACK, 50),
    "simple_light": ("random", RT_BG_BLACK, 50),
    "two_spheres": ("random", RT_BG_BLACK, 50),
    "edge_empty": ("random", RT_BG_SKY, 50),        # the tests' edge scenes (oracle/ref_harness.cpp edge_*)
    "edge_single": ("random", RT_BG_SKY, 50),
    "edge_degenerate": ("random", RT_BG_SKY, 50),
    "test": ("random", RT_BG_BLACK, 50),
    "earth": ("cornell", RT_BG_BLACK, 50),
}


def RenderParams(nx, ny, spp, max_depth=50, t_min=0.001, background=RT_BG_BLACK, chunk=0, flags=0, seed=0,
                 sample_offset=0) -> RtRenderParams:
    return RtRenderParams(nx=nx, ny=ny, spp=spp, max_depth=max_depth, t_min=t_min, background=background,
                          chunk=chunk, flags=flags, sample_offset=sample_offset, seed=seed)


class SceneDesc:
    """A flattened scene built by the host API (owned by librt_hip)."""

    def __init__(self, ptr):
        self.ptr = ptr

    @classmethod
    def builtin(cls, name: str, earth_png: str | None = None) -> "SceneDesc":
        """earth() reads its texture like the reference (main.cpp:93): "picture.png" in
        the working directory, or earth_png / $RTNW_EARTH_PNG."""
        if name == "earth" and earth_png:
            os.environ["RTNW_EARTH_PNG"] = earth_png
        p = ctypes.POINTER(RtSceneDesc)()
        _check(lib().rt_builtin_scene_desc(name.encode(), ctypes.byref(p)))
        return cls(p)

    def dump(self) -> str:
        n = lib().rt_scene_desc_dump(self.ptr, None, 0)
        buf = ctypes.create_string_buffer(int(n))
        lib().rt_scene_desc_dump(self.ptr, buf, n)
        return buf.raw[:n].decode()

    @property
    def contents(self) -> RtSceneDesc:
        return self.ptr.contents

    def free(self):
        if self.ptr:
            lib().rt_scene_desc_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Scene:
    """A scene resident in one GPU's HBM (rt_scene_create)."""

    def __init__(self, desc: SceneDesc, device: int = 0):
        self.desc = desc
        self.handle = ctypes.c_void_p()
        _check(lib().rt_scene_create(desc.ptr, device, ctypes.byref(self.handle)))

    @classmethod
    def builtin(cls, name: str, device: int = 0, earth_png: str | None = None) -> "Scene":
        return cls(SceneDesc.builtin(name, earth_png), device)

    def render_tile(self, cam: Camera, params: RtRenderParams, x0, y0, w, h, stats: bool = False, sums=None):
        """Mean radiance of the w x h tile ([h, w, 3] float32).  With RT_FLAG_SUM_IN,
        `sums` holds the running sums of samples [0, params.sample_offset) (e.g. from
        read_checkpoint); with RT_FLAG_SUM_OUT the result is sums, not means."""
        out = np.zeros((h, w, 3), dtype=np.float32)
        if params.flags & RT_FLAG_SUM_IN:
            if sums is None:
                raise ValueError("RT_FLAG_SUM_IN needs the running sums")
            out[...] = np.asarray(sums, np.float32).reshape(h, w, 3)
        st = RtStats()
        _check(lib().rt_render_tile(self.handle, ctypes.byref(cam.desc), ctypes.byref(params), x0, y0, w, h,
                                    out.ctypes.data, ctypes.byref(st)))
        return (out, st.as_dict()) if stats else out

    def render_tiles(self, cam: Camera, params: RtRenderParams, tiles, out_dev_ptr: int, stream_ptr: int = 0,
                     stats: bool = True):
        t = np.ascontiguousarray(np.asarray(tiles, dtype=np.int32).reshape(-1, 4))
        st = RtStats()
        _check(lib().rt_render_tiles(self.handle, ctypes.byref(cam.desc), ctypes.byref(params), t.ctypes.data,
                                     int(t.shape[0]), ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(stream_ptr),
                                     ctypes.byref(st) if stats else None))
        return st.as_dict()

    def close(self):
        if self.handle:
            lib().rt_scene_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------ multi-GPU (RCCL)
RT_DIST_ID_BYTES = 128


def dist_unique_id() -> bytes:
    """ncclGetUniqueId (rt_dist_unique_id): created on the root, handed to every rank."""
    buf = ctypes.create_string_buffer(RT_DIST_ID_BYTES)
    _check(lib().rt_dist_unique_id(buf))
    return buf.raw


class Dist:
    """One rank's RCCL communicator (rt_dist_init = ncclCommInitRank)."""

    def __init__(self, uid: bytes, rank: int, world: int, device: int):
        assert len(uid) == RT_DIST_ID_BYTES
        self.rank, self.world = rank, world
        self.handle = ctypes.c_void_p()
        _check(lib().rt_dist_init(ctypes.create_string_buffer(uid, RT_DIST_ID_BYTES), rank, world, device,
                                  ctypes.byref(self.handle)))

    def gather(self, send_dev: int, count: int, recv_dev: int, root: int = 0, stream: int = 0):
        """ncclGather (rccl.h:745) of `count` floats per rank to `root` (world x count floats)."""
        _check(lib().rt_dist_gather(self.handle, ctypes.c_void_p(send_dev), count, ctypes.c_void_p(recv_dev), root,
                                    ctypes.c_void_p(stream)))

    def set_layout(self, layout: int):
        """rt_dist_set_layout: the split rt_dist_render uses (RT_LAYOUT_*; blocks by default)."""
        _check(lib().rt_dist_set_layout(self.handle, layout))

    def render(self, scene: "Scene", cam: "Camera", params: RtRenderParams):
        """rt_dist_render: this rank's pixels -> render -> gather; the image on rank 0."""
        img = np.zeros((params.ny, params.nx, 3), np.float32) if self.rank == 0 else None
        st = RtStats()
        _check(lib().rt_dist_render(self.handle, scene.handle, ctypes.byref(cam.desc), ctypes.byref(params),
                                    img.ctypes.data if img is not None else None, ctypes.byref(st)))
        return img, st.as_dict()

    def close(self):
        if self.handle:
            lib().rt_dist_destroy(self.handle)
            self.handle = ctypes.c_void_p()


def rank_pixels_c(nx, ny, rank, world):
    """The C ABI's pixel interleave (rt_rank_pixels); equals pixels_for_rank."""
    n = lib().rt_rank_pixels(nx, ny, rank, world, None, 0)
    _check(0 if n >= 0 else int(n))
    t = np.zeros((n, 4), np.int32)
    _check(0 if lib().rt_rank_pixels(nx, ny, rank, world, t.ctypes.data, n) == n else -1)
    return t


# include/rt_hip.h RT_LAYOUT_*: how a job's pixels are split over the ranks
RT_LAYOUT_BLOCKS, RT_LAYOUT_INTERLEAVED, RT_LAYOUT_LATTICE = 0, 1, 2
RT_LAYOUT_BLOCK = 8


def rank_tiles_c(nx, ny, rank, world, layout, block=RT_LAYOUT_BLOCK):
    """The C ABI's rank share (rt_rank_tiles) as 1x1 tiles in claim order."""
    n = lib().rt_rank_tiles(nx, ny, rank, world, layout, block, None, 0)
    _check(0 if n >= 0 else int(n))
    t = np.zeros((n, 4), np.int32)
    _check(0 if lib().rt_rank_tiles(nx, ny, rank, world, layout, block, t.ctypes.data, n) == n else -1)
    return t


# ------------------------------------------------------- checkpoint / resume
def write_checkpoint(path: str, sums: np.ndarray, *, nx, ny, samples_done, params: RtRenderParams | None = None,
                     job_hash: int = 0):
    """Persists per-pixel sums (rt_checkpoint_write: atomic replace, checksummed)."""
    a = np.ascontiguousarray(sums, dtype=np.float32)
    h = RtCheckpoint(nx=nx, ny=ny, samples_done=samples_done, job_hash=job_hash, count=a.size)
    if params is not None:
        h.max_depth, h.background, h.t_min, h.seed = params.max_depth, params.background, params.t_min, params.seed
    _check(lib().rt_checkpoint_write(os.fsencode(path), ctypes.byref(h), a.ctypes.data))


def read_checkpoint(path: str):
    """Returns (header dict, float32 sums) of a checkpoint file."""
    h = RtCheckpoint()
    _check(lib().rt_checkpoint_read(os.fsencode(path), ctypes.byref(h), None, 0))
    a = np.zeros(h.count, np.float32)
    _check(lib().rt_checkpoint_read(os.fsencode(path), ctypes.byref(h), a.ctypes.data, a.size))
    return {n: getattr(h, n) for n, _ in h._fields_}, a


# -------------------------------------------------------------------- resolve
def quantize(mean: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(mean, dtype=np.float32)
    out = np.zeros(m.shape, dtype=np.uint8)
    lib().rt_quantize(m.ctypes.data, m.size // 3, out.ctypes.data)
    return out


def ppm_text(rgb: np.ndarray) -> bytes:
    r = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = r.shape
    n = lib().rt_ppm_text(r.ctypes.data, w, h, None, 0)
    buf = ctypes.create_string_buffer(int(n))
    lib().rt_ppm_text(r.ctypes.data, w, h, buf, n)
    return buf.raw[:n]


def _mix64(z):
    M = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def tiles_for_rank(nx, ny, tile, rank, world, order="diagonal"):
    """Tiles of one rank, in raster order.
    order="diagonal": tile (tx, ty) goes to rank (tx + ty) % world.  Neighbouring
      tiles land on different ranks and the narrow edge tiles rotate over the ranks.
    order="hashed": the tiles are ranked by a hash of their raster index and dealt
      round-robin, so every rank holds the same number of tiles (+-1) scattered
      uniformly over the image: its expected path cost is the image mean whatever
      the scene's spatial structure (bench.py uses 8x8 tiles = one wave claim)."""
    cols = (nx + tile - 1) // tile
    rows = (ny + tile - 1) // tile
    if order == "hashed":
        ranked = sorted(range(cols * rows), key=lambda i: (_mix64(i ^ 0x243F6A8885A308D3), i))
        mine = sorted(ranked[rank::world])
    elif order == "diagonal":
        mine = [ty * cols + tx for ty in range(rows) for tx in range(cols) if (tx + ty) % world == rank]
    else:
        raise ValueError(f"unknown tile order {order!r}")
    out = []
    for i in mine:
        x0, y0 = (i % cols) * tile, (i // cols) * tile
        out.append((x0, y0, min(tile, nx - x0), min(tile, ny - y0)))
    return out


def interleave_factors(world):
    """world = a x b with a >= b as close to square as possible (8 -> 4 x 2)."""
    b = int(world ** 0.5)
    while world % b:
        b -= 1
    return world // b, b


def pixels_for_rank(nx, ny, rank, world, block=8):
    """Pixel interleave: with world = a x b, rank (ry, rx) = divmod(rank, a) renders
    the pixels x = rx (mod a), y = ry (mod b) — a sub-sampled copy of the whole view,
    so every rank's expected path cost is the image mean, whatever the scene's
    spatial structure.  Returned as 1x1 tiles in the order of the rank's
    sub-lattice: bands of `block` rows, each listed column by column, so ANY
    64 consecutive pixels (one wave claim, wherever it starts) cover 8 neighbouring
    columns of one band (two bands at a band's end)."""
    a, b = interleave_factors(world)
    ry, rx = divmod(rank, a)
    xs = np.arange(rx, nx, a, dtype=np.int64)
    ys = np.arange(ry, ny, b, dtype=np.int64)
    if xs.size == 0 or ys.size == 0:
        return np.zeros((0, 4), np.int32)
    J, I = np.meshgrid(np.arange(ys.size), np.arange(xs.size), indexing="ij")
    key = ((J // block) * xs.size + I) * block + J % block
    o = np.argsort(key.ravel(), kind="stable")
    t = np.ones((o.size, 4), np.int32)
    t[:, 0] = xs[I.ravel()[o]]
    t[:, 1] = ys[J.ravel()[o]]
    return t


def blocks_for_rank(nx, ny, rank, world, block=RT_LAYOUT_BLOCK):
    """Block deal (the C ABI's rt_rank_tiles, RT_LAYOUT_BLOCKS — what rt_dist_render and
    bench.py split a job by): the image's block x block pixel blocks, in Hilbert-curve
    order, dealt to the ranks in turn (block k to rank k mod world) — every rank's blocks
    spread evenly over the view (equal counts +-1), and each block keeps the 1-GPU
    render's ray coherence: a wave's 64 items are one 8 x 8 block (pixels_for_rank's
    lattice spreads them over a x 8 by b x 8 pixels).  Returned as 1x1 tiles, block by
    block, each block column by column."""
    return rank_tiles_c(nx, ny, rank, world, RT_LAYOUT_BLOCKS, block)


def lattice_blocks_for_rank(nx, ny, rank, world, block=RT_LAYOUT_BLOCK):
    """Block lattice (rt_rank_tiles, RT_LAYOUT_LATTICE): with world = a x b, rank
    (ry, rx) = divmod(rank, a) renders the block x block pixel blocks (bx, by) with
    bx = rx (mod a), by = ry (mod b) — the pixel interleave's regular sub-sampling of the
    view at block granularity, so each wave's 64 items stay one 8 x 8 block.  Returned as
    1x1 tiles, block by block in row-major block order, each block column by column."""
    return rank_tiles_c(nx, ny, rank, world, RT_LAYOUT_LATTICE, block)


def rank_layout(nx, ny, tile, world, order="diagonal"):
    """Tiles and packed float counts of every rank."""
    if order in ("interleaved", "blocks", "lattice"):   # 1x1 tiles (blocks, lattice: rt_rank_tiles)
        fn = {"blocks": blocks_for_rank, "lattice": lattice_blocks_for_rank}.get(order, pixels_for_rank)
        tiles = [fn(nx, ny, r, world) for r in range(world)]
        return tiles, [len(t) * 3 for t in tiles]
    tiles = [tiles_for_rank(nx, ny, tile, r, world, order) for r in range(world)]
    counts = [sum(w * h for _, _, w, h in t) * 3 for t in tiles]
    return tiles, counts


def unpack_tiles(packed, tiles, img):
    """Scatters one rank's packed tiles (as rt_render_tiles writes them) into img [ny, nx, 3]."""
    t = np.asarray(tiles, dtype=np.int64).reshape(-1, 4)
    if t.size and (t[:, 2:] == 1).all():   # pixel layouts: one vectorised scatter
        img[t[:, 1], t[:, 0]] = np.asarray(packed[: 3 * len(t)]).reshape(-1, 3)
        return img
    off = 0
    for x0, y0, w, h in tiles:
        img[y0:y0 + h, x0:x0 + w] = np.asarray(packed[off:off + w * h * 3]).reshape(h, w, 3)
        off += w * h * 3
    return img
