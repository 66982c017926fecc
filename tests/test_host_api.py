"""Host side of the product (librt_hip.so), no GPU needed.

* the library loads and exports every function include/rt_hip.h declares;
* the host API's scene builders + flattener reproduce the reference's scenes
  exactly (leaf dump == reference dump, golden SHA-256);
* the camera, quantiser and PPM writer match the reference arithmetic;
* without a GPU, rendering fails loudly (there is no CPU fallback);
* the device log of constant_medium (host-compiled from the same header) matches glibc.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import rtnw
from conftest import ROOT


def test_library_exports_every_header_symbol():
    L = rtnw.lib()
    declared = rtnw.header_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rtnw.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(declared) <= exported


def test_library_has_gfx950_code_object():
    # the offload bundle carries the target triple amdgcn-amd-amdhsa--gfx950
    data = open(rtnw.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


@pytest.mark.parametrize("scene", list(O.SCENES))
def test_scene_builders_match_reference(golden, scene):
    d = rtnw.SceneDesc.builtin(scene, earth_png=O.EARTH_PNG)
    text = d.dump()
    assert hashlib.sha256(text.encode()).hexdigest() == golden["scene_dump_sha256"][scene]
    assert text == O.scene_dump(scene)


def test_final_scene_shape():
    keep = rtnw.SceneDesc.builtin("final")   # owns the arrays .contents points into
    d = keep.contents
    # 100 boxes x 6 rects + light + moving sphere + 3 spheres + noise sphere + 1000 spheres
    assert d.nprims == 600 + 1 + 1 + 3 + 1 + 1000
    assert d.nmedia == 2 and d.nboundary == 2
    kinds = [d.prims[i].kind for i in range(d.nprims)]
    assert kinds.count(1) == 1 and kinds.count(0) == 1004


def test_cornell_instances():
    keep = rtnw.SceneDesc.builtin("cornell_box")
    d = keep.contents
    assert d.ninstances == 2
    ops = [[d.instances[i].ops[k][0] for k in range(d.instances[i].nops)] for i in range(2)]
    assert ops == [[1.0, 2.0], [1.0, 2.0]]      # translate(rotate_y(box)), outermost first


def _oracle_camera(preset, nx, ny):
    """camera.h:21-39 restated in numpy float32 (the oracle keeps its camera private)."""
    f = np.float32
    p = rtnw.CAMERA_PRESETS[preset]
    lookfrom = np.array(p["lookfrom"], f)
    lookat = np.array(p["lookat"], f)
    vup = np.array([0, 1, 0], f)
    aspect = f(nx) / f(ny)
    fd = f(10.0)

    def unit(v):
        return v / f(np.sqrt(f(f(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])))

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], -(a[0] * b[2] - a[2] * b[0]), a[0] * b[1] - a[1] * b[0]], f)
    theta = f(np.float64(f(p["vfov"])) * np.pi / 180)
    hh = f(np.tan(np.float32(theta / f(2))))
    hw = f(aspect * hh)
    w = unit(lookfrom - lookat)
    u = unit(cross(vup, w))
    v = cross(w, u)
    llc = ((lookfrom - f(hw * fd) * u) - f(hh * fd) * v) - fd * w
    return llc, f(f(f(2) * hw) * fd) * u, f(f(f(2) * hh) * fd) * v


@pytest.mark.parametrize("preset,nx,ny", [("cornell", 500, 500), ("random", 200, 100), ("random", 800, 400)])
def test_camera_matches_reference_arithmetic(preset, nx, ny):
    cam = rtnw.Camera.preset(preset, nx, ny)
    llc, hor, ver = _oracle_camera(preset, nx, ny)
    d = cam.desc
    assert np.allclose(np.array(d.lower_left_corner), llc, rtol=2e-7, atol=1e-6)
    assert np.allclose(np.array(d.horizontal), hor, rtol=2e-7)
    assert np.allclose(np.array(d.vertical), ver, rtol=2e-7)
    assert d.lens_radius == np.float32(rtnw.CAMERA_PRESETS[preset]["aperture"]) / 2


def test_quantize_and_ppm_match_oracle():
    rng = np.random.default_rng(0)
    mean = (rng.random((7, 9, 3)) * 1.5).astype(np.float32)
    mean[0, 0] = [0.0, 1.0, 4.0]
    a = rtnw.quantize(mean)
    b = O.quantize(mean)
    assert np.array_equal(a, b)
    assert rtnw.ppm_text(a) == O.ppm_text(b)
    assert a[0, 0].tolist() == [0, 255, 255]


def test_tiles_cover_image_once():
    nx, ny, t = 100, 70, 32
    seen = np.zeros((ny, nx), np.int32)
    for r in range(3):
        for x0, y0, w, h in rtnw.tiles_for_rank(nx, ny, t, r, 3):
            seen[y0:y0 + h, x0:x0 + w] += 1
    assert (seen == 1).all()


@pytest.mark.skipif(rtnw.device_count() > 0, reason="a GPU is present")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(rtnw.RtError) as e:
        rtnw.Scene.builtin("cornell_box")
    assert e.value.code == -2   # RT_ERR_HIP


def test_descriptor_validation_rejects_bad_material():
    d = rtnw.SceneDesc.builtin("two_spheres")
    c = d.contents
    saved = c.prims[0].material
    c.prims[0].material = 999
    try:
        h = ctypes.c_void_p()
        rc = rtnw.lib().rt_scene_create(d.ptr, 0, ctypes.byref(h))
        assert rc == -1
        assert b"material" in rtnw.lib().rt_last_error()
    finally:
        c.prims[0].material = saved


def test_device_log_matches_glibc(tmp_path):
    """log_f64 (rt_device.h), the device log of constant_medium's free flight
    (constant_medium.h:36), against glibc's log on counter-stream draws: within 1 ulp,
    and never a different float hit_distance for a range of densities."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    pkg = os.path.dirname(rtnw.LIB_PATH)
    exe = str(tmp_path / "log_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(pkg, "csrc"), "-I", os.path.join(pkg, "csrc", "hip"),
                    os.path.join(ROOT, "tests", "native", "log_check.cpp"), "-o", exe],
                   check=True, capture_output=True)
    tested, maxulp, fdiff = (int(v) for v in subprocess.run([exe, "2000000"], check=True, capture_output=True,
                                                            text=True).stdout.split())
    assert tested > 2000000
    assert maxulp <= 1
    assert fdiff == 0


def test_libm_restatement_matches_glibc(tmp_path):
    """csrc/hip/rt_libm.h (the device's sinf / asinf / atan2f, restated from glibc) against
    this host's glibc: every 4,099th finite float and 10^6 atan2f pairs bitwise (the
    exhaustive run over all 2^32 - 2^24 finite floats: profiles/r05/libm_exhaustive.log)."""
    import subprocess
    pkg = os.path.dirname(rtnw.LIB_PATH)
    exe = str(tmp_path / "libm_check")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-I", os.path.join(pkg, "csrc", "hip"),
                    os.path.join(ROOT, "tools", "libm_exhaustive.c"), "-o", exe, "-lm"], check=True, capture_output=True)
    out = subprocess.run([exe, "4099", "1000000"], capture_output=True, text=True)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert "sinf   1043716 finite floats, 0 differ" in out.stdout and "atan2f 1000000 pairs, 0 differ" in out.stdout


def test_bvh_builder_invariants(tmp_path):
    """tests/native/bvh_check.cpp: for BVH widths 2, 4, 8 and compressed 8, on every built-in scene and on
    adversarial synthetic ones (200k uniform, 50k identical, 20k geometric spheres):
    each primitive in exactly one leaf, child boxes contain their primitives,
    breadth-first numbering, and the stack bound within the 24-entry LDS stack."""
    pkg = os.path.dirname(rtnw.LIB_PATH)
    exe = str(tmp_path / "bvh_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(pkg, "csrc"),
                    "-I", os.path.join(pkg, "csrc", "host"), os.path.join(ROOT, "tests", "native", "bvh_check.cpp"),
                    "-o", exe, "-L", pkg, "-lrt_hip", f"-Wl,-rpath,{pkg}"], check=True, capture_output=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK")


def test_c_pixel_interleave_matches_python_layout():
    """rt_rank_pixels (the C ABI the RCCL driver uses) == rtnw.pixels_for_rank (bench.py,
    tests): same factors, same pixels, same claim order; the ranks cover the image once."""
    import ctypes
    for world in (1, 2, 3, 4, 6, 8, 16):
        a, b = ctypes.c_int(), ctypes.c_int()
        rtnw.lib().rt_interleave_factors(world, ctypes.byref(a), ctypes.byref(b))
        assert (a.value, b.value) == rtnw.interleave_factors(world)
        for nx, ny in ((1000, 1000), (37, 23), (3, 2)):
            seen = np.zeros((ny, nx), np.int32)
            for r in range(world):
                t = rtnw.rank_pixels_c(nx, ny, r, world)
                assert np.array_equal(t, rtnw.pixels_for_rank(nx, ny, r, world)), (world, nx, ny, r)
                seen[t[:, 1], t[:, 0]] += 1
            assert (seen == 1).all()


def test_c_unpack_matches_python_unpack():
    import ctypes
    nx, ny = 13, 7
    rng = np.random.default_rng(1)
    t = rtnw.pixels_for_rank(nx, ny, 1, 3)
    packed = rng.random(len(t) * 3).astype(np.float32)
    a = np.zeros((ny, nx, 3), np.float32)
    b = np.zeros((ny, nx, 3), np.float32)
    rtnw.unpack_tiles(packed, t, a)
    assert rtnw.lib().rt_unpack_tiles(packed.ctypes.data, np.ascontiguousarray(t).ctypes.data, len(t), nx, ny,
                                      b.ctypes.data) == 0
    assert np.array_equal(a, b)
    bad = np.array([[nx, 0, 1, 1]], np.int32)
    assert rtnw.lib().rt_unpack_tiles(packed.ctypes.data, bad.ctypes.data, 1, nx, ny, b.ctypes.data) != 0


def test_checkpoint_round_trip_and_corruption(tmp_path):
    """rt_checkpoint_write / rt_checkpoint_read: header and sums survive, a flipped byte
    or a truncated file is refused (checksum), and the write is an atomic replace."""
    sums = np.arange(3 * 20 * 10, dtype=np.float32).reshape(10, 20, 3) * 0.25
    p = rtnw.RenderParams(20, 10, 7, seed=99, max_depth=8, background=rtnw.RT_BG_SKY)
    path = tmp_path / "a.rtck"
    rtnw.write_checkpoint(str(path), sums, nx=20, ny=10, samples_done=7, params=p, job_hash=0xABCDEF)
    assert not (tmp_path / "a.rtck.tmp").exists()
    hdr, back = rtnw.read_checkpoint(str(path))
    assert hdr["magic"] == rtnw.RT_CHECKPOINT_MAGIC and hdr["samples_done"] == 7 and hdr["seed"] == 99
    assert hdr["max_depth"] == 8 and hdr["background"] == rtnw.RT_BG_SKY and hdr["job_hash"] == 0xABCDEF
    assert np.array_equal(back, sums.ravel())
    raw = bytearray(path.read_bytes())
    raw[100] ^= 0x40
    (tmp_path / "b.rtck").write_bytes(bytes(raw))
    with pytest.raises(rtnw.RtError, match="checksum"):
        rtnw.read_checkpoint(str(tmp_path / "b.rtck"))
    (tmp_path / "c.rtck").write_bytes(path.read_bytes()[:-20])
    with pytest.raises(rtnw.RtError):
        rtnw.read_checkpoint(str(tmp_path / "c.rtck"))
    with pytest.raises(rtnw.RtError):
        rtnw.read_checkpoint(str(tmp_path / "missing.rtck"))
    # a crafted header is refused before any buffer is sized by it: count beyond the
    # image (3 nx ny), count not matching the file size, a non-positive image
    off = rtnw.RtCheckpoint.count.offset
    for field_off, value, width in ((off, 1 << 40, 8), (off, 3 * 20 * 10 - 3, 8),
                                    (rtnw.RtCheckpoint.nx.offset, 0, 4)):
        raw = bytearray(path.read_bytes())
        raw[field_off:field_off + width] = int(value).to_bytes(width, "little")
        (tmp_path / "d.rtck").write_bytes(bytes(raw))
        with pytest.raises(rtnw.RtError, match="corrupt checkpoint header"):
            rtnw.read_checkpoint(str(tmp_path / "d.rtck"))
    # a count whose byte size wraps 64 bits: 2^62 + 602 (divisible by 3, within
    # 3 nx ny for a 2^31 - 1 square image) times 4 is 2408 mod 2^64, the size of 602
    # floats, so a multiply-based size check would pass it; the header-only read
    # (the one that sizes the caller's buffer) must refuse it too
    raw = bytearray(path.read_bytes())
    payload_end = len(raw) - 8
    raw[payload_end:payload_end] = bytes(8)   # 600 -> 602 floats of payload
    raw[off:off + 8] = ((1 << 62) + 602).to_bytes(8, "little")
    for f in (rtnw.RtCheckpoint.nx, rtnw.RtCheckpoint.ny):
        raw[f.offset:f.offset + 4] = (2 ** 31 - 1).to_bytes(4, "little")
    (tmp_path / "e.rtck").write_bytes(bytes(raw))
    with pytest.raises(rtnw.RtError, match="corrupt checkpoint header"):
        rtnw.read_checkpoint(str(tmp_path / "e.rtck"))   # refused by its header-only call


def test_shared_reciprocal_division_is_ieee(tmp_path):
    """tests/native/div_rn_check.c: the kernel's div_rn (Markstein: q = RN(x y),
    fma(fma(-q, b, x), y, q) with y = RN(1/b)) equals IEEE x / b on 1e8 random
    divisions of the kernel's shapes (normal reciprocals and quotients)."""
    exe = str(tmp_path / "div_rn_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "native", "div_rn_check.c"),
                    "-o", exe, "-lm"], check=True, capture_output=True)
    out = subprocess.run([exe, "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().startswith("0 mismatches")


def test_block_lattice_partitions_the_image():
    """rtnw.lattice_blocks_for_rank (8 x 8 blocks on the a x b interleave lattice, bench.py
    RTNW_LAYOUT=lattice): the ranks' pixels partition the image, each block's 64 pixels
    consecutive and one block."""
    for nx, ny, world in [(1000, 1000, 8), (37, 23, 3), (64, 8, 2), (500, 500, 4)]:
        seen = np.zeros((ny, nx), int)
        for r in range(world):
            t = rtnw.lattice_blocks_for_rank(nx, ny, r, world)
            seen[t[:, 1], t[:, 0]] += 1
            if nx % 8 == 0 and ny % 8 == 0 and len(t):
                blk = t[:, :2].reshape(-1, 64, 2) // 8
                assert (blk == blk[:, :1]).all()
        assert (seen == 1).all()


def test_block_deal_partitions_the_image():
    """rtnw.blocks_for_rank (the 8 x 8 block deal along a Hilbert curve, bench.py
    RTNW_LAYOUT=blocks and tools/scaling_probe.py --layout blocks): the ranks' pixels
    partition the image, counts within one block, each block's 64 pixels consecutive."""
    for nx, ny, world in [(1000, 1000, 8), (37, 23, 3), (64, 8, 2)]:
        seen = np.zeros((ny, nx), int)
        counts = []
        for r in range(world):
            t = rtnw.blocks_for_rank(nx, ny, r, world)
            counts.append(len(t))
            seen[t[:, 1], t[:, 0]] += 1
            if nx % 8 == 0 and ny % 8 == 0 and len(t):
                blk = t[:, :2].reshape(-1, 64, 2) // 8
                assert (blk == blk[:, :1]).all()
        assert (seen == 1).all()
        assert max(counts) - min(counts) <= 64


def test_math_probe_rejects_bad_arguments():
    """rt_math_probe (the device-transcendental diagnostic) validates before touching the GPU."""
    RT_ERR_INVALID = -1   # include/rt_hip.h
    L = rtnw.lib()
    x = np.zeros(4, np.float32)
    out = np.zeros(4, np.float32)
    assert L.rt_math_probe(6, x.ctypes.data, x.ctypes.data, out.ctypes.data, 4) == RT_ERR_INVALID
    assert L.rt_math_probe(-1, x.ctypes.data, x.ctypes.data, out.ctypes.data, 4) == RT_ERR_INVALID
    assert b"rt_math_probe" in L.rt_last_error()
    assert L.rt_math_probe(4, x.ctypes.data, None, out.ctypes.data, 4) == RT_ERR_INVALID   # atan2f needs b
    assert L.rt_math_probe(0, None, None, out.ctypes.data, 4) == RT_ERR_INVALID
    assert L.rt_math_probe(0, None, None, None, 0) == rtnw.RT_OK   # nothing to do


def test_wave_log_record_size_matches_the_reader():
    """tools/wave_log.py reads the profile variant's per-wave records (RTNW_WAVE_LOG) in
    RT_WAVE_LOG_WORDS words each (rt_kernel.h; capi.cpp sizes the buffer by it)."""
    import re
    hdr = open(os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd", "csrc", "hip", "rt_kernel.h")).read()
    words = int(re.search(r"#define RT_WAVE_LOG_WORDS (\d+)", hdr).group(1))
    tool = open(os.path.join(ROOT, "tools", "wave_log.py")).read()
    assert f"raw.reshape(-1, {words})" in tool
