"""Sanitizer builds: the host code of librt_hip.so and the oracle
restatement under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU.

The device code object is linked in unsanitised (GPU sanitizers are not available on
this pool); the host objects are rebuilt here with ``-fsanitize=address,undefined``
and ``-fno-sanitize-recover=all``, so any finding aborts the driver.  Leak detection is
off for the host driver: the reference's scene API allocates its hitables with ``new``
and never frees them (main.cpp builders), which the host API mirrors on purpose.
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
HOST_SOURCES = ["capi.cpp", "bvh.cpp", "flatten.cpp", "rtnw.cpp", "png.cpp", "dist.cpp"]


def _env():
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)   # the sanitizer runtime must come first in the process
    return env


def _run(cmd, **kw):
    out = subprocess.run(cmd, capture_output=True, text=True, **kw)
    assert out.returncode == 0, " ".join(cmd) + "\n" + out.stdout[-4000:] + out.stderr[-4000:]
    return out


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_sanitize")
    _run(["gcc", "-std=c99", "-ffp-contract=off", *SAN, "-I", os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "oracle", "rt_oracle.c"), os.path.join(ROOT, "tests", "native", "oracle_sanitize.c"),
          "-o", exe, "-lm"])
    out = _run([exe], env=dict(_env(), ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1"),
               timeout=600)
    assert out.stdout.strip().endswith("OK")


def test_host_runtime_under_asan_ubsan(tmp_path):
    kernel_obj = os.path.join(PKG, "build", "rt_kernel.o")
    if not os.path.exists(kernel_obj):
        pytest.skip("build/rt_kernel.o missing: run __graft_entry__.build() first")
    inc = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(PKG, "csrc"), "-I", os.path.join(PKG, "csrc", "host")]
    flags = ["g++", "-std=c++17", "-ffp-contract=off", *SAN, *inc]

    def compile_one(src):
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        _run(flags + ["-c", src, "-o", obj])
        return obj

    srcs = [os.path.join(PKG, "csrc", "host", s) for s in HOST_SOURCES]
    srcs.append(os.path.join(ROOT, "tests", "native", "host_sanitize.cpp"))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    exe = str(tmp_path / "host_sanitize")
    _run(["g++", *SAN, *objs, kernel_obj, "-o", exe, "-lz", "-L/opt/rocm/lib", "-lamdhip64", "-lrccl",
          "-Wl,-rpath,/opt/rocm/lib"])
    env = dict(_env(), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:protect_shadow_gap=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = _run([exe, os.path.join(ROOT, "tests", "golden", "picture.png")], env=env, timeout=900)
    assert out.stdout.strip().endswith("OK")
