"""examples/render_main.cpp — the reference's main() with the pixel loop replaced by
the C ABI: it must compile against the compat headers, and on
the GPU produce the same PPM as the Python path with the same parameters."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import rtnw
from conftest import ROOT

EX = os.path.join(ROOT, "examples")


def _build():
    subprocess.run(["make", "-s", "-C", EX], check=True, capture_output=True)
    return os.path.join(EX, "render_main")


def test_example_compiles_against_compat_headers():
    exe = _build()
    assert os.access(exe, os.X_OK)


@pytest.mark.skipif(rtnw.device_count() > 0, reason="a GPU is present")
def test_example_fails_loudly_without_gpu():
    r = subprocess.run([_build(), "final", "8", "8", "1", os.devnull], capture_output=True, text=True)
    assert r.returncode != 0 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["final", "cornell_box"])
def test_example_matches_python_path(scene):
    exe = _build()
    out = os.path.join(tempfile.mkdtemp(), "t.ppm")
    r = subprocess.run([exe, scene, "48", "40", "8", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    sc = rtnw.Scene.builtin(scene)
    cam = rtnw.Camera.preset("cornell", 48, 40)
    mean = sc.render_tile(cam, rtnw.RenderParams(48, 40, 8, seed=1), 0, 0, 48, 40)
    assert open(out, "rb").read() == rtnw.ppm_text(rtnw.quantize(mean))


def test_dist_example_compiles():
    _build()
    assert os.access(os.path.join(EX, "render_dist"), os.X_OK)


@pytest.mark.gpu
def test_dist_example_one_rank_matches_python_path():
    """examples/render_dist (the RCCL driver, no PyTorch) with one rank per GPU of this
    box: its PPM == the Python path's PPM with the same parameters."""
    exe = os.path.join(EX, "render_dist")
    _build()
    out = os.path.join(tempfile.mkdtemp(), "d.ppm")
    r = subprocess.run([exe, "--ranks", "1", "--nx", "40", "--ny", "32", "--ns", "8", "--seed", "5", "--ppm", out],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    sc = rtnw.Scene.builtin("final")
    mean = sc.render_tile(rtnw.Camera.preset("cornell", 40, 32), rtnw.RenderParams(40, 32, 8, seed=5), 0, 0, 40, 32)
    assert open(out, "rb").read() == rtnw.ppm_text(rtnw.quantize(mean))


def _run_dist_with_failing_rank():
    _build()
    env = dict(os.environ, RTNW_DIST_FAIL_RANK="1")
    return subprocess.run([os.path.join(EX, "render_dist"), "--ranks", "2", "--nx", "16", "--ny", "16", "--ns", "1",
                           "--ppm", os.devnull], capture_output=True, text=True, timeout=120, env=env)


@pytest.mark.skipif(rtnw.device_count() > 0, reason="a GPU is present")
def test_dist_example_with_a_failing_rank_ends_without_gpu():
    r = _run_dist_with_failing_rank()
    assert r.returncode != 0


@pytest.mark.gpu
def test_dist_example_stops_the_ranks_when_one_fails():
    """Rank 1 exits after the communicator id exchange, before ncclCommInitRank (as a
    failed scene build would): rank 0 would wait in ncclCommInitRank forever; the
    launcher stops it and returns rank 1's code."""
    r = _run_dist_with_failing_rank()
    assert r.returncode == 3, r.stderr[-2000:]
    assert "stopping the other ranks" in r.stderr
