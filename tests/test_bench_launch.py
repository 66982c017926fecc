"""bench.py as the driver runs it for N GPUs: `python bench.py --gpus N` with no
launcher around it starts the N rank processes itself (bench.launch_ranks), a
`--gpus` that disagrees with a launcher's WORLD_SIZE is refused, a rank that dies
takes the job down instead of leaving its peers in the rendezvous, and (GPU) the
2- and 8-rank jobs render config 5's workload whose gathered image is bitwise the
1-GPU image (the RNG is keyed by pixel and sample)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_must_match_the_launchers_world_size():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


def test_self_launch_stops_the_job_when_a_rank_dies():
    """Rank 1 exits before the rendezvous; rank 0 would wait in init_process_group
    for it (gloo's default timeout is 30 min): the launcher must stop it and return
    rank 1's code."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--no-cpu-baseline"],
                       env=_env(RTNW_BENCH_FAIL_RANK="1"), capture_output=True, text=True, timeout=180)
    assert p.returncode == 3, p.stderr[-2000:]
    assert "stopping the other ranks" in p.stderr


def test_rccl_refuses_more_ranks_than_gpus():
    """backend nccl (RCCL) with more ranks than GPUs is refused up front (exit 2),
    not left to fail inside ncclCommInitRank."""
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--no-cpu-baseline"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "one GPU per rank" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,spp", [(2, 8), (8, 2)])
def test_self_launched_bench_gathers_the_one_gpu_image(tmp_path, n, spp):
    """The driver's N-GPU command shape, rehearsed on one GPU with gloo: N ranks
    (2 and 8, the 8-GPU node's count; bench.py's rank layout: 8x8 blocks dealt along a
    Hilbert curve, or RTNW_LAYOUT's), config 5's image
    (final() 1000 x 1000), strong scaling, through bench.py's own launcher, its gather
    and rank 0's unpack; the gathered image equals a 1-GPU render of the same job bit
    for bit."""
    dump = str(tmp_path / f"c5_{n}ranks.npy")
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dist-backend", "gloo", "--spp", str(spp),
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dump", dump],
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == n and line["scaling"] == "strong"
    assert line["config"]["workload"].startswith("c5: final() 1000x1000")
    assert line["config"]["image"] == [1000, 1000] and line["config"]["spp"] == spp
    layout = os.environ.get("RTNW_LAYOUT", "blocks")
    want = {"blocks": "8x8 blocks dealt along a Hilbert curve",
            "interleaved": "pixel interleave %dx%d" % {2: (2, 1), 8: (4, 2)}[n],
            "lattice": "8x8 block lattice %dx%d" % {2: (2, 1), 8: (4, 2)}[n]}[layout]
    assert line["config"]["rank_layout"] == want
    img = np.load(dump)

    import rtnw
    sc = rtnw.Scene.builtin("final", device=0)
    cam = rtnw.Camera.preset("cornell", 1000, 1000)
    one = sc.render_tile(cam, rtnw.RenderParams(1000, 1000, spp, max_depth=50, seed=2024), 0, 0, 1000, 1000)
    sc.close()
    assert np.array_equal(img.view(np.uint32), one.view(np.uint32))
