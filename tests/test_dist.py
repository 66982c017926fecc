"""Multi-rank path on CPU (gloo, world size 2): interleaved tile sharding, packed
per-rank buffers padded to a common length, one collective gather to rank 0,
unpack on the root.  The per-tile renderer here is the oracle's statement of the
kernel (the same per-pixel values the GPU produces; tests/test_gpu_parity.py
checks GPU sharding bitwise on the device), so the gathered image must equal the
single-rank image bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
import rtnw

NX, NY, NS, TILE, SEED = 40, 24, 4, 8, 17


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render_rank(rank, world):
    tiles, counts = rtnw.rank_layout(NX, NY, TILE, world)
    buf = np.zeros(max(counts), np.float32)
    off = 0
    for (x0, y0, w, h) in tiles[rank]:
        m, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED, rect=(x0, y0, w, h)))
        buf[off:off + w * h * 3] = m.reshape(-1)
        off += w * h * 3
    return buf, tiles, counts


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, tiles, counts = render_rank(rank, world)
    t = torch.from_numpy(buf)
    gl = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gl, dst=0)
    if rank == 0:
        img = np.zeros((NY, NX, 3), np.float32)
        for r in range(world):
            rtnw.unpack_tiles(gl[r][: counts[r]].numpy(), tiles[r], img)
        q.put(img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_gather_equals_single_rank_image(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED))
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


def test_layout_balances_ranks():
    for world in (2, 4, 8):
        nx, ny = {2: (1000, 500), 4: (1000, 1000), 8: (2000, 1000)}[world]
        _, counts = rtnw.rank_layout(nx, ny, 32, world)
        assert sum(counts) == nx * ny * 3
        assert max(counts) / min(counts) < 1.02
