"""Multi-rank path on CPU (gloo, world size 2): rank sharding (the Hilbert block deal
bench.py and rt_dist_render use, the pixel interleave, the block lattice and diagonal
tiles), packed
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


def render_rank(rank, world, order):
    tiles, counts = rtnw.rank_layout(NX, NY, TILE, world, order)
    buf = np.zeros(max(counts), np.float32)
    if order in ("interleaved", "blocks", "lattice"):   # 1x1 tiles: this rank's pixels of the image
        full, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED))
        t = tiles[rank]
        buf[: 3 * len(t)] = full[t[:, 1], t[:, 0]].reshape(-1)
        return buf, tiles, counts
    off = 0
    for (x0, y0, w, h) in tiles[rank]:
        m, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED, rect=(x0, y0, w, h)))
        buf[off:off + w * h * 3] = m.reshape(-1)
        off += w * h * 3
    return buf, tiles, counts


def _worker(rank, world, port, order, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, tiles, counts = render_rank(rank, world, order)
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


@pytest.mark.parametrize("world,order", [(2, "blocks"), (2, "interleaved"), (2, "lattice"), (2, "diagonal")])
def test_gloo_gather_equals_single_rank_image(world, order):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, order, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED))
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


@pytest.mark.parametrize("order", ["blocks", "interleaved", "diagonal", "hashed"])
def test_layout_covers_image_once_and_balances_ranks(order):
    import bench
    for world in (2, 3, 4, 8):
        nx, ny = bench.image_for(world)
        tiles, counts = rtnw.rank_layout(nx, ny, 8, world, order)
        assert sum(counts) == nx * ny * 3
        assert max(counts) / min(counts) < 1.02
        cover = np.zeros((ny, nx), np.int32)
        for t in tiles:
            for x0, y0, w, h in np.asarray(t).reshape(-1, 4).tolist():
                cover[y0:y0 + h, x0:x0 + w] += 1
        assert (cover == 1).all(), (order, world)


def test_interleave_claims_are_local():
    """64 consecutive pixels of a rank (one wave claim) mostly stay within an 8x8
    block of its sub-lattice, i.e. an 8a x 8b window of the image (a partial block
    at the sub-lattice's right edge shifts the claims that follow it)."""
    for world in (2, 4, 8):
        a, b = rtnw.interleave_factors(world)
        t = rtnw.pixels_for_rank(1000, 1000, world - 1, world)
        local = [np.ptp(g[:, 0]) < 8 * a and np.ptp(g[:, 1]) < 16 * b
                 for g in (t[k:k + 64] for k in range(0, len(t) - 64, 64))]
        assert np.mean(local) > 0.9, (world, np.mean(local))


def _gpu_worker(rank, world, port, q, layout=1):
    """One rank of the product path: its pixels (rt_rank_tiles' layout) through
    librt_hip.so (rt_render_tiles into device memory), gathered with gloo to rank 0."""
    import ctypes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tiles = rtnw.rank_tiles_c(NX, NY, rank, world, layout)
    nmax = max(len(rtnw.rank_tiles_c(NX, NY, r, world, layout)) for r in range(world)) * 3
    sc = rtnw.Scene.builtin("final", device=0)
    cam = rtnw.Camera.preset("cornell", NX, NY)
    p = rtnw.RenderParams(NX, NY, NS, seed=SEED)
    L = rtnw.lib()
    dev = ctypes.c_void_p()
    assert L.rt_device_alloc(0, nmax * 4, ctypes.byref(dev)) == 0
    st = sc.render_tiles(cam, p, tiles, dev.value)
    buf = np.zeros(nmax, np.float32)
    assert L.rt_copy_to_host(buf.ctypes.data, dev, len(tiles) * 12) == 0
    L.rt_device_free(dev)
    t = torch.from_numpy(buf)
    gl = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gl, dst=0)
    if rank == 0:
        img = np.zeros((NY, NX, 3), np.float32)
        for r in range(world):
            tr = rtnw.rank_tiles_c(NX, NY, r, world, layout)
            rtnw.unpack_tiles(gl[r][: 3 * len(tr)].numpy(), tr, img)
        q.put((img, st["samples"]))
    dist.barrier()
    sc.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [rtnw.RT_LAYOUT_BLOCKS, rtnw.RT_LAYOUT_INTERLEAVED])
def test_gloo_gather_of_product_renders_equals_single_gpu_image(layout):
    """World size 2 on one GPU, each rank driving librt_hip.so (not the oracle) with the
    C ABI's split (rt_rank_tiles: the Hilbert block deal, the pixel interleave): the
    gathered image == the 1-rank GPU image bitwise == the oracle within the bar."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q, layout)) for r in range(2)]
    for p in procs:
        p.start()
    img, samples = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert samples == len(rtnw.rank_tiles_c(NX, NY, 0, 2, layout)) * NS
    sc = rtnw.Scene.builtin("final", device=0)
    one = sc.render_tile(rtnw.Camera.preset("cornell", NX, NY), rtnw.RenderParams(NX, NY, NS, seed=SEED), 0, 0, NX, NY)
    assert np.array_equal(img.view(np.uint32), one.view(np.uint32))
    ora, _ = O.render(O.kernel_spec("final", NX, NY, NS, seed=SEED, chunk=1))
    g = np.sqrt(np.clip(img, 0, 1)) - np.sqrt(np.clip(ora, 0, 1))
    assert (np.sqrt(np.mean(g ** 2, axis=(0, 1))) <= 1e-3).all()


@pytest.mark.gpu
def test_rccl_one_rank_communicator_gather_equals_render_tile():
    """The native multi-GPU path (rt_dist_*: ncclGetUniqueId, ncclCommInitRank,
    ncclGather) with a 1-rank communicator — the gather to self — returns exactly the
    rt_render_tile image; then the raw gather of a device buffer to itself."""
    nx, ny, ns = 64, 48, 6
    sc = rtnw.Scene.builtin("final", device=0)
    cam = rtnw.Camera.preset("cornell", nx, ny)
    p = rtnw.RenderParams(nx, ny, ns, seed=3)
    d = rtnw.Dist(rtnw.dist_unique_id(), 0, 1, 0)
    ref = sc.render_tile(cam, p, 0, 0, nx, ny)
    for layout in (rtnw.RT_LAYOUT_BLOCKS, rtnw.RT_LAYOUT_INTERLEAVED, rtnw.RT_LAYOUT_LATTICE):
        d.set_layout(layout)
        img, st = d.render(sc, cam, p)
        assert st["samples"] == nx * ny * ns
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    data = torch.arange(1000, dtype=torch.float32, device="cuda")
    recv = torch.zeros(1000, dtype=torch.float32, device="cuda")
    d.gather(data.data_ptr(), 1000, recv.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(recv, data)
    d.close()


@pytest.mark.gpu
def test_dist_render_refuses_running_sum_flags():
    """rt_dist_render gathers freshly rendered MEAN shares: RT_FLAG_SUM_IN (which would
    start from zero sums yet divide by sample_offset + spp) and RT_FLAG_SUM_OUT (sums
    delivered as the root's mean image) are refused, on every rank alike."""
    sc = rtnw.Scene.builtin("final", device=0)
    cam = rtnw.Camera.preset("cornell", 16, 16)
    d = rtnw.Dist(rtnw.dist_unique_id(), 0, 1, 0)
    for flag in (rtnw.RT_FLAG_SUM_IN, rtnw.RT_FLAG_SUM_OUT):
        with pytest.raises(rtnw.RtError, match="not supported"):
            d.render(sc, cam, rtnw.RenderParams(16, 16, 2, seed=1, flags=flag, sample_offset=3))
    img, st = d.render(sc, cam, rtnw.RenderParams(16, 16, 2, seed=1))   # the communicator is still usable
    assert st["samples"] == 16 * 16 * 2 and np.isfinite(img).all()
    d.close()
    sc.close()
