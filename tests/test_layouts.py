"""The C ABI's rank shares (rt_rank_tiles, include/rt_hip.h RT_LAYOUT_*) against an
independent numpy restatement: the 8 x 8 block deal along a Hilbert curve that
bench.py measured best is what rt_dist_render and examples/render_dist
split a job by, and bench.py / rtnw.blocks_for_rank call the same C function.

CPU only: the layout functions are host code of librt_hip.so (no GPU call)."""
import ctypes

import numpy as np
import pytest

import rtnw

RT_ERR_INVALID = -1   # include/rt_hip.h


def hilbert_index(n, x, y):
    """Position of cell (x, y) on the Hilbert curve over an n x n grid (n a power of 2),
    the quadrant rotation reflecting within the current sub-square."""
    x = np.asarray(x, dtype=np.int64).copy()
    y = np.asarray(y, dtype=np.int64).copy()
    d = np.zeros_like(x)
    s = n // 2
    while s > 0:
        rx = (x & s) > 0
        ry = (y & s) > 0
        d += s * s * ((3 * rx) ^ ry)
        flip = ~ry
        sw = flip & rx
        x = np.where(sw, s - 1 - x, x)
        y = np.where(sw, s - 1 - y, y)
        x, y = np.where(flip, y, x), np.where(flip, x, y)
        s //= 2
    return d


def _block_pixels(nx, ny, x0, y0, block):
    xs = np.arange(x0, min(x0 + block, nx))
    ys = np.arange(y0, min(y0 + block, ny))
    I, J = np.meshgrid(xs, ys, indexing="ij")   # column by column
    return np.stack([I.ravel(), J.ravel()], axis=1)


def _as_tiles(out):
    if not out:
        return np.zeros((0, 4), np.int32)
    xy = np.concatenate(out)
    t = np.ones((xy.shape[0], 4), np.int32)
    t[:, :2] = xy
    return t


def hilbert_blocks_ref(nx, ny, rank, world, block=8):
    bx, by = (nx + block - 1) // block, (ny + block - 1) // block
    n = 1
    while n < max(bx, by):
        n *= 2
    X, Y = np.meshgrid(np.arange(bx), np.arange(by), indexing="xy")
    order = np.argsort(hilbert_index(n, X.ravel(), Y.ravel()), kind="stable")
    return _as_tiles([_block_pixels(nx, ny, int(X.ravel()[k]) * block, int(Y.ravel()[k]) * block, block)
                      for k in order[rank::world]])


def lattice_blocks_ref(nx, ny, rank, world, block=8):
    a, b = rtnw.interleave_factors(world)
    ry, rx = divmod(rank, a)
    bx, by = (nx + block - 1) // block, (ny + block - 1) // block
    return _as_tiles([_block_pixels(nx, ny, xb * block, yb * block, block)
                      for yb in range(ry, by, b) for xb in range(rx, bx, a)])


SIZES = [(1000, 1000), (500, 500), (800, 400), (400, 400), (37, 23), (64, 8), (8, 8), (1, 1), (9, 300)]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_c_block_deal_equals_the_restatement(world):
    """rt_rank_tiles(RT_LAYOUT_BLOCKS) == the numpy Hilbert deal, tile for tile in claim order."""
    for nx, ny in SIZES:
        for r in range(world):
            c = rtnw.blocks_for_rank(nx, ny, r, world)
            assert np.array_equal(c, hilbert_blocks_ref(nx, ny, r, world)), (nx, ny, r, world)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c_block_lattice_equals_the_restatement(world):
    for nx, ny in SIZES:
        for r in range(world):
            c = rtnw.lattice_blocks_for_rank(nx, ny, r, world)
            assert np.array_equal(c, lattice_blocks_ref(nx, ny, r, world)), (nx, ny, r, world)


def test_interleaved_layout_is_rank_pixels():
    for nx, ny in SIZES[:5]:
        for world in (2, 8):
            for r in range(world):
                assert np.array_equal(rtnw.rank_tiles_c(nx, ny, r, world, rtnw.RT_LAYOUT_INTERLEAVED),
                                      rtnw.rank_pixels_c(nx, ny, r, world))


def test_block_sizes_other_than_eight():
    for block in (4, 16):
        for world in (2, 8):
            seen = np.zeros((123, 77), int)
            for r in range(world):
                t = rtnw.blocks_for_rank(77, 123, r, world, block)
                assert np.array_equal(t, hilbert_blocks_ref(77, 123, r, world, block))
                seen[t[:, 1], t[:, 0]] += 1
            assert (seen == 1).all()


def test_hilbert_curve_steps_to_neighbours():
    """Consecutive curve positions are neighbouring cells: the block deal's coherence."""
    for n in (2, 4, 16, 128):
        X, Y = np.meshgrid(np.arange(n), np.arange(n), indexing="xy")
        d = hilbert_index(n, X.ravel(), Y.ravel())
        o = np.argsort(d)
        assert np.array_equal(np.sort(d), np.arange(n * n))
        assert (np.abs(np.diff(X.ravel()[o])) + np.abs(np.diff(Y.ravel()[o])) == 1).all()


def test_rank_tiles_rejects_bad_arguments():
    L = rtnw.lib()
    buf = np.zeros((64, 4), np.int32)
    assert L.rt_rank_tiles(0, 8, 0, 1, 0, 8, None, 0) == RT_ERR_INVALID
    assert L.rt_rank_tiles(8, 8, 2, 2, 0, 8, None, 0) == RT_ERR_INVALID
    assert L.rt_rank_tiles(8, 8, 0, 1, 7, 8, None, 0) == RT_ERR_INVALID       # unknown layout
    assert L.rt_rank_tiles(8, 8, 0, 1, 0, 8, buf.ctypes.data, 63) == RT_ERR_INVALID   # short buffer
    assert L.rt_rank_tiles(8, 8, 0, 1, 0, 0, buf.ctypes.data, 64) == 64       # block 0 -> 8
    assert L.rt_dist_set_layout(None, 0) == RT_ERR_INVALID
