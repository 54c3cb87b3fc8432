"""CPU checks of the big-buffer block route's decomposition (no GPU): every
4 KiB block of every routed buffer is checksummed exactly once, by whichever
wave grabs it, with the address, index from the buffer's end, first-block lead
(lo, k0) and trailing gap the kernel needs, no load leaves the buffer's
16-byte-rounded span, and a wave's window of route entries only moves forward.
Mirrors crc32c_varlen.hip (prep) and crc32c_kernels.hip (k_bigblocks) via
tests/block_route_model.py."""
import numpy as np
import pytest

import block_route_model as M


@pytest.mark.parametrize("grid", [1, 3, 16, 256])
def test_chunk_like_batches_cover_exactly_once(grid):
    rng = np.random.default_rng(grid)
    n = 300
    lengths = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), n)).astype(np.int64)
    offsets = rng.integers(0, 1 << 30, n)
    _, errors = M.simulate(offsets, lengths, 4096, grid, rng=rng, check_loads=(grid <= 16))
    assert not errors, errors[:5]


@pytest.mark.parametrize("bigmin", [4096, M.SMALL_SPAN + 1])
def test_mixed_batches_and_block_only_route(bigmin):
    """Blocks-only route (bigmin 129: every windowed span, one-block buffers
    with large leads) and the both-routes threshold, on mixed sizes, unaligned
    starts, empty and tiny buffers, and grabs that straddle many buffers."""
    rng = np.random.default_rng(bigmin)
    n = 2500
    lengths = np.where(rng.random(n) < 0.6, rng.integers(0, 6000, n), rng.integers(6000, 200000, n))
    offsets = rng.integers(0, 1 << 28, n)
    _, errors = M.simulate(offsets, lengths, bigmin, 64, rng=rng, check_loads=False)
    assert not errors, errors[:5]


def test_every_lead_and_trailing_gap():
    """Every start mod 16 x span mod 4096 in 16-byte steps around the block
    boundaries, checked with the loads."""
    offs, lens = [], []
    for k0 in range(16):
        for extra in (0, 16, 1008, 2032, 4064, 4080):
            for t in (0, 5, 15):
                offs.append((1 << 24) * (len(offs) + 1) + k0)
                lens.append(3 * 4096 + extra - k0 - t)
    _, errors = M.simulate(np.array(offs), np.array(lens), 4096, 7, rng=np.random.default_rng(3))
    assert not errors, errors[:5]


def test_thousands_of_entries_refill_windows():
    """Many small routed buffers per workgroup: windows refill as grabs move
    past them; the 64-ary entry search needs three levels."""
    rng = np.random.default_rng(9)
    n = 6000
    lengths = rng.integers(4096, 9000, n)
    offsets = np.concatenate([[5], 5 + np.cumsum(lengths + 64)[:-1]])
    visits, errors = M.simulate(offsets, lengths, 4096, 8, rng=rng, check_loads=False)
    assert not errors, errors[:5]
    assert visits.size == sum(M.geo((1 << 32) + int(o), int(n_), 4096)[3] for o, n_ in zip(offsets, lengths))


def test_no_routed_buffers_and_single_block_batches():
    _, errors = M.simulate(np.array([0, 100]), np.array([10, 4000]), 4096, 4)
    assert not errors
    for n in (1, 2, 3, 5):  # total blocks not a multiple of the 4-block grab
        _, errors = M.simulate(np.arange(n) * 8192 + 3, np.full(n, 4096), 4096, 2)
        assert not errors, (n, errors[:3])
