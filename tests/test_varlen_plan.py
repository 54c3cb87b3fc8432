"""CPU checks of the variable-length engine's work decomposition (no GPU):
every byte of every buffer is assigned to exactly one wavefront piece, every
zero-length buffer is visited once, and no lane ever loads a 16-byte chunk
outside the piece it is checksumming.  Mirrors crc32c_varlen.hip via
tests/varlen_model.py."""
import numpy as np
import pytest

import varlen_model as M


@pytest.mark.parametrize("nwave", [1, 7, 64, 4096])
def test_random_batches_cover_exactly_once(nwave):
    rng = np.random.default_rng(nwave)
    n = 3000
    lengths = np.where(rng.random(n) < 0.7, rng.integers(0, 3000, n), rng.integers(0, 300_000, n))
    lengths[rng.random(n) < 0.05] = 0
    offsets = rng.integers(0, 1 << 30, n)
    _, errors = M.check_decomposition(lengths, offsets, nwave, check_loads=(nwave <= 64))
    assert not errors, errors[:5]


def test_zipf_like_small_packets():
    rng = np.random.default_rng(1)
    k = rng.choice(np.arange(1, 257), size=5000, p=(1 / np.arange(1, 257)) / (1 / np.arange(1, 257)).sum())
    lengths = np.clip(64 * k - rng.integers(0, 64, k.size), 64, 16384)
    offsets = np.concatenate([[0], np.cumsum((lengths + 255) // 256 * 256)[:-1]])
    _, errors = M.check_decomposition(lengths, offsets + 4096, 64)
    assert not errors, errors[:5]


@pytest.mark.parametrize("length,stride,count", [(4088, 4096, 3000), (77, 100, 20000), (1 << 20, 1 << 20, 40),
                                                 ((1 << 20) - 13, 1 << 20, 40), (33, 33, 5000), (4092, 4100, 999)])
def test_fixed_mode_cover_exactly_once(length, stride, count):
    offsets = np.arange(count, dtype=np.uint64) * stride + 3
    lengths = np.full(count, length, dtype=np.uint64)
    _, errors = M.check_decomposition(lengths, offsets, 4096, fixed=length, check_loads=False)
    assert not errors, errors[:5]


def test_all_empty_and_single_byte():
    lengths = np.array([0] * 100 + [1] * 50 + [0] * 10)
    offsets = np.arange(lengths.size) * 7
    _, errors = M.check_decomposition(lengths, offsets, 4096)
    assert not errors, errors[:5]


def test_window_loads_stay_inside_piece():
    for P0, P1 in [(16, 32), (1, 17), (15, 1039), (4096, 4096 + 1024), (100, 100 + 4095), (7, 7 + 70_000),
                   (4096 * 3 + 5, 4096 * 9 - 3)]:
        for ca in M.loads_for_piece(P0, P1):
            assert ca % 16 == 0 and ca + 16 > P0 and ca < P1
