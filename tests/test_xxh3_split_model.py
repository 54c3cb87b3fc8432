"""CPU checks of the split XXH3 route's arithmetic (tests/xxh3_split_model.py)
against the oracle, which is pinned to the reference's flow/xxhash.c."""
import numpy as np

from oracle import oracle as O
from tests import xxh3_split_model as XS


def _bytes(n, state):
    return O.splitmix64((n + 7) // 8, state).view(np.uint8)[:n].tobytes()


def test_block_sums_and_chain_equal_xxh3():
    data = _bytes(70000, 0x5A17)
    rng = np.random.default_rng(11)
    lengths = [241, 1023, 1024, 1025, 1088, 2047, 2048, 2049, 16384, 16385, 20000, 65536, 65537]
    lengths += [int(x) for x in rng.integers(241, 69000, 12)]
    for L in lengths:
        off = int(rng.integers(0, len(data) - L + 1))
        for seed in (0, 1, 0xFDBEEFDB, 0x9E3779B97F4A7C15):
            buf = data[off:off + L]
            assert XS.xxh3_split(buf, seed) == O.xxh3_64(np.frombuffer(buf, np.uint8), seed), (L, off, seed)


def test_block_sums_are_independent_of_the_chain():
    # the stripe sums of a block depend only on the block's bytes (and the seed)
    data = _bytes(8192, 0x77)
    a = XS.block_sums(data[:5000], 3)
    b = XS.block_sums(data[:8000], 3)
    assert a[:4] == b[:4]


def test_piece_list_covers_every_block_once():
    rng = np.random.default_rng(5)
    lengths = [int(x) for x in rng.integers(0, 300000, 200)] + [16384, 16385, 65536 * 3 + 1]
    split, pcs, total = XS.pieces(lengths, 16384)
    seen = {}
    for s, b0, nb in pcs:
        i, F = split[s]
        nbk = ((lengths[i] - 1) >> 10) + 1
        assert 0 < nb <= 64 and b0 + nb <= nbk
        for b in range(b0, b0 + nb):
            assert (F + b) not in seen
            seen[F + b] = (i, b)
    assert len(seen) == total
    assert all(lengths[i] > 16384 for i, _ in split)
    assert sum(((L - 1) >> 10) + 1 for L in lengths if L > 16384) == total
