"""CPU checks of the variable-length engine's work decomposition (no GPU):
every slot belongs to exactly one wavefront, the chunks a buffer's windows
checksum tile its 16-byte span exactly once, and no lane ever loads a 16-byte
chunk that does not overlap its buffer.  Mirrors crc32c_varlen.hip (v7) via
tests/varlen_model.py."""
import numpy as np
import pytest

import varlen_model as M


@pytest.mark.parametrize("nwave", [1, 7, 64, 3072])
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
    _, errors = M.check_decomposition(lengths, offsets, 3072, check_loads=False)
    assert not errors, errors[:5]


def test_all_empty_and_single_byte():
    lengths = np.array([0] * 100 + [1] * 50 + [0] * 10)
    offsets = np.arange(lengths.size) * 7
    _, errors = M.check_decomposition(lengths, offsets, 3072)
    assert not errors, errors[:5]


def test_every_alignment_and_threshold_length():
    """All 16 start alignments x lengths around the small-buffer span, the
    1 KiB window and 4 KiB pass geometry."""
    lens = [16, 17, 100, 112, 113, 127, 128, 129, 1007, 1008, 1009, 1023, 1024, 1025, 2047, 4095, 4096, 4097, 12289]
    offs, lengths = [], []
    for a in range(16):
        for n in lens:
            offs.append(1 << 20 | a)
            lengths.append(n)
    cover, errors = M.check_decomposition(lengths, offs, 64)
    assert not errors, errors[:5]
    # buffers spanning more than SMALL_SPAN bytes are windowed, the rest finish in prep
    for i, (o, n) in enumerate(zip(offs, lengths)):
        A, E, W, _, _, _ = M.geo7(o, n)
        assert (W > 0) == (E - A > M.SMALL_SPAN), (o, n)


def test_tail_term_identity():
    """The window kernel does not mask the zt < 16 bytes after a buffer's end;
    prep cancels them with T = chain(0, garbage) * x^(-8 zt), written as out[]'s
    initial value (crc32c_varlen.hip, v7prep).  Checked here in the forward
    form on the C oracle: chain(r, B || G) = chain(r, B) * x^(8 zt) ^ chain(0, G),
    so (chain(r, B || G) ^ T * x^(8 zt)) * x^(-8 zt) = chain(r, B), and
    ~chain(r, B) is crc32c_append's result (crc32c.cpp:197, 310)."""
    from oracle import oracle as O
    rng = np.random.default_rng(7)

    def chain(reg, data):  # raw register after feeding data into reg
        return (~O.crc32c(~reg & 0xFFFFFFFF, bytes(data))) & 0xFFFFFFFF

    for _ in range(200):
        n = int(rng.integers(16, 300))
        zt = int(rng.integers(1, 16))
        buf = rng.integers(0, 256, n + zt, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        body, garbage = buf[:n], buf[n:]
        r0 = ~seed & 0xFFFFFFFF
        unmasked = chain(r0, body + garbage)        # what the window kernel's chains hold at E
        t_fwd = chain(0, garbage)                  # T * x^(8 zt): leading zeros of the chunk are free
        assert t_fwd == chain(0, bytes(16 - zt) + garbage)
        assert unmasked ^ t_fwd == O.shift(chain(r0, body), zt)
        assert (~chain(r0, body)) & 0xFFFFFFFF == O.crc32c(seed, body)
