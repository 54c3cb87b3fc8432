"""The extent route's arithmetic (tests/extent_model.py) against the oracle on
small packed batches: packets back to back with gaps, any alignment, zero
lengths, points on block and lane boundaries, the extent's first and last
bytes.  CPU only."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import extent_model as X


def sm(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


@pytest.mark.parametrize("case", range(6))
def test_extent_model_matches_oracle(case):
    rng = np.random.default_rng(case)
    mem = sm(1 << 16, 0xE7 + case)
    lens, offs, pos = [], [], int(rng.integers(0, 40))
    while True:
        L = int(rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 200, 1000, 4095, 4096, 4097, 9000]) if case % 2
                else rng.integers(1, 5000))
        g = int(rng.integers(0, min(max(L, 256), 300)))
        if pos + L > mem.size - 64:
            break
        offs.append(pos)
        lens.append(L)
        pos += L + g
    if case == 4:  # points exactly on lane / block boundaries, starting at byte 0
        offs, lens, pos = [], [], 0
        for L in (64, 4032, 4096, 64, 1, 8191, 4096):
            offs.append(pos)
            lens.append(L)
            pos += L
    for seed in (0, 0xFDBEEFDB):
        got = X.extent_crcs(mem, offs, lens, seed)
        want = O.batch_varlen(mem, np.array(offs, np.uint64), np.array(lens, np.uint64), seed=seed)
        assert np.array_equal(got, want), case
        # the range-local form (per-wave prefixes, a scan over waves only)
        for nwave in (1, 2, 5):
            got = X.extent_crcs_ranges(mem, offs, lens, seed, nwave)
            assert np.array_equal(got, want), (case, nwave)


def test_eligibility_rule():
    assert X.eligible([0, 100], [100, 200])
    assert not X.eligible([0, 50], [100, 150])          # overlap
    assert not X.eligible([100, 0], [200, 100])         # descending
    assert X.eligible([0, 300], [64, 400])              # gap 236 <= 256
    assert not X.eligible([0, 1000], [64, 1100])        # gap 936 > max(64, 256)
    assert X.eligible([0, 9000], [5000, 9100])          # gap 4000 <= len 5000
    assert not X.eligible([0, 20000], [10000, 20100])   # gap 10000 >= 4096


def _check_schedule(P0, P1, nwave):
    from tests import extent_sched_model as M
    vs, ve, blk, S, nblk = M.schedule(P0, P1, nwave)
    assert all(len(b) == 1 for b in blk), "every block folded into its range prefix exactly once"
    for i, (a, b) in enumerate(zip(P0, P1)):
        for p, rec in ((a - S, vs[i]), (b - S, ve[i])):
            k = M.x_blk(p)
            c = M.x_cnt(p, k)
            want = (k, c - 1) if c else 0
            if p == 0:
                assert len(rec) <= 1 and all(v == 0 for _, v in rec)
                continue
            assert len(rec) == 1, (i, p, rec)
            assert rec[0][1] == want, (i, p, rec, want)


@pytest.mark.parametrize("nwave", [1, 3, 7, 64])
def test_stream_schedule_captures_every_point_once(nwave):
    """k_xstream's control flow (static unit ranges, window search and
    retirement, the extent's last block): every point is captured exactly
    once, by the wave whose range holds its block, from the right block and
    lane span; every block is folded into its range prefix exactly once."""
    rng = np.random.default_rng(nwave)
    for trial in range(12):
        P0, P1, pos = [], [], int(rng.integers(0, 4096))
        n = int(rng.integers(1, 600))
        kind = trial % 4
        for _ in range(n):
            L = int({0: rng.integers(1, 300), 1: rng.integers(0, 20000), 2: rng.choice([0, 1, 63, 64, 65, 4096]),
                     3: rng.integers(2000, 70000)}[kind])
            g = int(rng.integers(0, min(max(L, 256), 4095) + 1)) if trial % 3 else 0
            P0.append(pos)
            P1.append(pos + L)
            pos += L + g
        _check_schedule(P0, P1, nwave)
    # single buffers, aligned and not; a batch inside one block
    _check_schedule([0], [1 << 20], nwave)
    _check_schedule([5], [5 + 4091], nwave)
    _check_schedule([16, 100], [50, 4000], nwave)


def test_stream_schedule_window_retired_before_the_last_block():
    """A window whose last buffer ends in the extent's last block, reached by a
    partial iteration of the main loop: the window must not retire before the
    last block's points are captured (the retire bound is the iteration's last
    block before kend, not the iteration's end)."""
    for nblk_tail in range(1, 9):
        # 64-buffer windows of tiny packets filling the extent up to its last block
        P0, P1, pos = [], [], 0
        target = 4096 * (4 + nblk_tail) - 40
        while pos < target:
            P0.append(pos)
            P1.append(pos + 48)
            pos += 64
        for nwave in (1, 2, 3):
            _check_schedule(P0, P1, nwave)


@pytest.mark.parametrize("nwave", [1, 2, 3])
def test_range_form_across_block_groups(nwave):
    """Ranges of more than 64 blocks (several lane-parallel groups per range,
    the carry between them) and buffers straddling ranges."""
    rng = np.random.default_rng(40 + nwave)
    mem = sm(700 << 10, 0x9A + nwave)
    offs, lens, pos = [], [], 5
    while True:
        L = int(rng.integers(0, 30000)) if rng.random() < 0.8 else int(rng.integers(60000, 200000))
        if pos + L > mem.size - 64:
            break
        offs.append(pos)
        lens.append(L)
        pos += L + int(rng.integers(0, min(max(L, 256), 4095) + 1))
    want = O.batch_varlen(mem, np.array(offs, np.uint64), np.array(lens, np.uint64), seed=7)
    got = X.extent_crcs_ranges(mem, offs, lens, 7, nwave)
    assert np.array_equal(got, want)


def _check_grabs(P0, P1, gsz, rng):
    from tests import extent_sched_model as M
    wq, S, nblk, ngrab = M.grab_map(P0, P1, gsz)
    order = list(rng.permutation(ngrab))
    vs, ve, blk, S, nblk = M.schedule_grabs(P0, P1, gsz, order)
    assert all(len(b) == 1 for b in blk), "every block folded into its grab's prefix exactly once"
    for i, (a, b) in enumerate(zip(P0, P1)):
        for p, rec in ((a - S, vs[i]), (b - S, ve[i])):
            k = M.x_blk(p)
            c = M.x_cnt(p, k)
            want = (k, c - 1) if c else 0
            if p == 0:
                assert len(rec) <= 1 and all(v == 0 for _, v in rec)
                continue
            assert len(rec) == 1, (i, p, rec)
            assert rec[0][1] == want, (i, p, rec, want)
            assert rec[0][0] == k // gsz


@pytest.mark.parametrize("gsz", [8, 16, 24])
def test_grab_schedule_captures_every_point_once(gsz):
    """k_xgrab's control flow (grabs in any order, each from the window
    k_v7count's grab map gives it, windows retired inside a grab, only the
    grab's points flushed): every point is captured exactly once, by its
    block's grab, from the right block and lane span."""
    rng = np.random.default_rng(gsz)
    for trial in range(12):
        P0, P1, pos = [], [], int(rng.integers(0, 4096))
        n = int(rng.integers(1, 600))
        kind = trial % 4
        for _ in range(n):
            L = int({0: rng.integers(1, 300), 1: rng.integers(0, 20000), 2: rng.choice([0, 1, 63, 64, 65, 4096]),
                     3: rng.integers(2000, 70000)}[kind])
            g = int(rng.integers(0, min(max(L, 256), 4095) + 1)) if trial % 3 else 0
            P0.append(pos)
            P1.append(pos + L)
            pos += L + g
        _check_grabs(P0, P1, gsz, rng)
    _check_grabs([0], [1 << 20], gsz, rng)
    _check_grabs([5], [5 + 4091], gsz, rng)
    _check_grabs([16, 100], [50, 4000], gsz, rng)


@pytest.mark.parametrize("gsz", [8, 16])
def test_grab_form_matches_oracle(gsz):
    """The grab form's arithmetic: per = gsz blocks chained by the finishing
    pass (straddling buffers: Horner over the grab aggregates)."""
    rng = np.random.default_rng(70 + gsz)
    mem = sm(900 << 10, 0x6A + gsz)
    offs, lens, pos = [], [], 3
    while True:
        L = int(rng.integers(0, 30000)) if rng.random() < 0.8 else int(rng.integers(60000, 300000))
        if pos + L > mem.size - 64:
            break
        offs.append(pos)
        lens.append(L)
        pos += L + int(rng.integers(0, min(max(L, 256), 4095) + 1))
    want = O.batch_varlen(mem, np.array(offs, np.uint64), np.array(lens, np.uint64), seed=11)
    got = X.extent_crcs_ranges(mem, offs, lens, 11, None, per=gsz)
    assert np.array_equal(got, want)


def _check_finish(P0, P1, gsz, grid):
    from tests import extent_sched_model as M
    fin, owners = M.finish_plan(P0, P1, gsz, grid)
    for i, f in enumerate(fin):
        assert len(f) == 1, ("every buffer finished exactly once", i, f, owners[i])
        kind, b = f[0]
        if kind == "own":  # k_xgf: only what its own grabs hold
            assert owners[i] == {b}, (i, b, owners[i])
        else:  # k_xshared: the buffers whose grabs several workgroups hold
            assert len(owners[i]) > 1 or (b == grid and owners[i] == {0}), (i, b, owners[i])


@pytest.mark.parametrize("grid", [1, 3, 8, 64])
def test_fused_route_finishes_every_buffer_once(grid):
    """k_xgf + k_xshared (crc32c_extent.hip): every buffer of a packed batch
    is finished exactly once -- by the workgroup whose grabs hold all of its
    points and the aggregates between them, inside k_xgf, or, when its grabs
    belong to several workgroups (range boundaries, long buffers over many
    ranges, the extent's last grab), by k_xshared after the kernel boundary."""
    rng = np.random.default_rng(500 + grid)
    for trial in range(10):
        P0, P1, pos = [], [], int(rng.integers(0, 4096))
        n = int(rng.integers(1, 500))
        kind = trial % 5
        for _ in range(n):
            L = int({0: rng.integers(1, 3000), 1: rng.integers(0, 20000), 2: rng.choice([0, 1, 64, 4096, 32768]),
                     3: rng.integers(2000, 70000), 4: rng.choice([100, 300000])}[kind])
            g = int(rng.integers(0, min(max(L, 256), 4095) + 1)) if trial % 3 else 0
            P0.append(pos)
            P1.append(pos + L)
            pos += L + g
        for gsz in (8, 16):
            _check_finish(P0, P1, gsz, grid)
    _check_finish([0], [1 << 22], 8, grid)
    _check_finish([0, 0], [0, 5], 8, grid)
    _check_finish([7], [7], 8, grid)
