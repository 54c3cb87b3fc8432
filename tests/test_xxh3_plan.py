"""CPU model of the XXH3 varlen planner (k_xplan / k_xscan / k_xassign in
foundationdb_amd/csrc/xxh3_kernels.hip): every wave w must get as its first
buffer the first buffer whose start (in cost units, length + 64 per buffer)
is >= w*Q, and the last entry must be `count`."""
import numpy as np


def plan(lengths, nwave):
    cost = lengths.astype(np.uint64) + 64
    start = np.concatenate([[0], np.cumsum(cost)[:-1]]).astype(np.uint64)
    total = int(cost.sum())
    q = (total + nwave - 1) // nwave
    wf = np.full(nwave + 1, -1, dtype=np.int64)
    n = lengths.size
    for i in range(n):  # one thread per buffer, as in k_xassign
        s = int(start[i])
        prev = 0 if i == 0 else s - int(lengths[i - 1] + 64)
        w_lo = 0 if i == 0 else prev // q + 1
        for w in range(w_lo, min(s // q, nwave - 1) + 1):
            wf[w] = i
        if i + 1 == n:
            for w in range(s // q + 1, nwave + 1):
                wf[w] = n
    return wf, start, q


def expected(start, q, nwave, n):
    wf = np.empty(nwave + 1, dtype=np.int64)
    for w in range(nwave + 1):
        wf[w] = int(np.searchsorted(start, w * q, side="left")) if w < nwave else n
    return wf


def test_planner_covers_every_wave():
    rng = np.random.default_rng(3)
    for trial in range(60):
        n = int(rng.integers(1, 3000))
        kind = trial % 4
        if kind == 0:
            lens = rng.integers(0, 300, n)
        elif kind == 1:
            lens = rng.integers(0, 40000, n)
        elif kind == 2:
            lens = np.where(rng.random(n) < 0.05, rng.integers(1 << 16, 1 << 20, n), rng.integers(0, 100, n))
        else:
            lens = np.zeros(n, dtype=np.int64)
        nwave = int(rng.choice([64, 1024, 5120]))
        wf, start, q = plan(lens, nwave)
        assert (wf >= 0).all(), "unassigned wave"
        assert np.array_equal(wf, expected(start, q, nwave, n))
        assert (np.diff(wf) >= 0).all() and wf[-1] == n
