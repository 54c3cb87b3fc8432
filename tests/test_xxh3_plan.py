"""CPU model of the XXH3 varlen planner (k_xplan / k_xscan / k_xassign in
foundationdb_amd/csrc/xxh3_kernels.hip): every wave w must get as its first
buffer the first buffer whose start (in cost units) is >= B(w), and the last
entry must be `count`.  A buffer's cost is its length + 64, or a flat 1152
for one of at most 1 KiB (xp_cost).  B(w) = w * qa for the `older` first
waves (the first-dispatched workgroups'), then qb per wave, qa = qb * 21 / 16
(xquant); older = 0 is the uniform split."""
import numpy as np

OLDER_W = 21  # kXOlderW (sixteenths)
TAIL_COST, QUAD_MAX = 1152, 1024  # kXTailCost, kXQuadMax


def xp_cost(lengths):
    """Row buffers: length + 64; short and quad ones (<= 1 KiB): a flat TAIL_COST."""
    lengths = lengths.astype(np.uint64)
    return np.where(lengths <= QUAD_MAX, np.uint64(TAIL_COST), lengths + np.uint64(64)).astype(np.uint64)


def xquant(total, nwave, older):
    if older == 0 or older >= nwave:
        q = max((total + nwave - 1) // nwave, 1)
        return q, q, 0
    den = 16 * (nwave - older) + OLDER_W * older
    qb = max((16 * total + den - 1) // den, 1)
    return (qb * OLDER_W + 15) // 16, qb, older


def xquant_wave(W, x):
    qa, qb, h = W
    return x // qa if x < h * qa else h + (x - h * qa) // qb


def boundary(W, w):
    qa, qb, h = W
    return w * qa if w <= h else h * qa + (w - h) * qb


def plan(lengths, nwave, older=0):
    cost = xp_cost(lengths)
    start = np.concatenate([[0], np.cumsum(cost)[:-1]]).astype(np.uint64)
    total = int(cost.sum())
    W = xquant(total, nwave, older)
    wf = np.full(nwave + 1, -1, dtype=np.int64)
    n = lengths.size
    for i in range(n):  # one thread per buffer, as in k_xassign
        s = int(start[i])
        prev = 0 if i == 0 else s - int(cost[i - 1])
        w_lo = 0 if i == 0 else xquant_wave(W, prev) + 1
        w_hi = xquant_wave(W, s)
        for w in range(w_lo, min(w_hi, nwave - 1) + 1):
            wf[w] = i
        if i + 1 == n:
            for w in range(w_hi + 1, nwave + 1):
                wf[w] = n
    return wf, start, W


def expected(start, W, nwave, n):
    wf = np.empty(nwave + 1, dtype=np.int64)
    for w in range(nwave + 1):
        wf[w] = int(np.searchsorted(start, boundary(W, w), side="left")) if w < nwave else n
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
        older = nwave // 2 if trial % 2 else 0
        wf, start, W = plan(lens, nwave, older)
        assert (wf >= 0).all(), "unassigned wave"
        assert np.array_equal(wf, expected(start, W, nwave, n))
        assert (np.diff(wf) >= 0).all() and wf[-1] == n
        # the boundaries cover the whole cost range: the last wave's start is within the total
        assert boundary(W, nwave) >= int(start[-1]) if n else True


def test_older_waves_get_longer_ranges():
    """With two workgroup generations the first half of the waves gets 21/16
    of the second half's cost each (so both end together on the GPU)."""
    lens = np.full(200000, 5000)
    wf, start, W = plan(lens, 2048, 1024)
    per = np.diff(wf)[:-1]
    a, b = per[:1024].mean(), per[1024:2047].mean()
    assert abs(a / b - 21 / 16) < 0.02


# ---- long-buffer route (k_xplan / k_xscan / k_xassign, then k_xlong's order)
SPLIT_MIN, NCLASS = 16384, 16


def size_class(nb):
    """xp_class: 0 for 2^19 blocks or more, then one per power of two down to 15."""
    lg = int(nb).bit_length() - 1
    return 0 if lg >= 19 else 19 - max(lg, 4)


def long_plan(lengths, capS):
    """Restates the planner's long route: every buffer over 16 KiB or none
    (the entries must fit the room), entries grouped by size class, largest
    class first, and the row kernel's costs with the routed buffers at 64."""
    lg = lengths > SPLIT_MIN
    nlong = int(lg.sum())
    routed = nlong != 0 and capS > 0 and nlong <= capS
    cls = [size_class((int(x) - 1) // 1024 + 1) if l else -1 for x, l in zip(lengths, lg)]
    order = sorted((i for i in range(lengths.size) if routed and lg[i]), key=lambda i: cls[i])
    cost = np.where(lg & routed, 64, lengths + 64)
    return routed, order, cost, cls


def test_long_route_entries_by_size_class():
    rng = np.random.default_rng(17)
    for trial in range(40):
        n = int(rng.integers(1, 3000))
        kind = trial % 4
        if kind == 0:
            lens = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), n)).astype(np.int64)
        elif kind == 1:
            lens = rng.integers(0, 70000, n)
        elif kind == 2:
            lens = np.where(rng.random(n) < 0.02, rng.integers(1 << 20, 8 << 20, n), rng.integers(0, 20000, n))
        else:
            lens = np.full(n, 16385 + int(rng.integers(0, 3000)))
        nlong = int((lens > SPLIT_MIN).sum())
        capS = int(rng.choice([0, nlong, max(1, nlong // 2), 10 ** 9]))
        routed, order, cost, cls = long_plan(lens, capS)
        if routed:
            assert sorted(order) == list(np.nonzero(lens > SPLIT_MIN)[0])
            assert [cls[i] for i in order] == sorted(cls[i] for i in order)
            # a class's buffers are within a factor of two of each other (largest first)
            blocks = [(int(lens[i]) - 1) // 1024 + 1 for i in order]
            for a, b in zip(blocks, blocks[1:]):
                assert b < 2 * a or cls[order[0]] == 0
        else:
            assert order == [] and (cost == lens + 64).all()
        # the row kernel's waves still cover every buffer (the cost model above)
        wf, start, W = plan(np.where(cost == 64, 0, cost - 64), 64)
        assert (wf >= 0).all() and wf[-1] == n
