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


# ---- split route layout (k_xplan / k_xscan / k_xassign, then k_xsplit_a's shares)
SPLIT_MIN, PIECE = 16384, 64


def split_plan(lengths, capD, nwa):
    """Restates the planner's split layout: the buffers over 16 KiB go to the
    split route if all their blocks / pieces / entries fit the room (else
    none does), pieces in buffer order at their flat D
    positions, and phase-A wave w's start (piece << 6 | block) for its share
    [w*pb, (w+1)*pb) of D."""
    capS = capD // 16 + 1 if capD else 0
    capP = capD // PIECE + capS if capD else 0
    n = lengths.size
    lg = lengths > SPLIT_MIN
    nb = np.where(lg, (lengths - 1) // 1024 + 1, 0).astype(np.int64)
    npc = (nb + PIECE - 1) // PIECE
    # every split candidate or none (k_xscan)
    tb_all, tp_all, ts_all = int(nb.sum()), int(npc.sum()), int(lg.sum())
    fits = tb_all == 0 or (capD > 0 and tb_all <= capD and tp_all <= capP and ts_all <= capS)
    split = lg & fits
    nbs = np.where(split, nb, 0)
    F = np.concatenate([[0], np.cumsum(nbs)[:-1]])
    pcs = []  # (buffer, first block, blocks, d)
    for i in np.nonzero(split)[0]:
        for j in range(int(npc[i])):
            b0 = PIECE * j
            pcs.append((int(i), b0, min(PIECE, int(nb[i]) - b0), int(F[i]) + b0))
    tb = int(nbs.sum())
    pb = (tb + nwa - 1) // nwa if nwa else 0
    astart = [None] * nwa
    pstart = 0
    for i in np.nonzero(split)[0]:
        w = (int(F[i]) + pb - 1) // pb
        while w * pb < int(F[i]) + int(nb[i]) and w < nwa:
            off = w * pb - int(F[i])
            astart[w] = (pstart + off // PIECE, off % PIECE)
            w += 1
        pstart += int(npc[i])
    return split, F, pcs, tb, pb, astart


def phase_a_rows(pcs, tb, pb, astart, w):
    """The (buffer, block, D index) rows wave w computes (k_xsplit_a's load cursor)."""
    if astart[w] is None:
        return []
    lq, lpos = astart[w]
    rem = min((w + 1) * pb, tb) - w * pb
    rows = []
    while rem:
        buf, b0, nbk, d = pcs[lq]
        n = min(nbk - lpos, 4, rem)
        rows += [(buf, b0 + lpos + r, d + lpos + r) for r in range(n)]
        lpos += n
        rem -= n
        if lpos >= nbk and rem:
            lq, lpos = lq + 1, 0
    return rows


def test_split_layout_phase_a_shares_cover_d_once():
    rng = np.random.default_rng(17)
    for trial in range(40):
        n = int(rng.integers(1, 2000))
        kind = trial % 4
        if kind == 0:
            lens = np.exp(rng.uniform(np.log(4096), np.log(1 << 20), n)).astype(np.int64)
        elif kind == 1:
            lens = rng.integers(0, 70000, n)
        elif kind == 2:
            lens = np.where(rng.random(n) < 0.02, rng.integers(1 << 20, 8 << 20, n), rng.integers(0, 20000, n))
        else:
            lens = np.full(n, 16385 + int(rng.integers(0, 3000)))
        need = int(np.where(lens > SPLIT_MIN, (lens - 1) // 1024 + 1, 0).sum())
        capD = int(rng.choice([0, max(256, need), max(256, need // 2), 10 ** 9]))
        nwa = int(rng.choice([4, 768, 3072]))
        split, F, pcs, tb, pb, astart = split_plan(lens, capD, nwa)
        assert tb <= max(capD, 0)
        seen = np.zeros(tb, dtype=np.int64)
        for w in range(nwa):
            for buf, blk, d in phase_a_rows(pcs, tb, pb, astart, w):
                assert split[buf] and d == F[buf] + blk and blk <= (lens[buf] - 1) // 1024
                seen[d] += 1
        assert (seen == 1).all(), "a stripe-sum block computed twice or never"
        if capD >= need:
            assert split.sum() == (lens > SPLIT_MIN).sum() or capD == 0
