"""CPU model of k_xstream's SCHEDULE (crc32c_extent.hip), symbolic: which
wave captures which point, from which block and lane span, and which blocks
each wave folds into its range prefix.  Lane prefixes are represented by their
(block, lane) coordinates, so the model checks the control flow -- static
ranges of whole units, the window search, window retirement inside a unit,
the extent's last block, the ownership of points at range boundaries --
without any CRC arithmetic (tests/extent_model.py checks that)."""

U = 2  # blocks per unit (kXU); an iteration is two units


def x_blk(p):
    return (p - 1) >> 12 if p else 0


def x_cnt(p, k):
    return (p - 4096 * k) >> 6 if p else 0


def schedule(P0, P1, nwave):
    """P0/P1: absolute starts/ends of a packed batch.  Returns (vs, ve, blk):
    vs[i] / ve[i] = list of (wave, value) writes, value = None (0) or the
    (block, lane) whose prefix was captured; blk[k] = list of waves that
    folded block k's register into its range's prefix X."""
    n = len(P0)
    S = P0[0] & ~15
    Eend = (P1[-1] + 15) & ~15
    nblk = (Eend - S + 4095) >> 12
    per = -(-(-(-nblk // nwave)) // (2 * U)) * (2 * U)
    vs = [[] for _ in range(n)]
    ve = [[] for _ in range(n)]
    blk = [[] for _ in range(nblk)]
    for w in range(nwave):
        k0 = min(w * per, nblk)
        k1 = min(k0 + per, nblk)
        km = min(k1, nblk - 1)
        T0 = S + 4096 * k0
        q = sum(1 for b in P1 if b <= T0)  # first buffer ending past the range's start
        win = {}

        def make_window(q0):
            nonlocal win
            win = {"q": q0, "bs": [], "be": [], "cs": [], "ce": [], "Vs": [0] * 64, "Ve": [0] * 64}
            for j in range(64):
                if q0 + j < n:
                    s, e = P0[q0 + j] - S, P1[q0 + j] - S
                    win["bs"].append(x_blk(s)); win["be"].append(x_blk(e))
                    win["cs"].append(x_cnt(s, x_blk(s))); win["ce"].append(x_cnt(e, x_blk(e)))
                else:
                    win["bs"].append(-2); win["be"].append(-2); win["cs"].append(0); win["ce"].append(0)
            win["last"] = win["be"][63] if q0 + 64 <= n else float("inf")

        def flush():
            q0 = win["q"]
            for j in range(64):
                if q0 + j >= n:
                    continue
                if k0 <= win["bs"][j] < k1:
                    vs[q0 + j].append((w, win["Vs"][j]))
                if k0 <= win["be"][j] < k1:
                    ve[q0 + j].append((w, win["Ve"][j]))

        def capture(kb, valid):
            for j in range(64):
                if valid and win["bs"][j] == kb:
                    c = win["cs"][j]
                    win["Vs"][j] = (kb, c - 1) if c else 0
                if valid and win["be"][j] == kb:
                    c = win["ce"][j]
                    win["Ve"][j] = (kb, c - 1) if c else 0

        def finish(k, kend):
            for j in range(2 * U):
                if k + j < kend:  # X = X * M ^ B[k + j]
                    blk[k + j].append(w)
            for j in range(2 * U):
                capture(k + j, k + j < kend)
            kn = min(k + 2 * U, kend)
            while win["last"] < kn:
                flush()
                make_window(win["q"] + 64)
                for j in range(2 * U):
                    capture(k + j, k + j < kend)

        make_window(q)
        if k0 >= k1:
            continue
        k = k0
        while k < km:
            finish(k, km)
            k += 2 * U
        if km < k1:
            finish(km, k1)
        flush()
    return vs, ve, blk, S, nblk


def grab_map(P0, P1, gsz):
    """k_v7count's wq[]: per grab, the first buffer ending past its start."""
    S = P0[0] & ~15
    Eend = (P1[-1] + 15) & ~15
    nblk = (Eend - S + 4095) >> 12
    ngrab = -(-nblk // gsz)
    tg = 4096 * gsz
    wq = [None] * ngrab
    for i in range(len(P0)):
        ep = P1[i - 1] - S if i else 0
        ei = P1[i] - S
        lo = -(-ep // tg) if i else 0
        hi = ngrab if i + 1 == len(P0) else -(-ei // tg)
        for g in range(lo, min(hi, ngrab)):
            wq[g] = i
    return wq, S, nblk, ngrab


def schedule_grabs(P0, P1, gsz, order):
    """k_xgrab's control flow: grab g (gsz blocks) is processed from a window
    starting at wq[g], in steps of 4 blocks, retiring windows inside the grab
    and flushing only the points of the grab's blocks.  `order` is the
    sequence in which grabs are processed (any order: they are independent).
    Returns (vs, ve, blk) as schedule() does, blk[k] = grabs that folded block k."""
    n = len(P0)
    wq, S, nblk, ngrab = grab_map(P0, P1, gsz)
    assert all(v is not None for v in wq), "every grab has its first buffer"
    vs = [[] for _ in range(n)]
    ve = [[] for _ in range(n)]
    blk = [[] for _ in range(nblk)]
    for g in order:
        gb0, gb1 = g * gsz, min(g * gsz + gsz, nblk)
        win = {}

        def make_window(q0):
            win.clear()
            win.update({"q": q0, "bs": [], "be": [], "cs": [], "ce": [], "Vs": [0] * 64, "Ve": [0] * 64})
            for j in range(64):
                if q0 + j < n:
                    s, e = P0[q0 + j] - S, P1[q0 + j] - S
                    win["bs"].append(x_blk(s)); win["be"].append(x_blk(e))
                    win["cs"].append(x_cnt(s, x_blk(s))); win["ce"].append(x_cnt(e, x_blk(e)))
                else:
                    win["bs"].append(-2); win["be"].append(-2); win["cs"].append(0); win["ce"].append(0)
            win["last"] = win["be"][63] if q0 + 64 <= n else float("inf")

        def flush():
            q0 = win["q"]
            for j in range(64):
                if q0 + j >= n:
                    continue
                if gb0 <= win["bs"][j] < gb1:
                    vs[q0 + j].append((g, win["Vs"][j]))
                if gb0 <= win["be"][j] < gb1:
                    ve[q0 + j].append((g, win["Ve"][j]))

        def capture(kb, valid):
            for j in range(64):
                if valid and win["bs"][j] == kb:
                    c = win["cs"][j]
                    win["Vs"][j] = (kb, c - 1) if c else 0
                if valid and win["be"][j] == kb:
                    c = win["ce"][j]
                    win["Ve"][j] = (kb, c - 1) if c else 0

        make_window(wq[g])
        for k in range(gb0, gb1, 4):
            for j in range(4):
                if k + j < gb1:
                    blk[k + j].append(g)
            for j in range(4):
                capture(k + j, k + j < gb1)
            kn = min(k + 4, gb1)
            while win["last"] < kn:
                flush()
                make_window(win["q"] + 64)
                for j in range(4):
                    capture(k + j, k + j < gb1)
        flush()
    return vs, ve, blk, S, nblk


def finish_plan(P0, P1, gsz, grid):
    """Who finishes each buffer on the fused route (crc32c_extent.hip:
    xgf_finish, x_shared_of), symbolic.  Workgroup b owns grabs [g0, g1)
    (b * gper, clamped to nd = the last grab, which workgroup 0 streams).
    k_xgf: each workgroup finishes the buffers whose end grab is its own --
    [wq[g0], wq[g1]), buffer 0 from grab 0, and in workgroup 0 the last
    grab's [wq[nd], n) -- except the first of a list when it starts in
    another workgroup's grabs; k_xshared finishes those (x_shared_of).
    Returns (fin, owners): fin[i] = list of ("own", b) / ("shared", b)
    records, owners[i] = the workgroups holding buffer i's grabs."""
    n = len(P0)
    wq, S, nblk, ngrab = grab_map(P0, P1, gsz)
    nd = ngrab - 1
    gper = -(-nd // grid) if nd else 0

    def grab(p):
        return x_blk(p) // gsz

    def owner(g):
        return 0 if g >= nd else g // gper

    def rng(b):
        g0 = min(b * gper, nd)
        return g0, min(g0 + gper, nd)

    owners = [{owner(g) for g in range(grab(P0[i] - S), grab(P1[i] - S) + 1)} for i in range(n)]
    fin = [[] for _ in range(n)]
    for b in range(grid):  # k_xgf: own buffers
        g0, g1 = rng(b)
        lo = 0 if g0 == 0 else wq[g0]
        hi = wq[g1] if g0 < g1 else lo
        sh1 = lo < hi and g0 != 0 and owner(grab(P0[lo] - S)) != b
        for i in range(lo + (1 if sh1 else 0), hi):
            fin[i].append(("own", b))
        if b == 0:
            c = 0 if nd == 0 else wq[nd]
            b0 = c + (1 if c < n and nd != 0 and grab(P0[c] - S) < nd else 0)
            for i in range(b0, n):
                fin[i].append(("own", b))
    for b in range(grid + 1):  # k_xshared: x_shared_of(b)
        if b < grid:
            g0, g1 = rng(b)
            if g0 == 0 or g0 >= g1:
                continue
            lo, hi = wq[g0], wq[g1]
            if lo < hi and owner(grab(P0[lo] - S)) != b:
                fin[lo].append(("shared", b))
        elif nd:
            c = wq[nd]
            if c < n and grab(P0[c] - S) < nd:
                fin[c].append(("shared", b))
    return fin, owners
