"""CPU model of the big-buffer block route's work decomposition (no GPU).

Restates, in plain Python, the indexing of crc32c_varlen.hip (prep: which
buffers are routed and their entries) and crc32c_kernels.hip (k_bigblocks:
grab ranges per workgroup, dynamic grabs, the per-wave window of route
entries, meta_of's one-lookup and per-block paths, the clamp of blocks past the
batch), so tests can check on the CPU that every block of every routed buffer
is checksummed exactly once, with the right address, index from the end, lead
and tail geometry, and that no load leaves its buffer's 16-byte-rounded span.
"""
import numpy as np

BLOCK = 4096
SMALL_SPAN = 128
BIG_MAX = 1 << 40


def geo(p0, length, bigmin):
    """(A, E, span, nb, lo, k0, t) of buffer [p0, p0 + length) -- geo7()."""
    a = p0 & ~15
    e = (p0 + length + 15) & ~15
    span = e - a
    big = bigmin and length >= 16 and span >= bigmin and span < BIG_MAX
    nb = (span + BLOCK - 1) // BLOCK if big else 0
    lo = BLOCK * nb - span if big else 0
    return a, e, span, nb, lo, p0 & 15, e - (p0 + length)


def entries(offsets, lengths, bigmin, base=1 << 32):
    """The route's entry list in buffer order: es (first block), eE, eidx,
    lo, k0, t -- what k_v7prep writes -- and the total block count."""
    es, ee, ix, lot = [], [], [], []
    s = 0
    for i, (o, n) in enumerate(zip(offsets, lengths)):
        a, e, span, nb, lo, k0, t = geo(base + int(o), int(n), bigmin)
        if nb:
            es.append(s)
            ee.append(e)
            ix.append(i)
            lot.append((lo, k0, t))
            s += nb
    return es, ee, ix, lot, s


class Wave:
    """One wavefront's window of 64 route entries and meta_of()."""

    def __init__(self, es, ee, ix, lot, count, first_block):
        self.es, self.ee, self.ix, self.lot, self.count = es, ee, ix, lot, count
        self.nbig = len(es)
        self.refills = []
        self.load_window(self.find(first_block))

    def find(self, b):
        """Last q with es[q] <= b (the kernel's 256-ary narrowing, four samples per lane)."""
        q0, n = 0, self.nbig
        while True:
            if n <= 64:
                return q0 + sum(1 for lane in range(n) if self.es[q0 + lane] <= b) - 1
            stp = (n + 255) // 256
            cnt = sum(1 for s in range(256) if s * stp < n and self.es[q0 + s * stp] <= b)
            if stp == 1:
                return q0 + cnt - 1
            q0 += (cnt - 1) * stp
            n = min(stp, n - (cnt - 1) * stp)

    def load_window(self, j0):
        self.wj = j0
        self.ws = []
        for lane in range(64):
            q = j0 + lane
            self.ws.append(self.es[q] if q < self.nbig else (self.count if q == self.nbig else None))
        self.wend = self.es[j0 + 64] if j0 + 64 < self.nbig else self.count
        self.refills.append(j0)

    def entry(self, b):
        """Window lane of block b: popcount(ballot(ws <= b)) - 1."""
        return sum(1 for v in self.ws if v is not None and v <= b) - 1

    def lane_e(self, e):
        q = self.wj + e
        return self.es[q], self.ee[q], self.ix[q], self.lot[q]

    def meta_of(self, g, C):
        """Per block j of grab g: (block b or None, address, k, lo, k0, t, first, idx)."""
        bf = g * C
        last = self.count - 1
        if bf >= self.count:  # nothing left: duplicates of entry 0's last block
            s0, e0, _, (lo0, _, _) = self.lane_e(0)
            nb0 = self.ws[1] - self.ws[0]
            lo = lo0 if nb0 == 1 else 0
            return [(None, e0 - BLOCK, 0, lo, 0, 0, False, None)] * C
        b0 = bf
        bl = min(bf + C - 1, last)
        while bl >= self.wend:
            adv = self.entry(b0) if b0 < self.wend else 64
            self.load_window(self.wj + adv)
        out = []
        e0 = self.entry(b0)
        se0 = self.ws[e0]
        sn0 = self.ws[e0 + 1] if e0 < 63 else self.wend
        if bl < sn0:  # one lookup for the grab
            _, e_end, idx, (lo, k0, t) = self.lane_e(e0)
            m0 = b0 - se0
            kk = sn0 - se0 - 1 - m0
            a0 = e_end - BLOCK * (kk + 1)
            for j in range(C):
                valid = b0 + j <= last
                addr = a0 + BLOCK * (j if valid else last - b0)
                first = valid and m0 == 0 and j == 0
                out.append((b0 + j if valid else None, addr, kk - j, lo if first else 0, k0 if first else 0, t,
                            first, idx if valid else None))
            return out
        for j in range(C):
            valid = b0 + j <= last
            b = b0 + j if valid else last
            e = self.entry(b)
            se = self.ws[e]
            sn = self.ws[e + 1] if e < 63 else self.wend
            m = b - se
            kk = sn - se - 1 - m
            _, e_end, idx, (lo, k0, t) = self.lane_e(e)
            first = m == 0
            out.append((b if valid else None, e_end - BLOCK * (kk + 1), kk, lo if first else 0, k0 if first else 0, t,
                        first, idx if valid else None))
        return out


def load_offsets(lo):
    """Block offsets the kernel's four loads per lane touch: max(ld_off + K, lo)."""
    offs = set()
    for lane in range(64):
        h, q, r = lane >> 5, (lane >> 4) & 1, lane & 15
        ld = 64 * r + 32 * q + 16 * h
        for k in range(4):
            offs.add(max(ld + 2048 * (k & 1) + 1024 * (k >> 1), lo))
    return offs


def simulate(offsets, lengths, bigmin, grid, wpb=16, C=4, rng=None, base=1 << 32, check_loads=True):
    """Runs the decomposition; returns (visits per block, errors)."""
    rng = rng or np.random.default_rng(0)
    es, ee, ix, lot, count = entries(offsets, lengths, bigmin, base)
    errors = []
    visits = np.zeros(count, dtype=np.int64)
    if count == 0:
        return visits, errors
    ngrab = (count + C - 1) // C
    per = (ngrab + grid - 1) // grid
    spans = {}
    for q in range(len(es)):
        a, e = geo(base + int(offsets[ix[q]]), int(lengths[ix[q]]), bigmin)[:2]
        spans[q] = (a, e)
    for wg in range(grid):
        g0 = wg * per
        g1 = min(g0 + per, ngrab)
        clamp = lambda g: g if g < g1 else ngrab  # noqa: E731
        first = g0 * C if g0 * C < count else count - 1
        waves = [Wave(es, ee, ix, lot, count, first) for _ in range(wpb)]
        # each wave's grab sequence: two static grabs, then grabs from the
        # workgroup counter in a random interleaving of the waves
        nxt = [[clamp(g0 + w), clamp(g0 + w + wpb)] for w in range(wpb)]
        ctr = 0
        active = list(range(wpb))
        while active:
            w = active[int(rng.integers(0, len(active)))]
            g = nxt[w].pop(0)
            if g >= ngrab:
                active.remove(w)
                continue
            nxt[w].append(clamp(g0 + 2 * wpb + ctr))
            ctr += 1
            for (b, addr, kk, lo, k0, t, fst, idx) in waves[w].meta_of(g, C):
                if b is None:  # a duplicate (result discarded): its loads must still stay inside a buffer
                    if check_loads:
                        lo_off = min(load_offsets(lo))
                        if not any(a <= addr + lo_off and addr + BLOCK <= e for a, e in spans.values()):
                            errors.append(("duplicate load", g, addr, lo))
                    continue
                visits[b] += 1
                q = max(i for i in range(len(es)) if es[i] <= b) if len(es) < 2000 else \
                    int(np.searchsorted(np.asarray(es), b, side="right")) - 1
                a, e = spans[q]
                nb = (es[q + 1] if q + 1 < len(es) else count) - es[q]
                want_k = nb - 1 - (b - es[q])
                want_lo, want_k0, want_t = lot[q]
                want_first = b == es[q]
                if (addr, kk, idx) != (e - BLOCK * (want_k + 1), want_k, ix[q]):
                    errors.append(("meta", b, addr, kk, idx))
                if fst != want_first or (fst and (lo, k0) != (want_lo, want_k0)) or t != want_t:
                    errors.append(("edge", b, fst, lo, k0, t))
                if check_loads:
                    for off in load_offsets(lo):
                        if addr + off < a or addr + off + 16 > e:
                            errors.append(("load", b, addr + off))
                            break
        for wv in waves:
            if any(b2 < b1 for b1, b2 in zip(wv.refills, wv.refills[1:])):
                errors.append(("window went backwards", wg))
    bad = np.nonzero(visits != 1)[0]
    if bad.size:
        errors.append(("coverage", bad[:8].tolist(), visits[bad[:8]].tolist()))
    return visits, errors
