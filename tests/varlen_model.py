"""Scalar model of the variable-length engine's work decomposition (v7,
foundationdb_amd/csrc/crc32c_varlen.hip: geo7 / k_v7count / k_v7prep /
k_varlen7).  Keep it in lockstep with the kernel.

It replays, on the CPU, how a batch is cut: every buffer of at least 16 bytes
whose 16-byte chunks span more than SMALL_SPAN bytes is cut into W windows of
1 KiB aligned to its end E = ceil16(P1) (window 0 starts `lo` bytes before
A = P0 & ~15); the windows of all buffers, in index order, are the batch's
slots; wave w streams slots [w*Qs, (w+1)*Qs).  Lane m of a load reads the 16
bytes at window + max(ld_off(m), min(lo, 1008)) for window 0 (the chunks
before the buffer are re-reads of its lead chunk, zeroed at compute time) and
window + ld_off(m) otherwise.  Shorter buffers are finished by the prep
kernel: byte-serially below 16 bytes, else one lane loading its chunks
[A, E) (clamped to the last one).  Tests check -- without a GPU -- that
(a) every slot belongs to exactly one wave, (b) the chunks a buffer's windows
checksum tile [A, E) exactly once, and (c) no lane ever loads a 16-byte chunk
that does not overlap its buffer.
"""
import numpy as np

SMALL_SPAN = 128  # FDBCRC_SMALL_SPAN


def lane_ld_off(lane):
    h, q, r = lane >> 5, (lane >> 4) & 1, lane & 15
    return 64 * r + 32 * q + 16 * h


LD_OFF = np.array([lane_ld_off(l) for l in range(64)], dtype=np.int64)


def geo7(P0, length):
    """(A, E, W, lo, k0, zt) exactly as the kernel's geo7()."""
    P1 = P0 + length
    E = (P1 + 15) & ~15
    A = P0 & ~15
    span = E - A
    W = (span + 1023) >> 10 if (length >= 16 and span > SMALL_SPAN) else 0
    lo = (1024 * W - span) & 1023
    return A, E, W, lo, P0 & 15, E - P1


def slots(lengths, offsets):
    """First slot g_i and window count W_i of every buffer; total slots."""
    g, Ws = [], []
    acc = 0
    for off, ln in zip(offsets, lengths):
        W = geo7(int(off), int(ln))[2]
        g.append(acc)
        Ws.append(W)
        acc += W
    return g, Ws, acc


def quantum(total, nwave):
    """Slots per wave (k_v7prep): ceil(total / nwave), at least 4, a multiple of 4."""
    q = (total + nwave - 1) // nwave
    return 4 if q < 4 else (q + 3) & ~3


def window_loads(P0, length, m):
    """16-byte chunk addresses of window m of a windowed buffer: (address, used)
    per lane -- `used` is False for the chunks before the buffer, which the
    kernel zeroes."""
    A, E, W, lo, _, _ = geo7(P0, length)
    wa = A - lo + 1024 * m
    lc = min(lo, 1008)
    out = []
    for lane in range(64):
        off = int(LD_OFF[lane])
        if m == 0:
            out.append((wa + max(off, lc), off >= lo))
        else:
            out.append((wa + off, True))
    return out


def small_loads(P0, length):
    """Chunk addresses the prep kernel loads for a small buffer (len >= 16)."""
    A, E, _, _, _, _ = geo7(P0, length)
    nch = (E - A) >> 4
    nc = SMALL_SPAN // 16
    return [A + 16 * min(j, nch - 1) for j in range(nc)]


def check_decomposition(lengths, offsets, nwave, check_loads=True):
    """Returns (coverage dict buf -> sorted chunk addresses, errors list)."""
    lengths = [int(x) for x in np.asarray(lengths, dtype=np.uint64)]
    offsets = [int(x) for x in np.asarray(offsets, dtype=np.uint64)]
    g, Ws, total = slots(lengths, offsets)
    errors = []
    # (a) slots -> waves: contiguous, disjoint, complete
    q = quantum(total, nwave)
    owner = {}
    for w in range(nwave):
        for s in range(w * q, min((w + 1) * q, total)):
            if s in owner:
                errors.append(("slot twice", s))
            owner[s] = w
    if len(owner) != total:
        errors.append(("slots uncovered", total - len(owner)))
    cover = {}
    for i, (off, ln) in enumerate(zip(offsets, lengths)):
        A, E, W, lo, k0, zt = geo7(off, ln)
        if ln < 16:
            continue  # byte-serial in prep: reads exactly [P0, P1)
        if W == 0:
            if check_loads:
                for ca in small_loads(off, ln):
                    if not (ca % 16 == 0 and ca + 16 > off and ca < off + ln):
                        errors.append(("small load outside", i, ca))
            continue
        if not (0 <= lo < 1024):
            errors.append(("lo", i, lo))
        used = []
        for m in range(W):
            for ca, u in window_loads(off, ln, m):
                if check_loads and not (ca % 16 == 0 and ca + 16 > off and ca < off + ln):
                    errors.append(("load outside", i, m, ca))
                if u:
                    used.append(ca)
        used.sort()
        # (b) the checksummed chunks tile [A, E) exactly once
        if used != list(range(A, E, 16)):
            errors.append(("coverage", i, len(used), (E - A) // 16))
        cover[i] = used
    return cover, errors
