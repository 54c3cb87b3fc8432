"""CPU model of the EXTENT route (crc32c_extent.hip), byte-exact, for small
batches: the arithmetic the kernels implement, checked against the oracle by
tests/test_extent_model.py before anything runs on a GPU.

A batch whose buffers lie in ascending order without overlaps and with small
gaps (packets back to back in a receive buffer, chunks of a file) is streamed
as ONE byte range -- the EXTENT [S, Eend), S = first buffer's start rounded
down to 16 -- in 4 KiB blocks exactly like 4 KiB pages.  Every buffer's CRC
comes from two PREFIX registers of that stream, by CRC linearity:

    raw(bytes [s, e)) = R(e) ^ R(s) * x^(8(e - s))      R(p) = raw(bytes [S, S+p))

so the gap bytes between buffers cancel and nothing is masked.  R(p) at a
point p (relative to S) inside block k = (p-1) >> 12, with cnt = (p - 4096k) >> 6
whole 64-byte lane spans before it:
    R(p64) = (Y[k] ^ V) * x^(-8*64*(64 - cnt))      p64 = 4096k + 64 cnt
    R(p)   = the raw register R(p64) fed the (p - p64) < 64 bytes after p64
where V = H_k[cnt-1] (0 for cnt = 0) is the inclusive XOR prefix over the
block's lanes of lane registers weighted to the block end (the page kernel's
fold as a prefix scan) and Y[k] = raw(bytes [S, S+4096k)) * x^(8*4096) is the
exclusive prefix of the block registers B[j] = H_j[63], positioned at block
k's end (a scan over blocks).  Finally
    crc32c_append(seed, buf) = ~(R(e) ^ (R(s) ^ ~seed) * x^(8 len)).
"""
import numpy as np

POLY = 0x82F63B78
ONE = 0x80000000


def gf2_mul(a, b):
    r = 0
    for _ in range(32):
        if a & 0x80000000:
            r ^= b
        a = (a << 1) & 0xFFFFFFFF
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return r


def xpow8(n):
    """x^(8n) mod P (reflected)."""
    r, p = ONE, ONE >> 8
    while n:
        if n & 1:
            r = gf2_mul(r, p)
        p = gf2_mul(p, p)
        n >>= 1
    return r


def xpow8_inv(n):
    xinv = ((POLY ^ ONE) << 1 | 1) & 0xFFFFFFFF
    p = ONE
    for _ in range(8):
        p = gf2_mul(p, xinv)
    r = ONE
    while n:
        if n & 1:
            r = gf2_mul(r, p)
        p = gf2_mul(p, p)
        n >>= 1
    return r


def feed(reg, data):
    """raw register fed bytes (no inversions)."""
    for b in bytes(data):
        reg ^= b
        for _ in range(8):
            reg = (reg >> 1) ^ POLY if reg & 1 else reg >> 1
    return reg


M = xpow8(4096)


def eligible(P0, P1):
    """Ascending, non-overlapping, each gap < 4096 and at most max(len, 256)
    (the gap bytes are read: this bounds the waste and keeps every gap byte in
    a page that holds buffer bytes)."""
    for i in range(len(P0) - 1):
        g = P0[i + 1] - P1[i]
        if g < 0 or g >= 4096 or g > max(P1[i] - P0[i], 256):
            return False
    return True


def extent_crcs(mem, offsets, lengths, seed):
    """mem: bytes-like (the device memory), offsets/lengths: the batch."""
    P0 = [int(o) for o in offsets]
    P1 = [int(o) + int(l) for o, l in zip(offsets, lengths)]
    assert eligible(P0, P1)
    S = P0[0] & ~15
    Eend = (P1[-1] + 15) & ~15
    nblk = (Eend - S + 4095) // 4096
    ext = bytes(mem[S:Eend]) + bytes(nblk * 4096 - (Eend - S))  # bytes past Eend: never used
    lane_w = [xpow8(64 * (63 - l)) for l in range(64)]
    H = []  # per block: inclusive prefix over lanes (weighted to the block end)
    for k in range(nblk):
        h, acc = [], 0
        for l in range(64):
            reg = feed(0, ext[4096 * k + 64 * l:4096 * k + 64 * l + 64])
            acc ^= gf2_mul(reg, lane_w[l])
            h.append(acc)
        H.append(h)
    B = [h[63] for h in H]
    Y, X = [], 0  # Y[k] = X_k * M, X_{k+1} = X_k * M ^ B_k
    for k in range(nblk):
        Y.append(gf2_mul(X, M))
        X = Y[-1] ^ B[k]

    def R(p):
        if p == 0:
            return 0
        k = (p - 1) >> 12
        cnt = (p - 4096 * k) >> 6
        V = H[k][cnt - 1] if cnt else 0
        r = gf2_mul(Y[k] ^ V, xpow8_inv(64 * (64 - cnt)))
        p64 = 4096 * k + 64 * cnt
        return feed(r, ext[p64:p])

    out = []
    for a, b in zip(P0, P1):
        s, e = a - S, b - S
        raw = R(e) ^ gf2_mul(R(s) ^ (~seed & 0xFFFFFFFF), xpow8(b - a))
        out.append(~raw & 0xFFFFFFFF)
    return np.array(out, dtype=np.uint32)


def _span_registers(ext):
    """raw register of every 64-byte span of ext (fed into 0), through the C
    oracle: feed(0, d) = ~crc32c_append(0xFFFFFFFF, d)."""
    from oracle import oracle as O
    n = len(ext) // 64
    buf = np.frombuffer(ext, np.uint8)
    offs = np.arange(n, dtype=np.uint64) * 64
    return ~O.batch_varlen(buf, offs, np.full(n, 64, np.uint64), seed=0xFFFFFFFF)


def ranges_per(nblk, nwave, unit=4):
    """Blocks per wave of k_xstream's static ranges (a multiple of `unit`)."""
    per = (nblk + nwave - 1) // nwave
    return (per + unit - 1) // unit * unit


def extent_crcs_ranges(mem, offsets, lengths, seed, nwave, per=None):
    """The same CRCs the way the kernels compute them since round 4, without a
    scan over all blocks: wave w streams the blocks [k0, k1) = [w*per, ...) of
    its RANGE and keeps the range-local prefix X (0 at k0) itself, block by
    block:  Z[k] = X_k * M,  X_{k+1} = Z[k] ^ B[k],  A[w] = X_{k1}.  A point
    p = 4096k + 64 cnt + 16 cq + r (r < 16) of block k is CAPTURED by the wave
    streaming block k as two words:
        G(p) = Z[k] ^ H_k[cnt-1]   (its range-local prefix at p64, positioned
                                    at block k's end)
        Y(p) = y_cq of lane span cnt: the raw register of that span's first
               16 cq bytes (0 for cq = 0)
    and the finishing pass forms
        R(p16) = G(p) * x^(-8*64*(64-cnt)) * x^(8*16 cq) ^ Y(p),
        R(p)   = R(p16) fed the r bytes of the 16-byte chunk at p16.
    The ranges' global start registers are X0[w+1] = X0[w] * M^per ^ A[w]; a
    buffer whose two points lie in one range needs only the local values (X0[w]
    cancels), others add X0 * M^(k-k0+1) to both."""
    P0 = [int(o) for o in offsets]
    P1 = [int(o) + int(l) for o, l in zip(offsets, lengths)]
    assert eligible(P0, P1)
    S = P0[0] & ~15
    Eend = (P1[-1] + 15) & ~15
    nblk = (Eend - S + 4095) // 4096
    ext = bytes(mem[S:Eend]) + bytes(nblk * 4096 - (Eend - S))
    lane_w = [xpow8(64 * (63 - l)) for l in range(64)]
    spans = _span_registers(ext)
    H = []
    for k in range(nblk):
        h, acc = [], 0
        for l in range(64):
            acc ^= gf2_mul(int(spans[64 * k + l]), lane_w[l])
            h.append(acc)
        H.append(h)
    if per is None:
        per = ranges_per(nblk, nwave) if nblk else 4
    else:  # k_xgrab's grabs of `per` blocks
        nwave = max(1, -(-nblk // per))
    Z, A = [0] * nblk, []
    for w in range(nwave):
        k0, k1 = min(w * per, nblk), min(w * per + per, nblk)
        X = 0
        for k in range(k0, k1):  # block by block, as k_xstream does
            Z[k] = gf2_mul(X, M)
            X = Z[k] ^ H[k][63]
        A.append(X)
    X0 = [0]
    for w in range(nwave - 1):
        X0.append(gf2_mul(X0[-1], xpow8(4096 * per)) ^ A[w])

    def point(p):
        k = (p - 1) >> 12 if p else 0
        cnt = (p - 4096 * k) >> 6 if p else 0
        return k, cnt, k // per

    def capture(p):
        """the two words k_xstream stores for point p"""
        if p == 0:
            return 0, 0
        k, cnt, _ = point(p)
        cq = ((p - 4096 * k) & 63) >> 4
        G = Z[k] ^ (H[k][cnt - 1] if cnt else 0)
        span = 4096 * k + 64 * cnt
        Y = feed(0, ext[span:span + 16 * cq]) if cq else 0
        return G, Y

    def R(p, glob):
        if p == 0:
            return 0
        k, cnt, w = point(p)
        G, Y = capture(p)
        if glob:
            G ^= gf2_mul(X0[w], xpow8(4096 * (k - w * per + 1)))
        rem = (p - 4096 * k) & 63
        cq, r = rem >> 4, rem & 15
        reg = gf2_mul(G, xpow8_inv(64 * (64 - cnt)))
        if cq:
            reg = gf2_mul(reg, xpow8(16 * cq)) ^ Y
        p16 = p - r
        return feed(reg, ext[p16:p])

    out = []
    for a, b in zip(P0, P1):
        s, e = a - S, b - S
        glob = point(s)[2] != point(e)[2]
        raw = R(e, glob) ^ gf2_mul(R(s, glob) ^ (~seed & 0xFFFFFFFF), xpow8(b - a))
        out.append(~raw & 0xFFFFFFFF)
    return np.array(out, dtype=np.uint32)
