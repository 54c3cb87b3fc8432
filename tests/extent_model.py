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
