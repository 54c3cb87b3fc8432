"""CPU model of the split XXH3-64 route for long buffers (test infrastructure;
the GPU kernels are foundationdb_amd/csrc/xxh3_split.hip).

XXH3 long inputs (xxhash.h:3641-3718, v0.8.0) accumulate 64-byte stripes into
eight 64-bit lanes and scramble the lanes after every 1 KiB block:

    acc <- scramble(acc + D[b])   for each full block b < nfull = (len-1) >> 10
    acc <- acc + D[nfull]         (the last block's stripes + the last stripe)
    h    = mergeAccs(acc, secret + 11, len * PRIME64_1)

where D[b] is the block's STRIPE SUM: the sum (mod 2^64, per lane) of the
accumulate_512 contributions of its 16 stripes -- a quantity that does not
depend on acc.  So the stripe sums of every block can be computed in parallel
(phase A, streaming), and only the 8-lane chain of scrambles is sequential
(phase B, 64 bytes of D per KiB).  This model restates both phases with
plain integers and is checked against the oracle (and so, transitively, the
reference's flow/xxhash.c) in tests/test_xxh3_split_model.py.
"""
M64 = (1 << 64) - 1
P32_1, P32_2, P32_3 = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D
P64_1, P64_2, P64_3 = 0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9
P64_4, P64_5 = 0x85EBCA77C2B2AE63, 0x27D4EB2F165667C5
INIT = [P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1]

# the default 192-byte secret (xxhash.h:2500-2511) as little-endian words
KSEC = [
    0xbe4ba423396cfeb8, 0x1cad21f72c81017c, 0xdb979083e96dd4de, 0x1f67b3b7a4a44072,
    0x78e5c0cc4ee679cb, 0x2172ffcc7dd05a82, 0x8e2443f7744608b8, 0x4c263a81e69035e0,
    0xcb00c391bb52283c, 0xa32e531b8b65d088, 0x4ef90da297486471, 0xd8acdea946ef1938,
    0x3f349ce33f76faa8, 0x1d4f0bc7c7bbdcf9, 0x3159b4cd4be0518a, 0x647378d9c97e9fc8,
    0xc3ebd33483acc5ea, 0xeb6313faffa081c5, 0x49daf0b751dd0d17, 0x9e68d429265516d3,
    0xfca1477d58be162b, 0xce31d07ad1b8f88f, 0x280416958f3acb45, 0x7e404bbbcafbd7af,
]


def secret(seed):
    """The 192-byte secret of XXH3_64bits_withSeed for long inputs
    (xxhash.h:3550-3566: word 2i + seed, word 2i+1 - seed)."""
    out = bytearray()
    for j, w in enumerate(KSEC):
        v = (w + seed) & M64 if j % 2 == 0 else (w - seed) & M64
        out += v.to_bytes(8, "little")
    return bytes(out)


def rd64(b, o):
    return int.from_bytes(b[o:o + 8], "little")


def stripe(data, off, sec, soff):
    """accumulate_512 contributions of the stripe at data[off:off+64] with
    secret + soff, as 8 lane deltas (xxhash.h:3641-3660)."""
    d = [0] * 8
    for i in range(8):
        v = rd64(data, off + 8 * i)
        k = v ^ rd64(sec, soff + 8 * i)
        d[i ^ 1] = (d[i ^ 1] + v) & M64
        d[i] = (d[i] + (k & 0xFFFFFFFF) * (k >> 32)) & M64
    return d


def block_sums(data, seed=0):
    """Phase A: D[0 .. nfull], one 8-lane stripe sum per block."""
    n = len(data)
    assert n > 240
    sec = secret(seed)
    nfull = (n - 1) >> 10
    D = []
    for b in range(nfull):
        acc = [0] * 8
        for s in range(16):
            acc = [(a + x) & M64 for a, x in zip(acc, stripe(data, 1024 * b + 64 * s, sec, 8 * s))]
        D.append(acc)
    ns = ((n - 1) - 1024 * nfull) >> 6
    acc = [0] * 8
    for s in range(ns):
        acc = [(a + x) & M64 for a, x in zip(acc, stripe(data, 1024 * nfull + 64 * s, sec, 8 * s))]
    acc = [(a + x) & M64 for a, x in zip(acc, stripe(data, n - 64, sec, 192 - 64 - 7))]
    D.append(acc)
    return D


def mulfold(a, b):
    p = a * b
    return (p & M64) ^ (p >> 64)


def avalanche(h):
    h ^= h >> 37
    h = (h * 0x165667919E3779F9) & M64
    return h ^ (h >> 32)


def chain(D, length, seed=0):
    """Phase B: the sequential scrambles over the stripe sums, then the merge."""
    sec = secret(seed)
    acc = list(INIT)
    for b in range(len(D) - 1):
        for j in range(8):
            a = (acc[j] + D[b][j]) & M64
            a ^= a >> 47
            a ^= rd64(sec, 128 + 8 * j)
            acc[j] = (a * P32_1) & M64
    acc = [(a + x) & M64 for a, x in zip(acc, D[-1])]
    r = (length * P64_1) & M64
    for k in range(4):
        r = (r + mulfold(acc[2 * k] ^ rd64(sec, 11 + 16 * k), acc[2 * k + 1] ^ rd64(sec, 19 + 16 * k))) & M64
    return avalanche(r)


def xxh3_split(data, seed=0):
    return chain(block_sums(data, seed), len(data), seed)


def pieces(lengths, split_min, piece_blocks=64):
    """The planner's piece list: every buffer longer than split_min is cut into
    pieces of piece_blocks blocks (the last one shorter); returns
    (split buffers [(i, F)], pieces [(split index, first block, blocks)])."""
    split, pcs, F = [], [], 0
    for i, L in enumerate(lengths):
        if L > split_min:
            nb = ((L - 1) >> 10) + 1
            s = len(split)
            split.append((i, F))
            for b0 in range(0, nb, piece_blocks):
                pcs.append((s, b0, min(piece_blocks, nb - b0)))
            F += nb
    return split, pcs, F
