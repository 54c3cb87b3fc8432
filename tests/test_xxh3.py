"""Batched XXH3-64 (include/fdb_xxh3.h) and the lookup3 checker.

CPU tests pin the oracle restatement (oracle/xxh3_oracle.c) to the fixtures
the reference's own flow/xxhash.c and flow/Hash3.c produced
(tests/golden/make_golden_xxh3.py) and to the known answers in
flow/Hash3.c:1248-1263.  GPU tests run the gfx950 kernels through the C ABI
and compare bit-for-bit with the fixtures and the oracle.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "xxh3_golden.json")


@pytest.fixture(scope="module")
def xg():
    with open(GOLDEN) as fh:
        return json.load(fh)


def sm_bytes(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


def hexs(a):
    return ["%016x" % int(v) for v in a]


def digest(a):
    """xor, sum and sha256 of a whole XXH3 result array (bench_shapes.digest64)."""
    import bench_shapes as S
    return S.digest64(a)


def pin(entry):
    import bench_shapes as S
    return S.pinned(entry)


# ------------------------------------------------------------------ CPU (oracle)

def test_oracle_grid_matches_reference_fixtures(xg):
    data = sm_bytes((1 << 20) + 64, 0x5EED)
    for row in xg["grid"]:
        off, seed = row["offset"], row["seed"]
        got = [O.xxh3_64(data[off:off + L], seed) for L in xg["lengths"]]
        assert hexs(got) == row["xxh3"], (off, seed)


def test_oracle_pages_match_reference_fixtures(xg):
    p = xg["pages"]
    pages = sm_bytes(p["count"] * 4096, p["state"])
    sq = O.xxh3_batch_fixed(pages, 4096, 4088, p["count"])
    assert hexs(sq[:4]) == p["sqlite_4088"]["first"]
    assert digest(sq) == pin(p["sqlite_4088"])
    dq = O.xxh3_batch_fixed(pages[8:], 4096, 4088, p["count"] - 1)
    assert digest(dq) == pin(p["diskqueue_4088_at8"])
    idx = np.arange(0, p["count"], 16, dtype=np.uint64)
    rw = O.xxh3_batch_varlen(pages, idx * 4096, np.full(idx.size, 4096, np.uint64), seeds=idx)
    assert digest(rw) == pin(p["redwood_seeded_4096_every16"])


def test_hashlittle2_known_answers(xg):
    # the reference's own expected outputs, flow/Hash3.c:1248-1259 (c, b)
    s = b"Four score and seven years ago"
    assert O.hashlittle2(b"", 0, 0) == (0xdeadbeef, 0xdeadbeef)
    assert O.hashlittle2(b"", 0, 0xdeadbeef) == (0xbd5b7dde, 0xdeadbeef)
    assert O.hashlittle2(b"", 0xdeadbeef, 0xdeadbeef) == (0x9c093ccd, 0xbd5b7dde)
    assert O.hashlittle2(s, 0, 0) == (0x17770551, 0xce7226e6)
    assert O.hashlittle2(s, 0, 1) == (0xe3607cae, 0xbd371de4)
    assert O.hashlittle2(s, 1, 0) == (0xcd628161, 0x6cbea4b3)
    for k in xg["hashlittle2"]["kat"]:
        assert list(O.hashlittle2(bytes.fromhex(k["hex"]), k["pc"], k["pb"])) == k["out"]
    pages = sm_bytes(64 * 4096, 0x5EED)
    for row in xg["hashlittle2"]["pages"]:
        pg = pages[4096 * row["page"]:4096 * (row["page"] + 1)]
        assert list(O.hashlittle2(pg[:4088], row["page"] + 1, 0x5ca1ab1e)) == row["sqlite"]
        assert list(O.hashlittle2(pg[16:], 0x12345678, 0xbeefabcd)) == row["diskqueue"]


@pytest.mark.skipif(not O.xxh3_reference_available(), reason="reference build absent")
@pytest.mark.parametrize("name", ["zipf", "chunks"])
def test_oracle_varlen_configs_exact_batches(xg, name):
    """The oracle restatement over the exact bench batches matches the
    reference's digests (make_golden_xxh3.py --varlen)."""
    import bench_shapes as S
    ent = xg["varlen_full"][name]
    lengths, offsets, extent = S.shape(name)
    assert S.lengths_digest(lengths) == ent["lengths_sha256"]
    data = O.splitmix64(extent // 8, ent["state"]).view(np.uint8)
    for d in ent["digests"]:
        seeds = S.xxh3_seeds(lengths.size) if d["kind"] == "seeds" else None
        got = O.xxh3_batch_varlen(data, offsets, lengths, seeds=seeds, threads=8)
        assert hexs(got[:64]) == d["first64"]
        assert digest(got) == pin(d)


def test_oracle_against_reference_random():
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    for _ in range(400):
        n = int(rng.integers(0, 5000))
        off = int(rng.integers(0, 64))
        seed = int(rng.integers(0, 2 ** 63)) if rng.random() < 0.5 else 0
        assert O.xxh3_64(data[off:off + n], seed) == O.ref_xxh3_64(data[off:off + n], seed)


# ------------------------------------------------------------------ GPU parity

def dev_bytes(h, cuda):
    import torch
    return torch.from_numpy(h).to(cuda)


def i64(a, cuda):
    import torch
    return torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)


def host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
def test_gpu_grid_golden(xg, cuda):
    import foundationdb_amd.xxh3 as X
    data = sm_bytes((1 << 20) + 64, 0x5EED)
    d = dev_bytes(data, cuda)
    L = np.array(xg["lengths"], dtype=np.int64)
    for row in xg["grid"]:
        offs = np.full(L.size, row["offset"], dtype=np.int64)
        got = host(X.batch_varlen(d, i64(offs, cuda), i64(L, cuda), seed=row["seed"]))
        assert hexs(got) == row["xxh3"], (row["offset"], row["seed"])


@pytest.mark.gpu
def test_gpu_pages_golden(xg, cuda):
    import torch
    import foundationdb_amd.xxh3 as X
    p = xg["pages"]
    pages = sm_bytes(p["count"] * 4096, p["state"])
    d = dev_bytes(pages, cuda)
    sq = host(X.batch_fixed(d, 4096, 4088, p["count"]))
    assert hexs(sq[:4]) == p["sqlite_4088"]["first"]
    assert digest(sq) == pin(p["sqlite_4088"])
    dq = host(X.batch_fixed(d, 4096, 4088, p["count"] - 1, byte_offset=8))
    assert digest(dq) == pin(p["diskqueue_4088_at8"])
    idx = np.arange(0, p["count"], 16, dtype=np.int64)
    seeds = torch.tensor(idx, device=cuda)
    rw = host(X.batch_fixed(d, 4096 * 16, 4096, idx.size, seeds=seeds))
    assert digest(rw) == pin(p["redwood_seeded_4096_every16"])


@pytest.mark.gpu
def test_gpu_fixed_lengths_vs_oracle(cuda):
    import foundationdb_amd.xxh3 as X
    h = sm_bytes(1 << 22, 0xC0FFEE)
    d = dev_bytes(h, cuda)
    for length in (0, 1, 3, 4, 8, 9, 16, 17, 128, 129, 240, 241, 1000, 1024, 1025, 4088, 4096, 5000, 16384):
        for stride in (length or 1, ((length + 15) & ~15) or 16, 4096 * 5):
            count = min(600, (h.size - length) // stride + 1)
            for seed in (0, 0xFDBEEFDB):
                got = host(X.batch_fixed(d, stride, length, count, seed=seed))
                assert np.array_equal(got, O.xxh3_batch_fixed(h, stride, length, count, seed=seed)), (length, stride)


@pytest.mark.gpu
def test_gpu_fixed_rows_eight_byte_aligned(cuda):
    """The row kernel's 8-byte-aligned form: rows starting at 8 mod 16 (the
    DiskQueue V2 region) load 16-byte aligned and shift by 8 bytes across
    lanes; a stride of 8 mod 16 (rows alternating 0 / 8 mod 16) keeps the
    exact loads.  Lengths around the block and stripe boundaries, batches that
    start at the tensor's first byte."""
    import foundationdb_amd.xxh3 as X
    h = sm_bytes(3 << 20, 0x5EA8)
    d = dev_bytes(h, cuda)
    for off, stride in ((8, 4096), (8, 2048), (8, 8192), (0, 4104), (8, 4104), (24, 1040)):
        for length in (241, 1000, 1024, 1025, 1032, 2047, 2048, 2049, 3000, 4088):
            if length > stride - (off & 15) and stride < 4096:
                continue
            count = min(300, (h.size - off - length) // stride + 1)
            for seed in (0, 0x1234567):
                got = host(X.batch_fixed(d, stride, length, count, seed=seed, byte_offset=off))
                want = O.xxh3_batch_fixed(h[off:], stride, length, count, seed=seed)
                assert np.array_equal(got, want), (off, stride, length, seed)


@pytest.mark.gpu
def test_gpu_varlen_random_vs_oracle(cuda):
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(5)
    h = sm_bytes(1 << 24, 0xBEEF)
    d = dev_bytes(h, cuda)
    n = 30000
    lens = np.where(rng.random(n) < 0.5, rng.integers(0, 300, n), rng.integers(0, 40000, n)).astype(np.int64)
    offs = rng.integers(0, h.size - 40000, n).astype(np.int64)
    seeds = rng.integers(0, 2 ** 63, n, dtype=np.int64)
    got = host(X.batch_varlen(d, i64(offs, cuda), i64(lens, cuda)))
    assert np.array_equal(got, O.xxh3_batch_varlen(h, offs, lens))
    got = host(X.batch_varlen(d, i64(offs, cuda), i64(lens, cuda), seeds=torch.tensor(seeds, device=cuda)))
    assert np.array_equal(got, O.xxh3_batch_varlen(h, offs, lens, seeds=seeds.view(np.uint64)))
    # a few large buffers mixed with tiny ones (one wave per large buffer)
    lens2 = np.array([1 << 20, 3, (1 << 20) + 17, 0, 100000, 241], dtype=np.int64)
    offs2 = np.array([0, 5, 1 << 21, 77, (1 << 22) + 9, 1 << 23], dtype=np.int64)
    got = host(X.batch_varlen(d, i64(offs2, cuda), i64(lens2, cuda), seed=7))
    assert np.array_equal(got, O.xxh3_batch_varlen(h, offs2, lens2, seed=7))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["zipf", "chunks"])
def test_gpu_varlen_configs_exact_batches(xg, cuda, name):
    """The exact xxh3-zipf (406 k packets, 64 B - 16 KiB) and xxh3-chunks
    (5773 chunks, 4 KiB - 1 MiB: the split route) batches bench.py measures,
    over the same splitmix64 bytes, unseeded and with per-buffer seeds, against
    the digests the reference's flow/xxhash.c produced for every buffer
    (make_golden_xxh3.py --varlen); the first 64 one by one."""
    import torch
    import bench_shapes as S
    import foundationdb_amd as F
    import foundationdb_amd.xxh3 as X
    ent = xg["varlen_full"][name]
    lengths, offsets, extent = S.shape(name)
    assert S.lengths_digest(lengths) == ent["lengths_sha256"] and lengths.size == ent["count"]
    buf = torch.empty(extent, dtype=torch.uint8, device=cuda)
    F.fill_splitmix64(buf, ent["state"])
    d_off, d_len = i64(offsets, cuda), i64(lengths, cuda)
    for d in ent["digests"]:
        seeds = torch.tensor(S.xxh3_seeds(lengths.size).view(np.int64), device=cuda) if d["kind"] == "seeds" else None
        got = host(X.batch_varlen(buf, d_off, d_len, seeds=seeds))
        assert hexs(got[:64]) == d["first64"], (name, d["kind"])
        assert digest(got) == pin(d), (name, d["kind"])
    del buf


@pytest.mark.gpu
def test_gpu_varlen_sparse_ranges_split_over_rows(cuda):
    """Batches with about one row buffer per wave (k_xxh3_vrows spreads such a
    buffer's blocks over the wave's four rows and chains them in order):
    every length class around the block edges, unaligned offsets, uniform and
    per-buffer seeds, against the oracle."""
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(41)
    h = sm_bytes(1 << 23, 0x5A5A)
    d = dev_bytes(h, cuda)
    edges = [1025, 1087, 1088, 2047, 2048, 2049, 3072, 4095, 4096, 4097, 8191, 8192, 15360, 16383, 16384]
    for n in (1, 3, 100, 1500):
        lens = np.array([edges[i % len(edges)] if i % 3 else int(rng.integers(1025, 16385)) for i in range(n)],
                        dtype=np.int64)
        if n == 1500:  # mixed with short and quad ones, as in the chunks batch's waves
            lens[::5] = rng.integers(0, 1025, lens[::5].size)
        offs = rng.integers(0, h.size - 16384, n).astype(np.int64)
        seeds = rng.integers(0, 2 ** 63, n, dtype=np.int64)
        got = host(X.batch_varlen(d, i64(offs, cuda), i64(lens, cuda), seed=0xFDBEEFDB))
        assert np.array_equal(got, O.xxh3_batch_varlen(h, offs, lens, seed=0xFDBEEFDB)), n
        got = host(X.batch_varlen(d, i64(offs, cuda), i64(lens, cuda), seeds=torch.tensor(seeds, device=cuda)))
        assert np.array_equal(got, O.xxh3_batch_varlen(h, offs, lens, seeds=seeds.view(np.uint64))), n


@pytest.mark.gpu
def test_gpu_empty_and_workspace(cuda):
    import torch
    import foundationdb_amd.xxh3 as X
    h = sm_bytes(1 << 16, 3)
    d = dev_bytes(h, cuda)
    assert X.batch_fixed(d, 4096, 4088, 0).numel() == 0
    n = 1000
    offs = np.arange(n, dtype=np.int64) * 37
    lens = (np.arange(n, dtype=np.int64) * 13) % 2000
    ws = torch.empty(X.varlen_workspace_bytes(n), dtype=torch.uint8, device=cuda)
    got = host(X.batch_varlen(d, i64(offs, cuda), i64(lens, cuda), workspace=ws))
    assert np.array_equal(got, O.xxh3_batch_varlen(h, offs, lens))


@pytest.mark.gpu
def test_gpu_xxh3_chained_packet_buffers(cuda):
    """XXH3-64 of packets spread over PacketBuffer chains (fdbrpc/FlowTransport.cpp:2025-2068):
    chains of 0..40 segments of 0..5000 bytes, any alignment, scattered through
    a buffer, uniform and per-chain seeds, against the reference's own
    flow/xxhash.c over each chain's concatenated bytes."""
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(2043)
    h = O.splitmix64((32 << 20) // 8, 0x2043).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    offs, lens, starts = [], [], [0]
    for c in range(3000):
        k = int(rng.choice([0, 1, 1, 1, 2, 3, 5, 17, 40]))
        offs += list(rng.integers(0, h.size - 5000, k))
        lens += list(rng.integers(0, 5000, k))
        starts.append(len(offs))
    offs[:4] = [0, 1, 3, 5]  # tiny, unaligned ones too
    lens[:4] = [1, 2, 0, 250]
    cat = lambda c: b"".join(h[o:o + l].tobytes() for o, l in zip(offs[starts[c]:starts[c + 1]], lens[starts[c]:starts[c + 1]]))
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)
    got = X.batch_chained(d, t(offs), t(lens), t(starts)).cpu().numpy().view(np.uint64)
    want = np.array([O.ref_xxh3_64(cat(c)) for c in range(len(starts) - 1)], dtype=np.uint64)
    assert np.array_equal(got, want)
    seeds = rng.integers(0, 2**63, len(starts) - 1, dtype=np.int64)
    got = X.batch_chained(d, t(offs), t(lens), t(starts), seeds=torch.from_numpy(seeds).to(cuda)).cpu().numpy().view(np.uint64)
    want = np.array([O.ref_xxh3_64(cat(c), int(seeds[c])) for c in range(len(starts) - 1)], dtype=np.uint64)
    assert np.array_equal(got, want)
    # more than one scan block of segments (4096 per block), and no segments at all
    n = 9000
    o2, l2 = rng.integers(0, h.size - 300, n), rng.integers(0, 300, n)
    s2 = np.arange(0, n + 1, 3)
    got = X.batch_chained(d, t(o2), t(l2), t(s2)).cpu().numpy().view(np.uint64)
    cat2 = lambda c: b"".join(h[o:o + l].tobytes() for o, l in zip(o2[s2[c]:s2[c + 1]], l2[s2[c]:s2[c + 1]]))
    assert all(int(got[c]) == O.ref_xxh3_64(cat2(c)) for c in range(0, len(s2) - 1, 7))
    e = torch.zeros(0, dtype=torch.int64, device=cuda)
    got = X.batch_chained(d, e, e, t([0, 0, 0]), seed=9).cpu().numpy().view(np.uint64)
    assert list(got) == [O.ref_xxh3_64(b"", 9)] * 2


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 0])
def test_gpu_xxh3_chained_in_place_rows(cuda, rows):
    """With the segment rows on (opt-in: fdbxxh_set_segrows),
    chains of 2..16 segments and 241 B .. 1 MiB are hashed where their
    segments lie (xxh3_segrows.hip), one 16-lane row per chain; off (the
    default), the same chains through staging.  Segment ends
    at every offset mod 16 and inside stripes, 1-byte segments, a segment
    boundary inside the last stripe (len - 64), lengths at the 240 / 241,
    1024 / 1025 and 1 MiB thresholds, 16 and 17 segments (the latter
    gathered), uniform and per-chain seeds -- against the reference's own
    flow/xxhash.c over each chain's concatenated bytes."""
    import torch
    import foundationdb_amd.xxh3 as X
    from foundationdb_amd import crc32c as F
    L = F.lib()
    prev = L.fdbxxh_set_segrows(rows)
    try:
        _chained_rows_case(cuda, X)
    finally:
        L.fdbxxh_set_segrows(prev)


def _chained_rows_case(cuda, X):
    import torch
    rng = np.random.default_rng(2046)
    h = O.splitmix64((48 << 20) // 8, 0x2046).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    offs, lens, starts = [], [], [0]

    def chain(parts):
        for L in parts:
            offs.append(int(rng.integers(0, h.size - max(L, 1) - 1)))
            lens.append(int(L))
        starts.append(len(offs))

    for total in (241, 242, 255, 256, 257, 300, 1023, 1024, 1025, 1088, 2047, 2048, 2049, 4096, 16384, 65536,
                  (1 << 20) - 1, 1 << 20, (1 << 20) + 1):
        for ns in (2, 3, 16, 17):
            if ns > total:
                continue
            cuts = np.sort(rng.choice(np.arange(1, total), ns - 1, replace=False))
            chain(np.diff(np.concatenate([[0], cuts, [total]])))
    for m in range(16):  # the boundary at every offset mod 16, inside the first block and inside the last stripe
        chain([320 + m, 700])
        chain([1000, 30 + m])
        chain([1, 1, 1, 500 + m, 1])
    for _ in range(400):  # PacketBuffer-like chains: a packet over 4 KiB buffers
        L = int(rng.integers(241, 16385))
        first = int(rng.integers(1, 4097))
        parts = [min(first, L)]
        while sum(parts) < L:
            parts.append(min(4096, L - sum(parts)))
        chain(parts)
    cat = lambda c: b"".join(h[o:o + l].tobytes() for o, l in zip(offs[starts[c]:starts[c + 1]], lens[starts[c]:starts[c + 1]]))
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)
    nc = len(starts) - 1
    got = X.batch_chained(d, t(offs), t(lens), t(starts)).cpu().numpy().view(np.uint64)
    want = np.array([O.ref_xxh3_64(cat(c)) for c in range(nc)], dtype=np.uint64)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(c), len(cat(c)), int(starts[c + 1] - starts[c])) for c in bad[:8]]
    seeds = rng.integers(0, 2**63, nc, dtype=np.int64)
    got = X.batch_chained(d, t(offs), t(lens), t(starts), seeds=torch.from_numpy(seeds).to(cuda)).cpu().numpy().view(np.uint64)
    want = np.array([O.ref_xxh3_64(cat(c), int(seeds[c])) for c in range(nc)], dtype=np.uint64)
    assert np.array_equal(got, want)
    got = X.batch_chained(d, t(offs), t(lens), t(starts), seed=0xFDBEEFDB).cpu().numpy().view(np.uint64)
    assert all(int(got[c]) == O.ref_xxh3_64(cat(c), 0xFDBEEFDB) for c in range(0, nc, 5))


@pytest.mark.gpu
@pytest.mark.parametrize("lc", [1, 0])
def test_gpu_xxh3_chained_lds_route(cuda, lc):
    """Short chains staged in LDS (k_xxh3_lchain, round 6: 2..8 segments, at
    most 16 KiB) and, with the route off, the same chains through staging:
    every short-form threshold (0, 1-3, 4-8, 9-16, 17-128, 129-240) and the
    long form's (241, 1024/1025, a last stripe cut by a boundary, 16383 /
    16384 / 16385 bytes, the last gathered), zero-length and 1-byte segments,
    boundaries at every offset mod 16 and several inside one 16-byte chunk,
    8 and 9 segments, segments at any alignment up to the buffer's last byte,
    uniform and per-chain seeds -- against the reference's own flow/xxhash.c
    over each chain's concatenated bytes."""
    import torch
    import foundationdb_amd.xxh3 as X
    from foundationdb_amd import crc32c as F
    Lb = F.lib()
    prev = Lb.fdbxxh_set_lchain(lc)
    try:
        rng = np.random.default_rng(2047)
        h = O.splitmix64((8 << 20) // 8, 0x2047).view(np.uint8)
        d = torch.from_numpy(h).to(cuda)
        offs, lens, starts = [], [], [0]

        def chain(parts, at_end=False):
            for L in parts:
                o = h.size - int(L) if at_end else int(rng.integers(0, h.size - max(int(L), 1)))
                offs.append(o)
                lens.append(int(L))
            starts.append(len(offs))

        for total in (0, 1, 2, 3, 4, 7, 8, 9, 15, 16, 17, 31, 32, 33, 127, 128, 129, 200, 239, 240, 241, 255, 256,
                      1023, 1024, 1025, 1088, 1090, 2047, 2048, 4095, 4096, 4097, 8000, 16383, 16384, 16385):
            for ns in (2, 3, 5, 8, 9):
                cuts = np.sort(rng.integers(0, total + 1, ns - 1))
                chain(np.diff(np.concatenate([[0], cuts, [total]])))
        for m in range(16):  # boundaries at every offset mod 16; three inside one chunk; inside the last stripe
            chain([320 + m, 700])
            chain([16 * 40 + m, 1, 2, 3000])
            chain([1000, 30 + m])
            chain([2, 0, 0, 1, 700 + m, 1])
        chain([5, 300], at_end=True)  # segments ending at the buffer's last byte
        chain([4096 - 7, 4096, 4096, 4000], at_end=True)
        for _ in range(300):  # PacketBuffer-like chains
            L = int(rng.integers(1, 16385))
            first = int(rng.integers(1, 4097))
            parts = [min(first, L)]
            while sum(parts) < L:
                parts.append(min(4096, L - sum(parts)))
            chain(parts)
        cat = lambda c: b"".join(h[o:o + l].tobytes() for o, l in zip(offs[starts[c]:starts[c + 1]], lens[starts[c]:starts[c + 1]]))
        t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)
        nc = len(starts) - 1
        got = X.batch_chained(d, t(offs), t(lens), t(starts)).cpu().numpy().view(np.uint64)
        want = np.array([O.ref_xxh3_64(cat(c)) for c in range(nc)], dtype=np.uint64)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(c), len(cat(c)), int(starts[c + 1] - starts[c])) for c in bad[:8]]
        seeds = rng.integers(0, 2**63, nc, dtype=np.int64)
        got = X.batch_chained(d, t(offs), t(lens), t(starts), seeds=torch.from_numpy(seeds).to(cuda)).cpu().numpy().view(np.uint64)
        want = np.array([O.ref_xxh3_64(cat(c), int(seeds[c])) for c in range(nc)], dtype=np.uint64)
        assert np.array_equal(got, want)
        got = X.batch_chained(d, t(offs), t(lens), t(starts), seed=0xFDBEEFDB).cpu().numpy().view(np.uint64)
        assert all(int(got[c]) == O.ref_xxh3_64(cat(c), 0xFDBEEFDB) for c in range(nc))
    finally:
        Lb.fdbxxh_set_lchain(prev)


@pytest.mark.gpu
def test_gpu_xxh3_chained_underestimated_total(cuda):
    """A total_bytes below the real sum of the segment lengths (caller error):
    the digests are undefined but every read stays inside the workspace
    (k_chain_ranges clamps to the staging area), so the call completes and the
    chains that fit in the bound are still exact; chain starts past nsegs are
    clamped too."""
    import torch
    import foundationdb_amd.xxh3 as X
    h = O.splitmix64((4 << 20) // 8, 0x51).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    n = 4000
    rng = np.random.default_rng(136)
    offs = rng.integers(0, h.size - 70000, n)
    lens = rng.integers(1000, 65536, n)
    starts = np.arange(0, n + 1, 4)
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)
    total = int(lens.sum())
    for bound in (total // 3, 4096, 0):
        got = X.batch_chained(d, t(offs), t(lens), t(starts), total_bytes=bound)
        torch.cuda.synchronize()
        got = got.cpu().numpy().view(np.uint64)
        # chains wholly inside the bound are exact
        pre = np.concatenate([[0], np.cumsum(lens)])
        c = 0
        while c + 1 < starts.size and pre[starts[c + 1]] <= bound:
            cat = b"".join(h[o:o + l].tobytes() for o, l in zip(offs[starts[c]:starts[c + 1]], lens[starts[c]:starts[c + 1]]))
            assert int(got[c]) == O.ref_xxh3_64(cat)
            c += 1
    # chain starts past nsegs: clamped, no out-of-range read of the prefix array
    got = X.batch_chained(d, t(offs[:8]), t(lens[:8]), t([0, 4, 1 << 40]), total_bytes=int(lens[:8].sum()))
    torch.cuda.synchronize()
    cat = b"".join(h[o:o + l].tobytes() for o, l in zip(offs[:4], lens[:4]))
    assert int(got.cpu().numpy().view(np.uint64)[0]) == O.ref_xxh3_64(cat)


@pytest.mark.gpu
def test_gpu_xxh3_split_route_long_buffers(cuda):
    """Buffers longer than 16 KiB on the split route (xxh3_split.hip: every
    1 KiB block's stripe sums in parallel, then one chain of scrambles per
    buffer): 1 MiB, 16 MiB and 100 MiB (FlowTransport's PACKET_LIMIT,
    flow/Knobs.cpp:237) buffers at unaligned offsets, the 16 KiB threshold and
    block-boundary lengths, mixed with short and mid-size buffers; uniform and
    per-buffer seeds; through a caller workspace sized for the route, and
    through the convenience form on a fresh stream (its first batch has no
    room yet and runs on the row kernel, the next ones take the split route).
    The three big buffers are also checked against the reference's own
    flow/xxhash.c."""
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(3641)
    h = O.splitmix64((150 << 20) // 8, 0x3718).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    big = [(1 << 20) + 3, 16 << 20, 100 << 20]
    edge = [16384, 16385, 17408, 17409, 20000, 65536, 65537, 1 << 20, 3, 0, 240, 241, 1024, 4096]
    mid = [int(x) for x in rng.integers(16000, 300000, 300)] + [int(x) for x in rng.integers(0, 5000, 300)]
    lens = np.array(big + edge + mid, dtype=np.int64)
    offs = np.array([int(rng.integers(0, h.size - L + 1)) for L in lens], dtype=np.int64)
    offs[:3] = [7, 101 << 20 | 5, 1 << 20 | 9]
    seeds = rng.integers(0, 2 ** 63, lens.size, dtype=np.int64)
    want = O.xxh3_batch_varlen(h, offs, lens)
    want_s = O.xxh3_batch_varlen(h, offs, lens, seeds=seeds.view(np.uint64))
    if O.xxh3_reference_available():
        for j in range(3):
            assert int(want[j]) == O.ref_xxh3_64(h[offs[j]:offs[j] + lens[j]].tobytes())
            assert int(want_s[j]) == O.ref_xxh3_64(h[offs[j]:offs[j] + lens[j]].tobytes(), int(seeds[j]))
    o, l, sd = i64(offs, cuda), i64(lens, cuda), torch.from_numpy(seeds).to(cuda)
    ws = torch.empty(X.varlen_workspace_bytes(lens.size, int(lens.sum())), dtype=torch.uint8, device=cuda)
    assert np.array_equal(host(X.batch_varlen(d, o, l, workspace=ws)), want)
    assert np.array_equal(host(X.batch_varlen(d, o, l, seeds=sd, workspace=ws)), want_s)
    # room for a third of the long blocks: the row kernel takes every buffer
    ws3 = torch.empty(X.varlen_workspace_bytes(lens.size, int(lens.sum()) // 3), dtype=torch.uint8, device=cuda)
    assert np.array_equal(host(X.batch_varlen(d, o, l, seeds=sd, workspace=ws3)), want_s)
    s = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s):
        for _ in range(3):
            got = X.batch_varlen(d, o, l, stream=s)
            got_s = X.batch_varlen(d, o, l, seeds=sd, stream=s)
            s.synchronize()
            assert np.array_equal(host(got), want)
            assert np.array_equal(host(got_s), want_s)


@pytest.mark.gpu
def test_gpu_xxh3_split_route_fixed_and_chained(cuda):
    """Fixed-length long buffers (batch_fixed > 16 KiB: the split route with
    the library's workspace) and one 100 MiB packet over a PacketBuffer chain
    of segments (fdbrpc/FlowTransport.cpp:2025-2068) with small chains around
    it, against the oracle / the reference."""
    import torch
    import foundationdb_amd.xxh3 as X
    h = O.splitmix64((110 << 20) // 8, 0x2068).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    for length, stride, count in ((65536 + 5, 65536 + 16, 300), (16385, 16400, 1000), (1 << 20, 1 << 20, 60)):
        for seed in (0, 0xFDBEEFDB):
            got = host(X.batch_fixed(d, stride, length, count, seed=seed, byte_offset=3))
            assert np.array_equal(got, O.xxh3_batch_fixed(h[3:], stride, length, count, seed=seed)), (length, seed)
    seeds = torch.arange(300, dtype=torch.int64, device=cuda) * 0x9E3779B97F4A7C15
    got = host(X.batch_fixed(d, 65536 + 16, 65536 + 5, 300, seeds=seeds))
    assert np.array_equal(got, O.xxh3_batch_fixed(h, 65536 + 16, 65536 + 5, 300, seeds=seeds.cpu().numpy().view(np.uint64)))
    rng = np.random.default_rng(9)
    nseg = 1000
    seg = rng.integers(1, 2 * (100 << 20) // nseg, nseg)
    seg[-1] = max(1, (100 << 20) - int(seg[:-1].sum())) if seg[:-1].sum() < (100 << 20) else 1
    so = rng.integers(0, h.size - int(seg.max()), nseg)
    offs = list(so) + [5, 77, 1000]
    lens = list(seg) + [300, 20000, 0]
    starts = [0, nseg, nseg + 1, nseg + 3]
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=cuda)
    got = X.batch_chained(d, t(offs), t(lens), t(starts)).cpu().numpy().view(np.uint64)
    cat = lambda c: b"".join(h[o:o + n].tobytes() for o, n in zip(offs[starts[c]:starts[c + 1]], lens[starts[c]:starts[c + 1]]))
    ref = O.ref_xxh3_64 if O.xxh3_reference_available() else (lambda b: O.xxh3_64(np.frombuffer(b, np.uint8)))
    for c in range(3):
        assert int(got[c]) == ref(cat(c)), c


@pytest.mark.gpu
def test_gpu_xxh3_long_route_reuses_slots(cuda):
    """More long buffers than k_xlong has chain slots (4 per CU): every slot
    takes several buffers in turn (its LDS ring's step numbers run on across
    buffers), largest first, over packed, overlapping and unaligned offsets;
    per-buffer seeds and a uniform one; twice on one stream (the dequeue
    counter and class cursors are re-planned per launch)."""
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(2068)
    h = O.splitmix64((96 << 20) // 8, 0x5107).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    n = 3000
    lens = np.exp(rng.uniform(np.log(16385), np.log(96 << 10), n)).astype(np.int64)
    lens[:40] = 16385 + rng.integers(0, 4096, 40)  # the smallest class, many per slot
    offs = np.array([int(rng.integers(0, h.size - L + 1)) for L in lens], dtype=np.int64)
    seeds = rng.integers(0, 2 ** 63, n, dtype=np.int64)
    want = O.xxh3_batch_varlen(h, offs, lens, seed=0xFDBEEFDB)
    want_s = O.xxh3_batch_varlen(h, offs, lens, seeds=seeds.view(np.uint64))
    o, l, sd = i64(offs, cuda), i64(lens, cuda), torch.from_numpy(seeds).to(cuda)
    ws = torch.empty(X.varlen_workspace_bytes(n, int(lens.sum())), dtype=torch.uint8, device=cuda)
    for _ in range(2):
        assert np.array_equal(host(X.batch_varlen(d, o, l, seed=0xFDBEEFDB, workspace=ws)), want)
        assert np.array_equal(host(X.batch_varlen(d, o, l, seeds=sd, workspace=ws)), want_s)


@pytest.mark.gpu
def test_gpu_xxh3_long_route_planner_forms(cuda):
    """Long buffers among tens of thousands of short ones: at 256 tiles of
    256 buffers (65536) the planner's assign pass reduces the tiles itself
    (no k_xscan, class bases from the earlier tiles' counts), past that it
    takes the separate scan; both against the oracle, uniform and per-buffer
    seeds."""
    import torch
    import foundationdb_amd.xxh3 as X
    rng = np.random.default_rng(1087)
    h = O.splitmix64((48 << 20) // 8, 0x1087).view(np.uint8)
    d = torch.from_numpy(h).to(cuda)
    for count in (65536, 70001):
        lens = rng.integers(0, 600, count).astype(np.int64)
        where = rng.choice(count, 60, replace=False)
        lens[where] = rng.integers(16385, 400000, where.size)
        lens[where[:3]] = [16385, 1 << 20, 17409]
        offs = rng.integers(0, h.size - lens.max() - 1, count).astype(np.int64)
        seeds = rng.integers(0, 2 ** 63, count, dtype=np.int64)
        o, l, sd = i64(offs, cuda), i64(lens, cuda), torch.from_numpy(seeds).to(cuda)
        ws = torch.empty(X.varlen_workspace_bytes(count, int(lens.sum())), dtype=torch.uint8, device=cuda)
        want = O.xxh3_batch_varlen(h, offs, lens)
        assert np.array_equal(host(X.batch_varlen(d, o, l, workspace=ws)), want), count
        want_s = O.xxh3_batch_varlen(h, offs, lens, seeds=seeds.view(np.uint64))
        assert np.array_equal(host(X.batch_varlen(d, o, l, seeds=sd, workspace=ws)), want_s), count
