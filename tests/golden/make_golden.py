"""Generate tests/golden/crc32c_golden.json from the REFERENCE implementation.

Runs FoundationDB's own contrib/crc32/crc32c.cpp, compiled unmodified by
oracle/Makefile into oracle/_ref/libcrc32c_ref.so, so the fixtures pin the
reference's behaviour (the oracle restatement and the GPU engine are both
checked against them).  Inputs are described, not stored: every data buffer is
a splitmix64 stream (BASELINE.md generator) or a closed-form pattern, so the
JSON holds parameters and the reference's outputs only.

Usage (in the container that has /root/reference):
    make -C oracle && python tests/golden/make_golden.py            # everything
    python tests/golden/make_golden.py --varlen                       # only "varlen_full"
    python tests/golden/make_golden.py --shards                       # only "pages_shards"
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
import bench_shapes as S  # noqa: E402  (digest: xor, sum and sha256 of a whole result array)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crc32c_golden.json")

SEEDS = [0x00000000, 0xFDBEEFDB, 0xAB12FD93, 0x12345678, 0xFFFFFFFF]


def sm_bytes(nbytes, state):
    w = O.splitmix64((nbytes + 7) // 8, state)
    return w.view(np.uint8)[:nbytes].copy()


def varlen_full(g):
    """BASELINE configs[2] (Zipf packets) and configs[4] (backup chunks) at their
    exact bench shapes (bench_shapes.py), and configs[2]'s packets scattered
    (shuffled, non-ascending offsets: the window route's batch): the reference's crc32c_append over
    every buffer of each ~1 GiB batch, as xor/sum/sha256 digests plus the first 64
    checksums, for seeds 0 and 0xFDBEEFDB."""
    ref = O.reference()
    out = {}
    for name in ("zipf", "chunks", "zipf-scattered"):
        lengths, offsets, extent = S.shape(name)
        data = O.splitmix64(extent // 8, S.STATE).view(np.uint8)
        ent = {"state": S.STATE, "count": int(lengths.size), "total_bytes": int(lengths.sum()),
               "extent": extent, "align": S.SHAPES[name][1], "lengths_sha256": S.lengths_digest(lengths),
               "digests": []}
        for seed in (0, 0xFDBEEFDB):
            c = np.zeros(lengths.size, np.uint32)
            f = ref.lib.ref_batch_varlen
            f.restype = None
            f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
            f(data.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, lengths.size, seed, c.ctypes.data)
            ent["digests"].append(dict(S.digest(c), seed=seed, first64=[int(x) for x in c[:64]]))
        out[name] = ent
        del data
    g["varlen_full"] = out


def pages_shards(g, nshard=8, threads=8):
    """BASELINE configs[3]: a whole-file scan (SQLiteDB::checkAllPageChecksums,
    fdbserver/kvstore/KeyValueStoreSQLite.cpp:1378-1470) sharded over up to 8
    GPUs -- rank r checksums bytes [r*4 GiB, (r+1)*4 GiB) of one splitmix64
    file.  The reference's crc32c_append over every page of every shard, as 8 KiB
    pages with the SQLite seed (pages8k) and as 4 KiB pages with seed 0
    (pages4k), xor/sum/sha256 digests per shard."""
    from concurrent.futures import ThreadPoolExecutor
    from bench_shapes import GOLDEN_GAMMA, SHARD_BYTES, shard_state
    import bench_shapes as S
    out = {"state": 0x5EED, "shard_bytes": SHARD_BYTES, "gamma": GOLDEN_GAMMA, "pages8k": [], "pages4k": []}
    for r in range(nshard):
        data = O.splitmix64(SHARD_BYTES // 8, shard_state(r)).view(np.uint8)
        for name, pb, seed in (("pages8k", 8192, 0xFDBEEFDB), ("pages4k", 4096, 0)):
            n = SHARD_BYTES // pb
            cuts = [n * k // threads for k in range(threads + 1)]
            with ThreadPoolExecutor(threads) as pool:
                parts = list(pool.map(lambda k: O.reference_batch_fixed(data[cuts[k] * pb:], pb, pb, cuts[k + 1] - cuts[k],
                                                                         seed=seed), range(threads)))
            c = np.concatenate(parts)
            out[name].append(dict(S.digest(c), rank=r, state=shard_state(r), count=n, page_bytes=pb, seed=seed))
            print(name, r, hex(out[name][-1]["xor"]), flush=True)
        del data
    g["pages_shards"] = out


def main():
    if "--shards" in sys.argv:
        with open(OUT) as fh:
            g = json.load(fh)
        pages_shards(g)
        with open(OUT, "w") as fh:
            json.dump(g, fh, separators=(",", ":"))
        print("updated pages_shards in", OUT)
        return
    if "--varlen" in sys.argv:
        with open(OUT) as fh:
            g = json.load(fh)
        varlen_full(g)
        with open(OUT, "w") as fh:
            json.dump(g, fh, separators=(",", ":"))
        print("updated varlen_full in", OUT)
        return
    ref = O.reference()
    crc = ref.append
    g = {"generator": "splitmix64: word k = mix(state + (k+1)*0x9E3779B97F4A7C15), little-endian u64",
         "source": "oracle/_ref/libcrc32c_ref.so = /root/reference/contrib/crc32/crc32c.cpp (unmodified)"}

    # --- known-answer tests (RFC 3720 B.4 + the classic check value)
    kats = []
    def kat(name, data, seed=0):
        kats.append({"name": name, "hex": bytes(data).hex(), "seed": seed, "crc": crc(seed, bytes(data))})
    kat("check-123456789", b"123456789")
    kat("rfc3720-zeros32", bytes(32))
    kat("rfc3720-ones32", b"\xff" * 32)
    kat("rfc3720-incr32", bytes(range(32)))
    kat("rfc3720-decr32", bytes(range(31, -1, -1)))
    kat("empty-seed0", b"")
    kat("empty-seed-fdbeefdb", b"", 0xFDBEEFDB)
    kat("single-a", b"a")
    kat("fdb", b"foundationdb", 0xFDBEEFDB)
    g["kat"] = kats

    # --- closed-form pages named in SURVEY §8c
    legacy = bytes(((i * 37 + 11) & 0xFF) for i in range(4088))  # KeyValueStoreSQLite.cpp:258-292 test page body
    g["pattern"] = [
        {"name": "sqlite-legacy-test-page", "pattern": "i*37+11", "length": 4088, "seed": 0xFDBEEFDB,
         "crc": crc(0xFDBEEFDB, legacy)},
        {"name": "zeros4096-seed0", "pattern": "zero", "length": 4096, "seed": 0, "crc": crc(0, bytes(4096))},
        {"name": "zeros4096-writechecker", "pattern": "zero", "length": 4096, "seed": 0xAB12FD93,
         "crc": crc(0xAB12FD93, bytes(4096))},
        {"name": "zeros4096-fdbeefdb", "pattern": "zero", "length": 4096, "seed": 0xFDBEEFDB,
         "crc": crc(0xFDBEEFDB, bytes(4096))},
        {"name": "diskqueue-v1-zero-page", "pattern": "zero", "length": 4092, "seed": 0xFDBEEFDB,
         "crc": crc(0xFDBEEFDB, bytes(4092))},
        {"name": "iota4096", "pattern": "i&255", "length": 4096, "seed": 0,
         "crc": crc(0, bytes(i & 255 for i in range(4096)))},
        {"name": "iota8192", "pattern": "i&255", "length": 8192, "seed": 0,
         "crc": crc(0, bytes(i & 255 for i in range(8192)))},
    ]

    # --- edge grid: every misalignment 0..15 x length 0..130 x seeds
    edge_state = 0xC0FFEE
    data = sm_bytes(4096, edge_state)
    grid = []
    for s in SEEDS:
        grid.append([[crc(s, data[off:off + n]) for n in range(131)] for off in range(16)])
    g["edge"] = {"state": edge_state, "nbytes": 4096, "offsets": 16, "max_len": 130, "seeds": SEEDS, "crc": grid}

    # --- threshold lengths around the reference's interleave boundaries
    # (3*SHORT_SHIFT=768, 3*LONG_SHIFT=24576) and the GPU's 1 KiB rows / 16 B chunks
    th_state = 0xBADC0DE
    th_data = sm_bytes((1 << 20) + 64, th_state)
    lens = sorted(set([0, 1, 3, 4, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 257, 767, 768, 769,
                       1008, 1023, 1024, 1025, 1040, 2047, 2048, 2049, 4087, 4088, 4092, 4095, 4096, 4097, 8191,
                       8192, 8193, 16384, 24575, 24576, 24577, 49152, 65535, 65536, 65537, 262144,
                       (1 << 20) - 1, 1 << 20]))
    th = []
    for off in (0, 1, 3, 7, 8, 13, 16, 33):
        for n in lens:
            for s in (0, 0xFDBEEFDB):
                th.append([off, n, s, crc(s, th_data[off:off + n])])
    g["threshold"] = {"state": th_state, "nbytes": len(th_data), "cases": th}

    # --- the BASELINE.md page batch (configs[0]): 65536 x 4 KiB, state 0x5EED
    pages = O.splitmix64(512 * 65536, 0x5EED).view(np.uint8)
    pb = {"state": 0x5EED, "page_bytes": 4096, "count": 65536, "digests": []}
    for s in (0, 0xFDBEEFDB, 0xAB12FD93):
        c = np.array([crc(s, pages[4096 * i:4096 * (i + 1)]) for i in range(65536)], dtype=np.uint32)
        pb["digests"].append(dict(S.digest(c), seed=s, first64=[int(x) for x in c[:64]]))
    # 8 KiB sqlite-sized pages over the same bytes
    c8 = np.array([crc(0xFDBEEFDB, pages[8192 * i:8192 * (i + 1)]) for i in range(32768)], dtype=np.uint32)
    pb["digest_8k_fdbeefdb"] = S.digest(c8)
    # 4088 / 4092 B sub-page regions (SQLite legacy codec, DiskQueue V1)
    c4088 = np.array([crc(0xFDBEEFDB, pages[4096 * i:4096 * i + 4088]) for i in range(65536)], dtype=np.uint32)
    c4092 = np.array([crc(0xFDBEEFDB, pages[4096 * i + 4:4096 * (i + 1)]) for i in range(65536)], dtype=np.uint32)
    pb["digest_4088_fdbeefdb"] = S.digest(c4088)
    pb["digest_4092_at4_fdbeefdb"] = S.digest(c4092)
    g["pages"] = pb

    # --- BASELINE configs[1] at full size: 1 Mi x 4 KiB (4 GiB), same stream
    big = O.splitmix64(512 * (1 << 20), 0x5EED).view(np.uint8)
    full = {"state": 0x5EED, "page_bytes": 4096, "count": 1 << 20, "digests": []}
    for s in (0, 0xFDBEEFDB):
        c = O.reference_batch_fixed(big, 4096, 4096, 1 << 20, seed=s)
        full["digests"].append(dict(S.digest(c), seed=s))
    c = O.reference_batch_fixed(big, 8192, 8192, 1 << 19, seed=0xFDBEEFDB)
    full["digest_8k_fdbeefdb"] = dict(S.digest(c), count=1 << 19)
    del big
    g["pages_full"] = full

    # --- FileTransfer-style chained CRC over 8 KiB reads (fdbrpc/FileTransfer.cpp:29-37)
    ch = 0
    for i in range(0, 1 << 20, 8192):
        ch = crc(ch, th_data[i:i + 8192])
    g["chained"] = {"state": th_state, "nbytes": 1 << 20, "read": 8192, "seed": 0, "crc": ch,
                    "oneshot": crc(0, th_data[:1 << 20])}

    varlen_full(g)
    pages_shards(g)

    with open(OUT, "w") as fh:
        json.dump(g, fh, separators=(",", ":"))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
