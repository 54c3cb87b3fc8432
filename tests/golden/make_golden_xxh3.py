"""Generate tests/golden/xxh3_golden.json from the REFERENCE implementation.

Runs FoundationDB's own flow/xxhash.c (xxHash v0.8.0) and flow/Hash3.c
(lookup3), compiled unmodified by oracle/Makefile into
oracle/_ref/libxxhash_ref.so.  Inputs are described, not stored: data are
splitmix64 streams (same generator as crc32c_golden.json), so the JSON holds
parameters and the reference's outputs only.

Usage (in the container that has /root/reference):
    make -C oracle && python tests/golden/make_golden_xxh3.py [--varlen]
(--varlen: only (re)compute the varlen_full section, keeping the rest.)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
import bench_shapes as S  # noqa: E402  (digest64: xor, sum and sha256 of a whole result array)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xxh3_golden.json")
SEEDS = [0, 0xFDBEEFDB, 0x8000000000000005, 0x0123456789ABCDEF]
LENGTHS = list(range(0, 300)) + [511, 512, 513, 1023, 1024, 1025, 1088, 2047, 2048, 4087, 4088, 4092, 4096,
                                 8192, 10000, 65536, 1 << 20]


def sm_bytes(nbytes, state):
    w = O.splitmix64((nbytes + 7) // 8, state)
    return w.view(np.uint8)[:nbytes].copy()


def varlen_full(g):
    """BASELINE configs[2] (Zipf packets) and configs[4] (backup chunks) at the
    exact bench shapes (bench_shapes.py), the bytes bench.py hashes (splitmix64,
    bench_shapes.STATE): the reference's XXH3_64bits over every buffer, and
    XXH3_64bits_withSeed with per-buffer seeds (bench_shapes.xxh3_seeds), as xor/sum/sha256 digests
    plus the first 64 digests."""
    import ctypes
    L = O.xxh3_reference()
    f = L.XXH3_64bits_withSeed
    out = {}
    for name in ("zipf", "chunks"):
        lengths, offsets, extent = S.shape(name)
        data = O.splitmix64(extent // 8, S.STATE).view(np.uint8)
        ent = {"state": S.STATE, "count": int(lengths.size), "lengths_sha256": S.lengths_digest(lengths),
               "digests": []}
        plain = O.ref_xxh3_batch_varlen(data, offsets, lengths)
        sd = S.xxh3_seeds(lengths.size)
        base = data.ctypes.data
        seeded = np.array([f(ctypes.c_void_p(base + int(o)), int(n), int(s))
                           for o, n, s in zip(offsets, lengths, sd)], dtype=np.uint64)
        for kind, h in (("seed0", plain), ("seeds", seeded)):
            ent["digests"].append(dict(S.digest64(h), kind=kind, first64=["%016x" % int(v) for v in h[:64]]))
        out[name] = ent
        del data
    g["varlen_full"] = out


def main():
    if "--varlen" in sys.argv:
        with open(OUT) as fh:
            g = json.load(fh)
        varlen_full(g)
        with open(OUT, "w") as fh:
            json.dump(g, fh, indent=0)
        print("wrote", OUT, os.path.getsize(OUT), "bytes")
        return
    g = {"generator": "splitmix64 (see crc32c_golden.json)",
         "source": "oracle/_ref/libxxhash_ref.so = /root/reference/flow/xxhash.c + flow/Hash3.c (unmodified)"}
    data = sm_bytes((1 << 20) + 64, 0x5EED)
    # --- lengths x offsets x seeds: digest lists
    grid = []
    for off in (0, 3, 8):
        for seed in SEEDS:
            h = [O.ref_xxh3_64(data[off:off + L], seed) for L in LENGTHS]
            grid.append({"offset": off, "seed": seed, "xxh3": ["%016x" % v for v in h]})
    g["lengths"] = LENGTHS
    g["grid"] = grid
    # --- 4 KiB pages of the splitmix stream (state 0x5EED): SQLite (4088 B at +0),
    # DiskQueue V2 (4088 B at +8), Redwood-style seeded (seed = page index)
    npg = 65536
    pages = sm_bytes(npg * 4096, 0x5EED)
    sq = O.ref_xxh3_batch_fixed(pages, 4096, 4088, npg)
    dq = O.ref_xxh3_batch_fixed(pages[8:], 4096, 4088, npg - 1)
    L = O.xxh3_reference()
    rw = np.array([L.XXH3_64bits_withSeed(pages.ctypes.data + 4096 * i, 4096, i) for i in range(0, npg, 16)],
                  dtype=np.uint64)
    digest = S.digest64
    g["pages"] = {"count": npg, "state": 0x5EED,
                  "sqlite_4088": dict(digest(sq), first=["%016x" % v for v in sq[:4]]),
                  "diskqueue_4088_at8": dict(digest(dq), count=npg - 1),
                  "redwood_seeded_4096_every16": digest(rw)}
    # --- the bench's full config: 1 Mi pages, SQLite layout, seed 0 (digests only)
    full = sm_bytes((1 << 20) * 4096, 0x5EED)
    fq = O.ref_xxh3_batch_fixed(full, 4096, 4088, 1 << 20)
    g["pages_full"] = dict(digest(fq), count=1 << 20, length=4088, stride=4096)
    del full
    # --- lookup3 hashlittle2: the reference's own known answers (flow/Hash3.c:1248-1263)
    # and pages with the SQLite / DiskQueue initial values
    s = b"Four score and seven years ago"
    kat = []
    for pc, pb in ((0, 0), (0, 0xdeadbeef), (0xdeadbeef, 0xdeadbeef)):
        kat.append({"hex": "", "pc": pc, "pb": pb, "out": list(O.ref_hashlittle2(b"", pc, pb))})
    for pc, pb in ((0, 0), (0, 1), (1, 0)):
        kat.append({"hex": s.hex(), "pc": pc, "pb": pb, "out": list(O.ref_hashlittle2(s, pc, pb))})
    hl = []
    for i in range(64):
        pg = pages[4096 * i:4096 * (i + 1)]
        hl.append({"page": i, "sqlite": list(O.ref_hashlittle2(pg[:4088], i + 1, 0x5ca1ab1e)),
                   "diskqueue": list(O.ref_hashlittle2(pg[16:], 0x12345678, 0xbeefabcd))})
    g["hashlittle2"] = {"kat": kat, "pages": hl}
    varlen_full(g)
    with open(OUT, "w") as f:
        json.dump(g, f, indent=0)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
