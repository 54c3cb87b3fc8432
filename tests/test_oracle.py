"""The CPU oracle (our restatement of contrib/crc32) against the reference's own outputs."""
import json
import os

import numpy as np
import pytest

import bench_shapes as S
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sm_bytes(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


def test_kats(golden, oracle_mod):
    for k in golden["kat"]:
        data = bytes.fromhex(k["hex"])
        assert O.crc32c(k["seed"], data) == k["crc"], k["name"]
        assert O.crc32c_bitwise(k["seed"], data) == k["crc"], k["name"]
    names = {k["name"]: k["crc"] for k in golden["kat"]}
    # published check values (RFC 3720 B.4 and the CRC-32C catalogue check value)
    assert names["check-123456789"] == 0xE3069283
    assert names["rfc3720-zeros32"] == 0x8A9136AA
    assert names["rfc3720-ones32"] == 0x62A8AB43
    assert names["rfc3720-incr32"] == 0x46DD794E
    assert names["rfc3720-decr32"] == 0x113FDB5C


def _pattern(p, n):
    if p == "zero":
        return bytes(n)
    if p == "i&255":
        return bytes(i & 255 for i in range(n))
    if p == "i*37+11":
        return bytes(((i * 37 + 11) & 0xFF) for i in range(n))
    raise ValueError(p)


def test_patterns(golden, oracle_mod):
    for e in golden["pattern"]:
        assert O.crc32c(e["seed"], _pattern(e["pattern"], e["length"])) == e["crc"], e["name"]
    legacy = [e for e in golden["pattern"] if e["name"] == "sqlite-legacy-test-page"][0]
    assert legacy["crc"] == 0x23E52E01


def test_edge_grid(golden, oracle_mod):
    e = golden["edge"]
    data = sm_bytes(e["nbytes"], e["state"])
    for si, s in enumerate(e["seeds"]):
        for off in range(e["offsets"]):
            for n in range(e["max_len"] + 1):
                assert O.crc32c(s, data[off:off + n]) == e["crc"][si][off][n], (s, off, n)


def test_edge_grid_bitwise_subset(golden, oracle_mod):
    e = golden["edge"]
    data = sm_bytes(e["nbytes"], e["state"])
    for si, s in enumerate(e["seeds"]):
        for off in (0, 5, 15):
            for n in range(0, e["max_len"] + 1, 7):
                assert O.crc32c_bitwise(s, data[off:off + n]) == e["crc"][si][off][n]


def test_thresholds(golden, oracle_mod):
    t = golden["threshold"]
    data = sm_bytes(t["nbytes"], t["state"])
    for off, n, s, want in t["cases"]:
        assert O.crc32c(s, data[off:off + n]) == want, (off, n, s)


def test_page_batch_digests(golden, oracle_mod):
    pb = golden["pages"]
    pages = O.splitmix64(512 * pb["count"], pb["state"]).view(np.uint8)
    for d in pb["digests"]:
        c = O.batch_fixed(pages, 4096, 4096, pb["count"], seed=d["seed"])
        assert S.digest(c) == S.pinned(d)
        assert [int(x) for x in c[:64]] == d["first64"]
    # SURVEY §8c / BASELINE.md published digest of this batch at seed 0
    d0 = [d for d in pb["digests"] if d["seed"] == 0][0]
    assert d0["xor"] == 0xC18E0D85 and d0["sum"] == 0x0000807AFF89425D
    assert d0["first64"][0] == 0x076DE509 and d0["first64"][1] == 0x808DD38F
    c8 = O.batch_fixed(pages, 8192, 8192, pb["count"] // 2, seed=0xFDBEEFDB)
    assert S.digest(c8) == S.pinned(pb["digest_8k_fdbeefdb"])
    c4088 = O.batch_fixed(pages, 4096, 4088, pb["count"], seed=0xFDBEEFDB)
    assert S.digest(c4088) == S.pinned(pb["digest_4088_fdbeefdb"])
    c4092 = O.batch_fixed(pages[4:], 4096, 4092, pb["count"], seed=0xFDBEEFDB)
    assert S.digest(c4092) == S.pinned(pb["digest_4092_at4_fdbeefdb"])


def test_digest_pins_catch_compensating_errors(golden, oracle_mod):
    """The full-size pins hold a sha256 of the whole result array: two swapped
    checksums (xor and sum unchanged) or a pair of errors that cancel in both
    still fail the comparison."""
    pb = golden["pages"]
    pages = O.splitmix64(512 * pb["count"], pb["state"]).view(np.uint8)
    d = pb["digests"][0]
    c = O.batch_fixed(pages, 4096, 4096, pb["count"], seed=d["seed"])
    assert S.digest(c) == S.pinned(d)
    swapped = c.copy()
    swapped[[10, 20]] = swapped[[20, 10]]
    assert S.digest(swapped)["xor"] == d["xor"] and S.digest(swapped)["sum"] == d["sum"]
    assert S.digest(swapped) != S.pinned(d)
    # every full-size entry carries the array hash
    for e in (golden["pages_full"]["digests"] + [golden["pages_full"]["digest_8k_fdbeefdb"]] +
              golden["pages_shards"]["pages4k"] + golden["pages_shards"]["pages8k"] +
              golden["varlen_full"]["zipf"]["digests"] + golden["varlen_full"]["chunks"]["digests"] +
              golden["varlen_full"]["zipf-scattered"]["digests"]):
        assert len(e["sha256"]) == 64


def test_chained_equals_oneshot(golden, oracle_mod):
    c = golden["chained"]
    data = sm_bytes(c["nbytes"] + 64, c["state"])[:c["nbytes"]]
    crc = 0
    for i in range(0, c["nbytes"], c["read"]):
        crc = O.crc32c(crc, data[i:i + c["read"]])
    assert crc == c["crc"] == c["oneshot"] == O.crc32c(0, data)


def test_combine_and_shift_identities(oracle_mod):
    rng = np.random.default_rng(7)
    for _ in range(200):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert O.combine(O.crc32c(s, a), O.crc32c(0, b), len(b)) == O.crc32c(s, a + b)
        # seed linearity: crc(s,M) ^ crc(0,M) depends only on (s, |M|)
        assert O.crc32c(s, b) ^ O.crc32c(0, b) == O.crc32c(s, bytes(len(b))) ^ O.crc32c(0, bytes(len(b)))


@pytest.mark.skipif(not O.reference_available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_matches_compiled_reference_random():
    ref = O.reference()
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 300_000, dtype=np.uint8)
    for _ in range(3000):
        off = int(rng.integers(0, 64))
        n = int(rng.integers(0, 70_000)) if rng.random() < 0.9 else int(rng.integers(0, 299_000))
        n = min(n, buf.size - off)
        s = int(rng.integers(0, 2**32))
        assert O.crc32c(s, buf[off:off + n]) == ref.append(s, buf[off:off + n])


@pytest.mark.parametrize("name", ["zipf", "chunks", "zipf-scattered"])
def test_oracle_varlen_configs_exact_batches(oracle_mod, golden, name):
    """The oracle reproduces the reference's digests of the exact configs[2] /
    configs[4] batches (and the shape generator still yields the pinned list)."""
    O = oracle_mod
    ent = golden["varlen_full"][name]
    lengths, offsets, extent = S.shape(name)
    assert S.lengths_digest(lengths) == ent["lengths_sha256"]
    data = O.splitmix64(extent // 8, ent["state"]).view(np.uint8)
    d = ent["digests"][1]
    got = O.batch_varlen(data, offsets, lengths, seed=d["seed"])
    assert S.digest(got) == S.pinned(d)
    assert [int(x) for x in got[:64]] == d["first64"]


def test_oracle_chained_matches_reference_file_transfer(golden, oracle_mod):
    """O.chained (the test oracle of crc32c_gpu_batch_chained) reproduces the
    reference's own FileTransfer-style chained CRC fixture."""
    c = golden["chained"]
    data = sm_bytes(c["nbytes"] + 64, c["state"])
    offs = list(range(0, c["nbytes"], c["read"]))
    lens = [min(c["read"], c["nbytes"] - o) for o in offs]
    assert int(O.chained(data, offs, lens, [0, len(offs)], seed=c["seed"])[0]) == c["crc"]
    assert int(O.chained(data, [0], [c["nbytes"]], [0, 1])[0]) == c["oneshot"] == c["crc"]


def test_shard_generator_jump_and_shard_digests():
    """configs[3]: rank r checksums bytes [r*4 GiB, (r+1)*4 GiB) of one splitmix64
    file, generated by jumping the generator (bench_shapes.shard_state); the jump
    is exact (checked at small word offsets against the continuous stream), and
    shard 0 of the reference-generated shard digests is the full-size page batch
    (tests/golden pages_shards vs pages_full)."""
    whole = O.splitmix64(4096, S.STATE)
    for w in (1, 7, 512, 3000):
        st = (S.STATE + w * S.GOLDEN_GAMMA) & 0xFFFFFFFFFFFFFFFF
        assert np.array_equal(O.splitmix64(64, st), whole[w:w + 64])
    assert S.shard_state(0) == S.STATE
    assert S.shard_state(3) == (S.STATE + 3 * (S.SHARD_BYTES // 8) * S.GOLDEN_GAMMA) % (1 << 64)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")))
    sh, full = g["pages_shards"], g["pages_full"]
    assert len(sh["pages8k"]) == 8 and len(sh["pages4k"]) == 8
    assert [d["state"] for d in sh["pages8k"]] == [S.shard_state(r) for r in range(8)]
    d0 = [d for d in full["digests"] if d["seed"] == 0][0]
    assert S.pinned(sh["pages4k"][0]) == S.pinned(d0)
    assert S.pinned(sh["pages8k"][0]) == S.pinned(full["digest_8k_fdbeefdb"])
    assert len({d["xor"] for d in sh["pages8k"]}) == 8  # the shards differ
