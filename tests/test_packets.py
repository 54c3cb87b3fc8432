"""Batched FlowTransport receive verification (include/fdb_packets.h) against
scanPackets (fdbrpc/FlowTransport.cpp:1260-1366).

CPU: the C restatement (oracle/packets_oracle.c) over our XXH3 restatement
and over the reference's own flow/xxhash.c agree, and both agree with a
line-by-line Python model, on receive buffers built to hit every exit of the
walk: clean runs of frames, a tail cut inside the length word, the checksum
or the payload, a payload corrupted with the reference's bit-flip injection
(:1321-1343), frames shorter than sizeof(UID), lengths over PACKET_LIMIT
(also on incomplete frames, which the reference rejects before waiting for
the bytes), checksums off (TLS peers, :1275), empty and 1-3 byte buffers.
GPU: fdb_packets_verify_ws gives the oracle's outcome for every buffer, and
its frame list holds exactly the frames the walk found."""
import numpy as np
import pytest

from oracle import oracle as O

PACKET_LIMIT = 100 << 20


def scan_model(buf, checksum, limit):
    """FlowTransport.cpp:1273-1366, one buffer (bytes), pure Python."""
    p, begin, n = 0, 0, 0
    e = len(buf)
    while True:
        if e - p < 4:
            return begin, n, 0
        L = int.from_bytes(buf[p:p + 4], "little")
        p += 4
        ck = 0
        if checksum:
            if e - p < 8:
                return begin, n, 0
            ck = int.from_bytes(buf[p:p + 8], "little")
            p += 8
        if L > limit:
            return begin, n, 2
        if e - p < L:
            return begin, n, 0
        if L < 16:
            return begin, n, 3
        if checksum and O.xxh3_64(buf[p:p + L]) != ck:
            return begin, n, 1
        p += L
        begin = p
        n += 1


def frame(payload, checksum=True, length=None, ck=None):
    L = len(payload) if length is None else length
    h = L.to_bytes(4, "little")
    if checksum:
        c = O.xxh3_64(payload) if ck is None else ck
        h += int(c).to_bytes(8, "little")
    return h + bytes(payload)


def flip_bits(rng, payload):
    """The reference's simulated corruption (FlowTransport.cpp:1330-1343):
    32 - floor(log2(u32)) bit flips, the first always applied, later ones
    skipped where they would undo the first."""
    b = bytearray(payload)
    u = int(rng.integers(1, 2**32))
    flips = 32 - int(np.floor(np.log2(u)))
    n = len(b)
    fb, fbit = int(rng.integers(0, 2**32)) % n, int(rng.integers(0, 8))
    b[fb] ^= 1 << fbit
    for _ in range(flips - 1):
        bl, bit = int(rng.integers(0, 2**32)) % n, int(rng.integers(0, 8))
        if bl != fb or bit != fbit:
            b[bl] ^= 1 << bit
    return bytes(b)


def build_buffers(seed, nbuf=120, checksum=True, limit=PACKET_LIMIT, big=False):
    """Receive buffers that end every way scanPackets can stop."""
    rng = np.random.default_rng(seed)
    bufs, kinds = [], []
    sizes = [16, 17, 31, 64, 100, 240, 241, 1000, 1024, 4096, 16384, 16385] + ([70000, 200000] if big else [])

    def payload(L):
        return rng.integers(0, 256, L, dtype=np.uint8).tobytes()

    for i in range(nbuf):
        kind = i % 10
        nf = int(rng.integers(0, 12))
        fr = []
        for _ in range(nf):
            L = int(rng.choice(sizes)) if rng.random() < 0.5 else int(rng.integers(16, 3000))
            fr.append(frame(payload(L), checksum))
        body = b"".join(fr)
        if kind == 1 and checksum and nf:  # a corrupted payload somewhere
            j = int(rng.integers(0, nf))
            raw = fr[j]
            hdr = 12
            fr[j] = raw[:hdr] + flip_bits(rng, raw[hdr:])
            body = b"".join(fr)
        elif kind == 2:  # tail cut inside the next frame: length word, checksum, payload
            nxt = frame(payload(int(rng.integers(16, 5000))), checksum)
            body += nxt[: int(rng.integers(0, len(nxt)))]
        elif kind == 3:  # a frame shorter than sizeof(UID)
            body += frame(payload(int(rng.integers(0, 16))), checksum) + frame(payload(40), checksum)
        elif kind == 4:  # a length over the limit, complete or not
            L = limit + int(rng.integers(1, 1000))
            body += L.to_bytes(4, "little") + (b"\0" * 8 if checksum else b"") + payload(int(rng.integers(0, 64)))
        elif kind == 5:  # a wrong stored checksum
            if checksum:
                body += frame(payload(300), checksum, ck=12345)
        elif kind == 6:
            body = body[: int(rng.integers(0, 4))] if rng.random() < 0.5 else b""
        elif kind == 7:  # garbage after good frames
            body += payload(int(rng.integers(0, 40)))
        bufs.append(body)
        kinds.append(kind)
    return bufs, kinds


def pack(bufs, rng, align_any=True):
    """All buffers in one byte array at random alignments (gaps of junk)."""
    parts, offs, pos = [], [], 0
    for b in bufs:
        g = int(rng.integers(0, 40)) if align_any else (-pos) % 16
        parts.append(rng.integers(0, 256, g, dtype=np.uint8).tobytes())
        pos += g
        offs.append(pos)
        parts.append(b)
        pos += len(b)
    parts.append(bytes(64))
    mem = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return mem, np.array(offs, np.uint64), np.array([len(b) for b in bufs], np.uint64)


@pytest.mark.parametrize("checksum", [True, False])
def test_oracle_matches_model(checksum):
    bufs, _ = build_buffers(11 + checksum, nbuf=80, checksum=checksum, limit=5000)
    mem, offs, lens = pack(bufs, np.random.default_rng(3))
    c, f, s = O.packets_verify(mem, offs, lens, checksum=checksum, packet_limit=5000)
    for i, b in enumerate(bufs):
        assert (int(c[i]), int(f[i]), int(s[i])) == scan_model(b, checksum, 5000), i
    # every outcome occurs
    if checksum:
        assert set(s.tolist()) == {0, 1, 2, 3}


@pytest.mark.skipif(not O.packets_reference_available(), reason="oracle/_ref not built")
def test_oracle_matches_reference_xxh3():
    bufs, _ = build_buffers(5, nbuf=200, big=True)
    mem, offs, lens = pack(bufs, np.random.default_rng(9))
    a = O.packets_verify(mem, offs, lens)
    b = O.packets_verify(mem, offs, lens, ref=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.fixture(scope="module")
def cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import foundationdb_amd as F
    F.gpu_init()
    return torch.device("cuda:0")


def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64) if a.dtype == np.uint64 else a).to(cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("checksum", [True, False])
def test_gpu_packets_match_oracle(cuda, checksum):
    import foundationdb_amd.packets as PK
    limit = 1 << 20
    bufs, kinds = build_buffers(21 + checksum, nbuf=600, checksum=checksum, limit=limit, big=True)
    rng = np.random.default_rng(17)
    mem, offs, lens = pack(bufs, rng)
    want_c, want_f, want_s = O.packets_verify(mem, offs, lens, checksum=checksum, packet_limit=limit)
    total = int(lens.sum())
    V = PK.PacketVerifier(cuda, len(bufs), total // 28 + len(bufs), total)
    d = _dev(mem, cuda)
    V.verify(d, _dev(offs, cuda), _dev(lens, cuda), checksum=checksum, packet_limit=limit)
    got = V.results_numpy()
    assert np.array_equal(got["frames"], want_f)
    assert np.array_equal(got["status"], want_s)
    assert np.array_equal(got["consumed"], want_c)
    # the frame list: every frame the walk found, payload located and checksum copied
    fr = V.frames_numpy()
    per = {}
    for r in fr:
        per.setdefault(int(r["buffer"]), []).append(r)
    for b, lst in per.items():
        lst.sort(key=lambda r: int(r["ordinal"]))
        assert [int(r["ordinal"]) for r in lst] == list(range(len(lst)))
        assert len(lst) >= int(want_f[b])
        pos = int(offs[b])
        hdr = 12 if checksum else 4
        for r in lst:
            L = int.from_bytes(mem[pos:pos + 4].tobytes(), "little")
            assert int(r["offset"]) == pos + hdr and int(r["length"]) == L
            pos += hdr + L
    assert sum(len(v) for v in per.values()) == fr.size


@pytest.mark.gpu
def test_gpu_packets_capacity_and_empty(cuda):
    """A frame list too small for the batch marks exactly the buffers whose
    frames did not fit (FDB_PACKET_ECAPACITY); buffers that fit are exact.
    Zero buffers is a no-op; empty buffers consume nothing."""
    import torch
    import foundationdb_amd.packets as PK
    bufs = [b"".join(frame(np.full(100, i % 256, np.uint8).tobytes()) for _ in range(50)) for i in range(8)]
    bufs.append(b"")
    mem, offs, lens = pack(bufs, np.random.default_rng(1))
    want = O.packets_verify(mem, offs, lens)
    V = PK.PacketVerifier(cuda, len(bufs), 120, int(lens.sum()))
    V.verify(_dev(mem, cuda), _dev(offs, cuda), _dev(lens, cuda))
    got = V.results_numpy()
    cap = got["status"] == PK.ECAPACITY
    assert cap.any() and (~cap).any()
    ok = ~cap
    assert np.array_equal(got["frames"][ok], want[1][ok])
    assert np.array_equal(got["consumed"][ok], want[0][ok])
    assert got["consumed"][-1] == 0 and got["status"][-1] == 0
    e = torch.empty(0, dtype=torch.int64, device=cuda)
    V.verify(_dev(mem, cuda), e, e)


def walk_model(buf, checksum, limit):
    """The frames the walk finds in one buffer: scan_model without the checksum
    check (k_pkt_walk records every complete, well-sized frame)."""
    p, n, e = 0, 0, len(buf)
    hdr = 12 if checksum else 4
    while e - p >= hdr:
        L = int.from_bytes(buf[p:p + 4], "little")
        if L > limit or e - p - hdr < L or L < 16:
            break
        p += hdr + L
        n += 1
    return n


@pytest.mark.gpu
def test_gpu_packets_capacity_with_corrupt_frames(cuda):
    """A frame list too small for a batch that also holds corrupted frames:
    the buffers whose frames all fit get the oracle's outcome; a buffer that
    overflowed (fewer frames recorded than its walk found -- the recorded ones
    are always an ordinal prefix, the list being reserved in walk order) reports
    CHECKSUM_FAILED when a recorded frame failed (the oracle's frame count and
    consumed bytes), FDB_PACKET_ECAPACITY otherwise.  Every buffer checked."""
    import foundationdb_amd.packets as PK
    bufs, kinds = build_buffers(57, nbuf=400)
    mem, offs, lens = pack(bufs, np.random.default_rng(5))
    want = O.packets_verify(mem, offs, lens)
    assert (want[2] == PK.CHECKSUM_FAILED).sum() >= 20  # corrupted frames throughout the batch
    walked = np.array([walk_model(b, True, PACKET_LIMIT) for b in bufs])
    for cap in (1, 64, int(walked.sum()) // 2, int(walked.sum()) - 1):
        V = PK.PacketVerifier(cuda, len(bufs), cap, int(lens.sum()))
        V.verify(_dev(mem, cuda), _dev(offs, cuda), _dev(lens, cuda))
        got = V.results_numpy()
        fr = V.frames_numpy()
        assert fr.size == min(cap, int(walked.sum()))
        rec = np.bincount(fr["buffer"].astype(np.int64), minlength=len(bufs))
        for b in range(len(bufs)):
            ords = sorted(int(r["ordinal"]) for r in fr[fr["buffer"] == b])
            assert ords == list(range(rec[b]))  # an ordinal prefix
        over = rec < walked
        assert over.any() or cap >= walked.sum()
        for b in range(len(bufs)):
            if not over[b] or (want[2][b] == PK.CHECKSUM_FAILED and want[1][b] < rec[b]):
                assert (got["consumed"][b], got["frames"][b], got["status"][b]) == \
                    (want[0][b], want[1][b], want[2][b]), (cap, b)
            else:
                assert got["status"][b] == PK.ECAPACITY, (cap, b)


@pytest.mark.gpu
def test_gpu_packets_one_shot_matches(cuda):
    import foundationdb_amd.packets as PK
    bufs, _ = build_buffers(33, nbuf=300)
    mem, offs, lens = pack(bufs, np.random.default_rng(2))
    got = PK.verify_packets(_dev(mem, cuda), _dev(offs, cuda), _dev(lens, cuda))
    want = O.packets_verify(mem, offs, lens)
    assert np.array_equal(got["consumed"], want[0])
    assert np.array_equal(got["frames"], want[1])
    assert np.array_equal(got["status"], want[2])


@pytest.mark.gpu
@pytest.mark.parametrize("checksum", [True, False])
def test_gpu_packets_many_small_frames(cuda, checksum):
    """Buffers of up to ~150 minimum-size frames (many 8-step flush groups of
    the walk per lane, every lane of a wave ending at a different step), at
    random alignments, with the batch's last buffer -- a frame cut inside its
    header -- ending at the device array's last byte: the walk's one 16-byte
    header load is moved back near a buffer's end and must stay inside it."""
    import foundationdb_amd.packets as PK
    rng = np.random.default_rng(41 + checksum)
    bufs = []
    for i in range(300):
        n = int(rng.integers(0, 150))
        body = b"".join(frame(rng.integers(0, 256, int(rng.integers(16, 40)), dtype=np.uint8).tobytes(), checksum)
                        for _ in range(n))
        if i % 7 == 3:  # a cut frame after the run: its length word or checksum incomplete
            nxt = frame(rng.integers(0, 256, 20, dtype=np.uint8).tobytes(), checksum)
            body += nxt[: int(rng.integers(1, 12 if checksum else 4))]
        bufs.append(body)
    last = frame(rng.integers(0, 256, 30, dtype=np.uint8).tobytes(), checksum)
    bufs.append(b"".join(frame(rng.integers(0, 256, 17, dtype=np.uint8).tobytes(), checksum) for _ in range(9))
                + last[:7])
    mem, offs, lens = pack(bufs, rng)
    mem = mem[: int(offs[-1] + lens[-1])].copy()  # no bytes after the last buffer
    want_c, want_f, want_s = O.packets_verify(mem, offs, lens, checksum=checksum)
    total = int(lens.sum())
    V = PK.PacketVerifier(cuda, len(bufs), total // 20 + len(bufs), total)
    V.verify(_dev(mem, cuda), _dev(offs, cuda), _dev(lens, cuda), checksum=checksum)
    got = V.results_numpy()
    assert int(want_f.max()) > 100
    assert np.array_equal(got["frames"], want_f)
    assert np.array_equal(got["status"], want_s)
    assert np.array_equal(got["consumed"], want_c)
    fr = V.frames_numpy()
    assert fr.size == int(want_f.sum())
