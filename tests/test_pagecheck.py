"""Batched page verifiers (include/fdb_pagecheck.h) against the reference's
page checksum logic (oracle restatement on the pinned CRC-32C / XXH3 / lookup3
primitives) and the reference's own unit test
/fdbserver/kvstore/SQLite/PageChecksum/LegacyCRC32
(fdbserver/kvstore/KeyValueStoreSQLite.cpp:258-292)."""
import numpy as np
import pytest

from oracle import oracle as O


def sm_bytes(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


def legacy_page():
    page = np.zeros(4096, np.uint8)
    page[:4088] = (np.arange(4088) * 37 + 11) & 0xFF
    page[4088:] = np.frombuffer(O.sqlite_trailer_crc(page), np.uint8)
    return page


def test_oracle_follows_reference_legacy_crc32_test():
    page = legacy_page()
    assert O.sqlite_verify_page(page, 2) == 1
    page[4088 // 2] ^= 0xFF
    assert O.sqlite_verify_page(page, 2) == 0
    page[4088 // 2] ^= 0xFF
    assert O.sqlite_verify_page(page, 2) == 1
    page[4088:] = np.frombuffer(O.sqlite_trailer_xxh3(page), np.uint8)  # rewrite upgrades to xxHash3
    assert O.sqlite_verify_page(page, 2) == 2
    # golden trailer of the LegacyCRC32 page (0x23e52e01)
    assert int.from_bytes(O.sqlite_trailer_crc(legacy_page())[4:], "little") == 0x23E52E01


def make_sqlite_batch(n, page_size, first_pgno, seed):
    rng = np.random.default_rng(seed)
    pages = sm_bytes(n * page_size, seed).reshape(n, page_size)
    kinds = rng.integers(0, 7, n)
    for i in range(n):
        pg, k = pages[i], kinds[i]
        if k in (0, 4):
            pg[-8:] = np.frombuffer(O.sqlite_trailer_crc(pg), np.uint8)
        elif k in (1, 5):
            pg[-8:] = np.frombuffer(O.sqlite_trailer_xxh3(pg), np.uint8)
        elif k in (2, 6):
            pg[-8:] = np.frombuffer(O.sqlite_trailer_hl2(pg, first_pgno + i), np.uint8)
        if k >= 4:  # corrupt after writing: a data byte or a trailer byte
            j = int(rng.integers(0, page_size))
            pg[j] ^= 1 << int(rng.integers(0, 8))
        # k == 3: random trailer (almost surely corrupt)
    exp = np.array([O.sqlite_verify_page(pages[i], first_pgno + i) for i in range(n)], np.uint8)
    return pages, exp


def make_dq_batch(n, seed):
    rng = np.random.default_rng(seed)
    pages = sm_bytes(n * 4096, seed).reshape(n, 4096)
    for i in range(n):
        pg = pages[i]
        ver = int(rng.choice([0, 1, 2, 2, 2, 3]))
        pg[8:10] = np.frombuffer((0x1234).to_bytes(2, "little"), np.uint8)  # magic
        pg[10:12] = np.frombuffer(ver.to_bytes(2, "little"), np.uint8)
        if ver == 0:
            pg[8:10] = np.frombuffer((0x0FDB).to_bytes(2, "little"), np.uint8)
        pg[:16] = np.frombuffer(O.diskqueue_hash(pg, min(ver, 2)), np.uint8)
        if rng.random() < 0.3:
            j = int(rng.integers(0, 4096))
            pg[j] ^= 0x10
    exp = np.array([O.diskqueue_check_page(pages[i]) for i in range(n)], np.uint8)
    return pages, exp


@pytest.mark.skipif(not O.pagecheck_reference_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("page_size", [4096, 8192, 512])
def test_oracle_page_checks_match_reference_composition(page_size):
    """The oracle's page-format restatements agree, page by page, with
    oracle/ref_pagecheck.c: the same checks composed from the reference's own
    crc32c_append, XXH3_64bits and hashlittle2 compiled unmodified
    (KeyValueStoreSQLite.cpp:118-155, DiskQueue.cpp:1077-1120) -- the C
    baseline the verifier bench lines time."""
    pages, exp = make_sqlite_batch(600, page_size, 9, page_size + 1)
    st, bad = O.ref_sqlite_verify_pages(pages, page_size, 600, first_pgno=9)
    assert np.array_equal(st, exp) and bad == int((exp == 0).sum())
    dq, dexp = make_dq_batch(400, page_size)
    ok, dbad = O.ref_diskqueue_check_pages(dq, 400)
    assert np.array_equal(ok, dexp) and dbad == int((dexp == 0).sum())


def test_oracle_diskqueue_roundtrip():
    pages, exp = make_dq_batch(200, 3)
    assert 0 < exp.sum() < exp.size


@pytest.mark.gpu
@pytest.mark.parametrize("page_size", [4096, 8192, 512, 65536])
def test_gpu_sqlite_verify_mixed(cuda, page_size):
    import torch
    import foundationdb_amd.pagecheck as PC
    n = {4096: 3000, 8192: 800, 512: 4000, 65536: 64}[page_size]
    first = 7
    pages, exp = make_sqlite_batch(n, page_size, first, page_size)
    d = torch.from_numpy(pages.reshape(-1)).to(cuda)
    status, bad = PC.sqlite_verify_pages(d, page_size, first_pgno=first)
    got = status.cpu().numpy()
    assert np.array_equal(got, exp)
    assert int(bad.cpu().numpy().view(np.uint64)[0]) == int((exp == 0).sum())
    assert set(np.unique(exp)) >= {0, 1, 2, 3} or page_size == 65536


@pytest.mark.gpu
def test_gpu_sqlite_legacy_page_sequence(cuda):
    import torch
    import foundationdb_amd.pagecheck as PC
    page = legacy_page()
    bad = page.copy()
    bad[4088 // 2] ^= 0xFF
    up = page.copy()
    up[4088:] = np.frombuffer(O.sqlite_trailer_xxh3(up), np.uint8)
    d = torch.from_numpy(np.concatenate([page, bad, page, up])).to(cuda)
    status, nbad = PC.sqlite_verify_pages(d, 4096, first_pgno=2)
    assert status.cpu().tolist() == [1, 0, 1, 2]
    assert int(nbad.cpu().numpy().view(np.uint64)[0]) == 1


@pytest.mark.gpu
def test_gpu_diskqueue_check(cuda):
    import torch
    import foundationdb_amd.pagecheck as PC
    pages, exp = make_dq_batch(3000, 11)
    d = torch.from_numpy(pages.reshape(-1)).to(cuda)
    ok, bad = PC.diskqueue_check_pages(d)
    assert np.array_equal(ok.cpu().numpy(), exp)
    assert int(bad.cpu().numpy().view(np.uint64)[0]) == int((exp == 0).sum())


@pytest.mark.gpu
def test_gpu_pagecheck_all_one_kind_and_empty(cuda):
    import torch
    import foundationdb_amd.pagecheck as PC
    n = 2048
    pages = sm_bytes(n * 4096, 99).reshape(n, 4096)
    for i in range(n):
        pages[i, -8:] = np.frombuffer(O.sqlite_trailer_xxh3(pages[i]), np.uint8)
    d = torch.from_numpy(pages.reshape(-1)).to(cuda)
    status, bad = PC.sqlite_verify_pages(d, 4096)
    assert (status.cpu().numpy() == 2).all() and int(bad.cpu().numpy().view(np.uint64)[0]) == 0
    s0, b0 = PC.sqlite_verify_pages(d, 4096, count=0)
    assert s0.numel() == 0 and int(b0.cpu().numpy().view(np.uint64)[0]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [True, False])
def test_gpu_host_resident_verifiers(cuda, pinned):
    """Pages that start in host memory (a file scan reading from disk,
    KeyValueStoreSQLite.cpp:1378-1470; DiskQueue page runs, DiskQueue.cpp:1230-1290)
    through the pipeline: small segments so a batch spans many segments and
    every lane, pinned and pageable sources, blocking and submit/poll forms."""
    import torch
    import foundationdb_amd as F
    pages, exp = make_sqlite_batch(3000, 4096, 5, 41)
    dq, dq_exp = make_dq_batch(2500, 43)

    def host(a):
        if not pinned:
            return a.reshape(-1).copy()
        t = torch.empty(a.size, dtype=torch.uint8).pin_memory()
        t.numpy()[:] = a.reshape(-1)
        return t
    hp, hd = host(pages), host(dq)
    pipe = F.Pipeline(segment_bytes=1 << 20, nstreams=3)
    status, bad = pipe.sqlite_verify_pages(hp, 4096, first_pgno=5)
    assert np.array_equal(status, exp) and int(bad[0]) == int((exp == 0).sum())
    ok, bad = pipe.diskqueue_check_pages(hd)
    assert np.array_equal(ok, dq_exp) and int(bad[0]) == int((dq_exp == 0).sum())
    j1 = pipe.sqlite_verify_pages(hp, 4096, first_pgno=5, submit=True)
    j2 = pipe.diskqueue_check_pages(hd, submit=True)
    while not (j1.poll() and j2.poll()):
        pass
    assert np.array_equal(j1.result[0], exp) and np.array_equal(j2.result[0], dq_exp)
    assert int(j2.result[1][0]) == int((dq_exp == 0).sum())
    s0, b0 = pipe.sqlite_verify_pages(hp, 4096, count=0)
    assert s0.size == 0 and int(b0[0]) == 0
    pipe.close()


# ------------------------------------------------------------------ write side

def _dq_versions(n, seed):
    """4 KiB pages with implementationVersion 0 / 1 / 2 and a few unknown ones."""
    rng = np.random.default_rng(seed)
    pages = sm_bytes(n * 4096, seed).reshape(n, 4096)
    vers = rng.choice([0, 1, 2, 2, 3, 0xFFFF], n)
    for i in range(n):
        pages[i, 10:12] = np.frombuffer(int(vers[i]).to_bytes(2, "little"), np.uint8)
    return pages, vers


@pytest.mark.skipif(not O.pagecheck_reference_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("page_size", [512, 1024, 4096, 8192])
def test_oracle_seal_matches_reference_composition(page_size):
    """The seal restatements (oracle.sqlite_seal_pages / diskqueue_seal_pages)
    write the same bytes as the codec's page writes and Page::updateHash
    composed from the reference's own primitives (oracle/ref_pagecheck.c), and
    the sealed pages verify (status 2 for SQLite; DiskQueue V0-V2 ok, unknown
    versions rejected by checkHash although updateHash sealed them, as in the
    reference).  Batches starting at page 0, 1 and 2 cover page 1's extra
    1024-byte seal."""
    n = 24
    pages = sm_bytes(n * page_size, page_size + 3)
    for first in (0, 1, 2):
        want = O.ref_sqlite_seal_pages(pages, page_size, n, first)
        assert np.array_equal(O.sqlite_seal_pages(pages, page_size, n, first), want)
        st, bad = O.ref_sqlite_verify_pages(want, page_size, n, first)
        assert bad == 0 and (st == 2).all()
        i1 = 1 - first
        if 0 <= i1 < n and page_size > 1024:  # page 1 also verifies as a 1024-byte page
            p1 = want[i1 * page_size:i1 * page_size + 1024]
            assert O.sqlite_verify_page(p1, 1) == 2
    dq, vers = _dq_versions(64, page_size)
    want = O.ref_diskqueue_seal_pages(dq, 64)
    assert np.array_equal(O.diskqueue_seal_pages(dq, 64), want)
    ok, _ = O.ref_diskqueue_check_pages(want, 64)
    assert np.array_equal(ok, (vers <= 2).astype(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("page_size", [512, 4096, 8192, 65536])
def test_gpu_sqlite_seal_pages(cuda, page_size):
    """fdb_sqlite_seal_pages writes exactly the bytes the reference's codec
    composition writes (byte for byte, every page, first_pgno 0 / 1 / 5), and
    the verifier then accepts every page as XXH3-sealed."""
    import torch
    import foundationdb_amd.pagecheck as PC
    n = {512: 3000, 4096: 2000, 8192: 700, 65536: 40}[page_size]
    pages = sm_bytes(n * page_size, page_size + 17)
    for first, shift in ((0, 0), (1, 0), (5, 0), (1, 16)):
        # shift 16: pages off the 64-byte line grid (the trailer-only store form)
        want = O.ref_sqlite_seal_pages(pages, page_size, n, first) if O.pagecheck_reference_available() else \
            O.sqlite_seal_pages(pages, page_size, n, first)
        whole = torch.zeros(pages.size + shift, dtype=torch.uint8, device=cuda)
        d = whole[shift:]
        d.copy_(torch.from_numpy(pages))
        PC.sqlite_seal_pages(d, page_size, first_pgno=first)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        assert np.array_equal(got, want), (page_size, first, int(np.flatnonzero(got != want)[0]))
        status, bad = PC.sqlite_verify_pages(d, page_size, first_pgno=first)
        assert (status.cpu().numpy() == 2).all() and int(bad.cpu().numpy().view(np.uint64)[0]) == 0
        PC.sqlite_seal_pages(d, page_size, first_pgno=first)  # sealing again changes nothing
        assert np.array_equal(d.cpu().numpy(), want)


@pytest.mark.gpu
def test_gpu_diskqueue_seal_pages(cuda):
    """fdb_diskqueue_seal_pages = Page::updateHash per page (V0 / V1 / V2 and
    unknown versions, which take XXH3), byte for byte against the reference
    composition; seal-then-check accepts every V0-V2 page."""
    import torch
    import foundationdb_amd.pagecheck as PC
    n = 3000
    dq, vers = _dq_versions(n, 21)
    want = O.ref_diskqueue_seal_pages(dq, n) if O.pagecheck_reference_available() else O.diskqueue_seal_pages(dq, n)
    for shift in (16, 0):  # 16: off the 64-byte line grid (the hash-only store form)
        whole = torch.zeros(dq.size + shift, dtype=torch.uint8, device=cuda)
        d = whole[shift:]
        d.copy_(torch.from_numpy(dq.reshape(-1)))
        PC.diskqueue_seal_pages(d)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        assert np.array_equal(got, want.reshape(-1)), shift
    ok, bad = PC.diskqueue_check_pages(d)
    assert np.array_equal(ok.cpu().numpy(), (vers <= 2).astype(np.uint8))
    assert int(bad.cpu().numpy().view(np.uint64)[0]) == int((vers > 2).sum())
    # one kind only, and a single page
    for v in (0, 1, 2):
        one = dq[:5].copy()
        one[:, 10:12] = np.frombuffer(v.to_bytes(2, "little"), np.uint8)
        d1 = torch.from_numpy(one.reshape(-1).copy()).to(cuda)
        PC.diskqueue_seal_pages(d1)
        assert np.array_equal(d1.cpu().numpy(), O.diskqueue_seal_pages(one, 5))


@pytest.mark.gpu
@pytest.mark.parametrize("page_size", [1024, 4096])
def test_gpu_sqlite_codec_pages(cuda, page_size):
    """fdb_sqlite_codec_pages = PageChecksumCodec::codec per page: reads verify
    (status = the accepting check, 0 = nullptr), writes seal in place, the
    reserve-size rule leaves every page but page 1 untouched and refused, and
    any op other than 3 / 6 / 7 is refused."""
    import torch
    import foundationdb_amd.pagecheck as PC
    from foundationdb_amd.crc32c import CRC32CError
    n = 600
    rng = np.random.default_rng(page_size)
    raw = sm_bytes(n * page_size, page_size + 3).reshape(n, page_size)
    for first in (1, 2):
        for reserve in (8, 0):
            # writes (db page, journal page): sealed bytes and statuses against the per-page restatement
            for op in (6, 7):
                want = [O.sqlite_codec_page(raw[i], first + i, reserve, op) for i in range(n)]
                d = torch.from_numpy(raw.reshape(-1).copy()).to(cuda)
                st = PC.sqlite_codec_pages(d, page_size, op, reserve_size=reserve, first_pgno=first)
                torch.cuda.synchronize()
                assert np.array_equal(st.cpu().numpy(), np.array([w[0] for w in want], np.uint8)), (first, reserve, op)
                assert np.array_equal(d.cpu().numpy().reshape(n, page_size), np.stack([w[1] for w in want]))
            # reads of a mixed batch: sealed, legacy CRC, corrupt and untouched pages
            sealed = O.sqlite_seal_pages(raw, page_size, n, first).reshape(n, page_size)
            pages = raw.copy()
            kind = rng.integers(0, 4, n)
            pages[kind == 0] = sealed[kind == 0]
            for i in np.flatnonzero(kind == 1):
                pages[i, -8:] = np.frombuffer(O.sqlite_trailer_crc(pages[i]), np.uint8)
            for i in np.flatnonzero(kind == 2):
                pages[i] = sealed[i]
                pages[i, 100] ^= 0x20
            want = [O.sqlite_codec_page(pages[i], first + i, reserve, 3) for i in range(n)]
            d = torch.from_numpy(pages.reshape(-1).copy()).to(cuda)
            st = PC.sqlite_codec_pages(d, page_size, PC.CODEC_READ, reserve_size=reserve, first_pgno=first)
            torch.cuda.synchronize()
            assert np.array_equal(st.cpu().numpy(), np.array([w[0] for w in want], np.uint8)), (first, reserve)
            assert np.array_equal(d.cpu().numpy().reshape(n, page_size), pages)  # reads change nothing
    d = torch.from_numpy(raw.reshape(-1).copy()).to(cuda)
    for op in (0, 2, 5, 8):
        with pytest.raises(CRC32CError):
            PC.sqlite_codec_pages(d, page_size, op)


@pytest.mark.gpu
def test_gpu_verify_and_seal_replay_from_a_hip_graph(cuda):
    """The _ws forms launch without allocating or synchronising; their counters
    live in the stream's own words and every call's last kernel puts them back
    to zero, so a captured graph of a seal and two verifications replays
    correctly again and again (a counter left non-zero would shift every later
    list)."""
    import ctypes
    import torch
    import foundationdb_amd.pagecheck as PC
    L = PC._lib()
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.fdb_sqlite_verify_pages_ws.argtypes = [vp, u64, u64, u32, vp, vp, vp, u64, vp]
    L.fdb_diskqueue_check_pages_ws.argtypes = [vp, u64, vp, vp, vp, u64, vp]
    L.fdb_sqlite_seal_pages_ws.argtypes = [vp, u64, u64, u32, vp, u64, vp]
    pages, exp = make_sqlite_batch(1500, 4096, 3, 77)
    dq, dq_exp = make_dq_batch(1200, 78)
    raw = sm_bytes(700 * 4096, 79)
    sealed = O.sqlite_seal_pages(raw, 4096, 700, 1)
    d_sq = torch.from_numpy(pages.reshape(-1).copy()).to(cuda)
    d_dq = torch.from_numpy(dq.reshape(-1).copy()).to(cuda)
    d_raw = torch.from_numpy(raw.copy()).to(cuda)
    nws = int(L.fdb_pagecheck_workspace_bytes(1500))
    ws = torch.empty(nws, dtype=torch.uint8, device=cuda)
    st = torch.empty(1500, dtype=torch.uint8, device=cuda)
    ok = torch.empty(1200, dtype=torch.uint8, device=cuda)
    bad = torch.empty(2, dtype=torch.int64, device=cuda)
    s = torch.cuda.Stream(cuda)
    h = ctypes.c_void_p(s.cuda_stream)

    def calls():
        assert L.fdb_sqlite_seal_pages_ws(d_raw.data_ptr(), 4096, 700, 1, ws.data_ptr(), nws, h) == 0
        assert L.fdb_sqlite_verify_pages_ws(d_sq.data_ptr(), 4096, 1500, 3, st.data_ptr(), bad.data_ptr(),
                                            ws.data_ptr(), nws, h) == 0
        assert L.fdb_diskqueue_check_pages_ws(d_dq.data_ptr(), 1200, ok.data_ptr(), bad.data_ptr() + 8,
                                              ws.data_ptr(), nws, h) == 0
    with torch.cuda.stream(s):
        calls()  # warm: the stream's counter words are allocated on first use
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        calls()
    for rep in range(3):
        st.zero_()
        ok.zero_()
        bad.fill_(-1)
        d_raw.copy_(torch.from_numpy(raw))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), exp), rep
        assert np.array_equal(ok.cpu().numpy(), dq_exp), rep
        b = bad.cpu().numpy()
        assert b[0] == int((exp == 0).sum()) and b[1] == int((dq_exp == 0).sum()), rep
        assert np.array_equal(d_raw.cpu().numpy(), sealed), rep
    del g


@pytest.mark.gpu
def test_gpu_verifiers_between_other_calls_on_one_stream(cuda):
    """The library's per-stream workspace is shared by every API on the stream;
    the verifiers' and the packet walk's counters are not in it, so verify,
    XXH3 and CRC varlen batches and packet verification interleaved on one
    stream all stay correct."""
    import torch
    import foundationdb_amd as F
    import foundationdb_amd.pagecheck as PC
    import foundationdb_amd.xxh3 as X
    pages, exp = make_sqlite_batch(900, 4096, 1, 81)
    dq, dq_exp = make_dq_batch(700, 82)
    d_sq = torch.from_numpy(pages.reshape(-1).copy()).to(cuda)
    d_dq = torch.from_numpy(dq.reshape(-1).copy()).to(cuda)
    rng = np.random.default_rng(83)
    h = sm_bytes(8 << 20, 84)
    lens = rng.integers(0, 40000, 500)
    offs = rng.integers(0, h.size - lens)
    d = torch.from_numpy(h).to(cuda)
    o, l = torch.from_numpy(offs).to(cuda), torch.from_numpy(lens).to(cuda)
    want_x = O.xxh3_batch_varlen(h, offs, lens)
    want_c = O.batch_varlen(h, offs, lens)
    s = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s):
        for rep in range(3):
            st, b1 = PC.sqlite_verify_pages(d_sq, 4096, stream=s)
            gx = X.batch_varlen(d, o, l, stream=s)
            ok, b2 = PC.diskqueue_check_pages(d_dq, stream=s)
            gc = F.batch_varlen(d, o, l, stream=s)
            s.synchronize()
            assert np.array_equal(st.cpu().numpy(), exp) and np.array_equal(ok.cpu().numpy(), dq_exp), rep
            assert int(b1.cpu().numpy().view(np.uint64)[0]) == int((exp == 0).sum())
            assert int(b2.cpu().numpy().view(np.uint64)[0]) == int((dq_exp == 0).sum())
            assert np.array_equal(gx.cpu().numpy().view(np.uint64), want_x)
            assert np.array_equal(gc.cpu().numpy().view(np.uint32), want_c)
    F.release_stream(s)


@pytest.mark.gpu
def test_gpu_ws_calls_from_two_threads_on_one_stream(cuda):
    """the _ws forms keep their list counters in words of the
    stream's own; two host threads each passing its own workspace on the same
    stream used to interleave their kernels on those counters.  The library now
    holds a per-stream lock from the counter lookup through the call's last
    launch: every call's verdicts stay exact."""
    import ctypes
    import threading
    import torch
    import foundationdb_amd.pagecheck as PC
    L = PC._lib()
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.fdb_sqlite_verify_pages_ws.argtypes = [vp, u64, u64, u32, vp, vp, vp, u64, vp]
    L.fdb_diskqueue_check_pages_ws.argtypes = [vp, u64, vp, vp, vp, u64, vp]
    pages, exp = make_sqlite_batch(1100, 4096, 5, 91)
    dq, dq_exp = make_dq_batch(900, 92)
    d_sq = torch.from_numpy(pages.reshape(-1).copy()).to(cuda)
    d_dq = torch.from_numpy(dq.reshape(-1).copy()).to(cuda)
    s = torch.cuda.Stream(cuda)
    h = ctypes.c_void_p(s.cuda_stream)
    reps = 12
    nws = int(L.fdb_pagecheck_workspace_bytes(1100))
    outs = {}

    def worker(kind):
        ws = torch.empty(nws, dtype=torch.uint8, device=cuda)
        res = torch.empty((reps, 1100), dtype=torch.uint8, device=cuda)
        bad = torch.empty(reps, dtype=torch.int64, device=cuda)
        for r in range(reps):
            if kind == "sq":
                rc = L.fdb_sqlite_verify_pages_ws(d_sq.data_ptr(), 4096, 1100, 5, res[r].data_ptr(),
                                                  bad[r:].data_ptr(), ws.data_ptr(), nws, h)
            else:
                rc = L.fdb_diskqueue_check_pages_ws(d_dq.data_ptr(), 900, res[r].data_ptr(), bad[r:].data_ptr(),
                                                    ws.data_ptr(), nws, h)
            assert rc == 0
        outs[kind] = (res, bad, ws)

    with torch.cuda.stream(s):
        warm = torch.empty(1100, dtype=torch.uint8, device=cuda)
        PC.sqlite_verify_pages(d_sq, 4096, first_pgno=5, stream=s, status=warm)
    s.synchronize()
    ts = [threading.Thread(target=worker, args=(k,)) for k in ("sq", "dq")]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    s.synchronize()
    res, bad, _ = outs["sq"]
    for r in range(reps):
        assert np.array_equal(res[r].cpu().numpy(), exp), r
        assert int(bad[r].item()) == int((exp == 0).sum()), r
    res, bad, _ = outs["dq"]
    for r in range(reps):
        assert np.array_equal(res[r, :900].cpu().numpy(), dq_exp), r
        assert int(bad[r].item()) == int((dq_exp == 0).sum()), r


@pytest.mark.gpu
def test_gpu_first_use_of_a_stream_inside_a_capture_is_refused(cuda):
    """a stream's counters are allocated and zeroed on its first use;
    inside a stream capture that would invalidate the capture (hipMalloc) and
    record the zeroing into the graph, so the call is refused with EINVAL and
    the capture stays usable; after one call outside the capture, capturing
    works."""
    import ctypes
    import torch
    import foundationdb_amd.pagecheck as PC
    FDB_CRC32C_EINVAL = -1  # include/fdb_crc32c.h
    L = PC._lib()
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.fdb_diskqueue_check_pages_ws.argtypes = [vp, u64, vp, vp, vp, u64, vp]
    dq, dq_exp = make_dq_batch(300, 93)
    d_dq = torch.from_numpy(dq.reshape(-1).copy()).to(cuda)
    nws = int(L.fdb_pagecheck_workspace_bytes(300))
    ws = torch.empty(nws, dtype=torch.uint8, device=cuda)
    ok = torch.zeros(300, dtype=torch.uint8, device=cuda)
    bad = torch.empty(1, dtype=torch.int64, device=cuda)
    x = torch.zeros(4, device=cuda)
    s = torch.cuda.Stream(cuda)
    h = ctypes.c_void_p(s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rc = L.fdb_diskqueue_check_pages_ws(d_dq.data_ptr(), 300, ok.data_ptr(), bad.data_ptr(), ws.data_ptr(), nws, h)
        x.add_(1)
    assert rc == FDB_CRC32C_EINVAL
    g.replay()
    torch.cuda.synchronize()
    assert x.cpu().tolist() == [1.0] * 4
    with torch.cuda.stream(s):
        assert L.fdb_diskqueue_check_pages_ws(d_dq.data_ptr(), 300, ok.data_ptr(), bad.data_ptr(), ws.data_ptr(),
                                              nws, h) == 0
    s.synchronize()
    assert np.array_equal(ok.cpu().numpy(), dq_exp)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        assert L.fdb_diskqueue_check_pages_ws(d_dq.data_ptr(), 300, ok.data_ptr(), bad.data_ptr(), ws.data_ptr(),
                                              nws, h) == 0
    ok.zero_()
    torch.cuda.synchronize()
    g2.replay()
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), dq_exp)
    del g, g2
