"""Batched Redwood page checks (include/fdb_redwood.h) against the reference's
ArenaPage checks (fdbserver/kvstore/IPager.h:297-331, 500-565): the oracle
restatement (oracle/oracle.py: redwood_*), the same checks composed from the
reference's own XXH3_64bits / XXH3_64bits_withSeed compiled unmodified
(oracle/ref_pagecheck.c -> oracle/_ref/libpagecheck_ref.so), and the
reference's unit test /fdbserver/IPager/ArenaPage/PageContentChecksum
(fdbserver/kvstore/IPager.cpp:27-50)."""
import numpy as np
import pytest

from oracle import oracle as O

KINDS = 10


def sm_bytes(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


def _rehash_header(pg):
    po = int(pg[3])
    pg[7:15] = 0
    pg[7:15] = np.frombuffer(O.xxh3_64(bytes(pg[:po])).to_bytes(8, "little"), np.uint8)


def make_redwood_batch(n, page_size, ids, seed):
    """Pages hitting every outcome of postReadHeader + postReadPayload: written
    by the reference's writer (init, setWriteInfo, preWrite), then corrupted in
    the payload, the header, the page ID, the version, the encoding; layouts
    other than the writer's (header lengths 10 .. 255, the encoding header
    overlapping the checksum field, a header past 240 bytes: XXH3's long form);
    raw random pages."""
    rng = np.random.default_rng(seed)
    pages = sm_bytes(n * page_size, seed).reshape(n, page_size)
    kinds = rng.integers(0, KINDS, n)
    for i in range(n):
        pg, k, pid = pages[i], int(kinds[i]), int(ids[i])
        if k == 9:
            continue  # raw bytes (version byte random: almost always unsupported)
        O.redwood_init_page(pg, pid if k != 3 else pid ^ 0x5A5A, write_version=i, write_time=i * 0.25)
        if k in (6, 7, 8):  # another layout: payloadOffset, encoding header anywhere in [0, po - 8]
            po = int(rng.choice([10, 16, 17, 33, 64, 65, 128, 129, 200, 240, 241, 255])) if k != 8 else 250
            eho = int(rng.integers(0, po - 7)) if po >= 8 else 0
            if k == 7:
                eho = min(9, po - 8) if po >= 8 else 0  # overlaps the checksum field
            pg[2], pg[3] = eho, po
        st, sealed = O.redwood_seal_page(pg, pid)
        pg[:] = sealed
        if k == 1:
            j = int(rng.integers(int(pg[3]), page_size))
            pg[j] ^= 1 << int(rng.integers(0, 8))
        elif k == 2:
            j = int(rng.integers(0, int(pg[3])))
            if 7 <= j < 15 or j < 4:
                j = 20 if pg[3] > 20 else j
            pg[j] ^= 0x40
        elif k == 4:
            pg[0] = 2
        elif k == 5:
            pg[1] = 1  # the deprecated XOR test encoding: needs the pager's xorWith
            _rehash_header(pg)
    exp = np.array([O.redwood_verify_page(pages[i], int(ids[i])) for i in range(n)], np.uint8)
    return pages, exp


def test_oracle_follows_reference_page_content_checksum_test():
    """IPager.cpp:27-50: an 8 KiB BTreeNode page with random payload written by
    preWrite(pageID) verifies; one flipped payload byte passes postReadHeader
    and fails postReadPayload with page_decoding_failed."""
    rng = np.random.default_rng(1)
    page = np.zeros(8192, np.uint8)
    O.redwood_init_page(page, 0, page_type=2, sub_type=1)
    page[O.REDWOOD_HEADER:] = rng.integers(0, 256, 8192 - O.REDWOOD_HEADER, dtype=np.uint8)
    pid = int(rng.integers(0, 2**32))
    O.redwood_init_page(page, pid)  # setWriteInfo(pageID, 1)
    st, page = O.redwood_seal_page(page, pid)
    assert st == 0 and O.redwood_verify_page(page, pid) == 0
    j = O.REDWOOD_HEADER + int(rng.integers(0, 8192 - O.REDWOOD_HEADER))
    page[j] = ~page[j]
    assert O.redwood_verify_page(page, pid) == 5
    assert O.redwood_verify_page(page, pid ^ 1) == 3


@pytest.mark.skipif(not O.pagecheck_reference_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("page_size", [512, 4096, 8192])
def test_oracle_redwood_matches_reference_composition(page_size):
    n = 400
    ids = np.random.default_rng(page_size).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    pages, exp = make_redwood_batch(n, page_size, ids, page_size + 3)
    assert set(np.unique(exp)) == {0, 1, 2, 3, 4, 5}
    st, bad = O.ref_redwood_verify_pages(pages, page_size, n, ids=ids)
    assert np.array_equal(st, exp) and bad == int((exp != 0).sum())
    # the writer: preWrite over the batch, page by page
    raw = sm_bytes(n * page_size, page_size + 4).reshape(n, page_size)
    for i in range(0, n, 3):
        O.redwood_init_page(raw[i], int(ids[i]))
    sealed, sst = O.ref_redwood_seal_pages(raw, page_size, n, ids=ids)
    for i in range(n):
        s, pg = O.redwood_seal_page(raw[i], int(ids[i]))
        assert s == sst[i] and np.array_equal(pg, sealed[i * page_size:(i + 1) * page_size]), i
    first = 77
    st2, _ = O.ref_redwood_verify_pages(sealed, page_size, n, first_id=first)
    want = [O.redwood_verify_page(sealed[i * page_size:(i + 1) * page_size], first + i) for i in range(n)]
    assert st2.tolist() == want


def _expect(pages, page_size, n, ids):
    if O.pagecheck_reference_available():
        st, bad = O.ref_redwood_verify_pages(pages, page_size, n, ids=ids)
        return st
    return np.array([O.redwood_verify_page(pages[i], int(ids[i])) for i in range(n)], np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("page_size", [512, 4096, 8192, 65536])
def test_gpu_redwood_verify_mixed(cuda, page_size):
    import torch
    import foundationdb_amd.redwood as RW
    n = {512: 3000, 4096: 2000, 8192: 1500, 65536: 120}[page_size]
    ids = np.random.default_rng(page_size + 1).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    pages, exp = make_redwood_batch(n, page_size, ids, page_size + 2)
    assert np.array_equal(_expect(pages, page_size, n, ids), exp)
    d = torch.from_numpy(pages.reshape(-1).copy()).to(cuda)
    d_ids = torch.from_numpy(ids.view(np.int32)).to(cuda)
    st, bad = RW.verify_pages(d, page_size, page_ids=d_ids)
    got = st.cpu().numpy()
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    assert int(bad.cpu().numpy().view(np.uint64)[0]) == int((exp != 0).sum())
    assert np.array_equal(d.cpu().numpy(), pages.reshape(-1))  # verification changes nothing


@pytest.mark.gpu
@pytest.mark.parametrize("page_size", [512, 8192, 65536])
def test_gpu_redwood_seal_then_verify(cuda, page_size):
    """preWrite over a batch (first_page_id form) equals the reference's, page
    for page (status and bytes), and the sealed pages verify."""
    import torch
    import foundationdb_amd.redwood as RW
    n = {512: 2500, 8192: 1200, 65536: 100}[page_size]
    first = 0xFFFFFF00  # page IDs wrap past 2^32 - 1
    ids = (first + np.arange(n, dtype=np.uint64)).astype(np.uint32)
    raw, _ = make_redwood_batch(n, page_size, ids, page_size + 5)
    rng = np.random.default_rng(6)
    for i in rng.integers(0, n, n // 10):
        raw[i, 1] = 1  # encoding other than XXHash64: refused, page untouched
    if O.pagecheck_reference_available():
        want, want_st = O.ref_redwood_seal_pages(raw, page_size, n, first_id=first)
    else:
        outs = [O.redwood_seal_page(raw[i], int(ids[i])) for i in range(n)]
        want = np.concatenate([o[1] for o in outs])
        want_st = np.array([o[0] for o in outs], np.uint8)
    d = torch.from_numpy(raw.reshape(-1).copy()).to(cuda)
    st = RW.seal_pages(d, page_size, first_page_id=first)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), want_st)
    got = d.cpu().numpy()
    bad = np.nonzero((got != want).reshape(n, page_size).any(axis=1))[0]
    assert bad.size == 0, bad[:10]
    vst, nbad = RW.verify_pages(d, page_size, first_page_id=first)
    exp = np.array([O.redwood_verify_page(want[i * page_size:(i + 1) * page_size], int(ids[i])) for i in range(n)],
                   np.uint8)
    assert np.array_equal(vst.cpu().numpy(), exp)
    # (pages sealed OK verify unless built with another page ID or a payload
    # the encoding header overlaps: most of them)
    assert (exp == 0).sum() > n // 3


@pytest.mark.gpu
def test_gpu_redwood_ws_forms_capture_and_empty(cuda):
    """The _ws forms keep no state outside the caller's workspace: a captured
    seal + verify replays bit-exact; count 0 writes a zero bad count."""
    import ctypes
    import torch
    import foundationdb_amd.redwood as RW
    L = RW._lib()
    n, ps = 900, 8192
    ids = np.arange(n, dtype=np.uint32) * 7 + 3
    raw = sm_bytes(n * ps, 41).reshape(n, ps)
    for i in range(n):
        O.redwood_init_page(raw[i], int(ids[i]))
    want = np.concatenate([O.redwood_seal_page(raw[i], int(ids[i]))[1] for i in range(n)])
    d = torch.from_numpy(raw.reshape(-1).copy()).to(cuda)
    d_ids = torch.from_numpy(ids.view(np.int32)).to(cuda)
    nws = RW.workspace_bytes(n, ps)
    ws = torch.empty(nws, dtype=torch.uint8, device=cuda)
    st = torch.empty(n, dtype=torch.uint8, device=cuda)
    bad = torch.empty(1, dtype=torch.int64, device=cuda)
    s = torch.cuda.Stream(cuda)
    h = ctypes.c_void_p(s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        assert L.fdb_redwood_seal_pages_ws(d.data_ptr(), ps, n, d_ids.data_ptr(), 0, None, ws.data_ptr(), nws, h) == 0
        assert L.fdb_redwood_verify_pages_ws(d.data_ptr(), ps, n, d_ids.data_ptr(), 0, st.data_ptr(), bad.data_ptr(),
                                             ws.data_ptr(), nws, h) == 0
    for rep in range(2):
        d.copy_(torch.from_numpy(raw.reshape(-1)))
        st.fill_(9)
        bad.fill_(-1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), want), rep
        assert (st.cpu().numpy() == 0).all() and int(bad.item()) == 0, rep
    del g
    bad.fill_(-1)
    assert L.fdb_redwood_verify_pages(d.data_ptr(), ps, 0, None, 0, st.data_ptr(), bad.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
