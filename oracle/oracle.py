"""ctypes bindings for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Two libraries, both built by oracle/Makefile:
  * liboracle_crc32c.so: our C restatement of contrib/crc32 (crc32c_oracle.c).
  * _ref/libcrc32c_ref.so: the reference's crc32c.cpp compiled unmodified
    (present wherever `make -C oracle` ran with /root/reference mounted; the
    .so travels to the GPU box with the repo snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(_HERE, "liboracle_crc32c.so")
REF_SO = os.path.join(_HERE, "_ref", "libcrc32c_ref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _ptr(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(t)


class _Lib:
    def __init__(self, path, symbol):
        self.path = path
        self.lib = ctypes.CDLL(path)
        self.fn = getattr(self.lib, symbol)
        self.fn.restype = ctypes.c_uint32
        self.fn.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]

    def append(self, crc, data):
        if isinstance(data, np.ndarray):
            data = np.ascontiguousarray(data, dtype=np.uint8)
            return self.fn(crc & 0xFFFFFFFF, data.ctypes.data, data.nbytes)
        b = bytes(data)
        return self.fn(crc & 0xFFFFFFFF, b, len(b))


_oracle = None
_ref = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build()
        _oracle = _Lib(ORACLE_SO, "oracle_crc32c_append")
        L = _oracle.lib
        L.oracle_crc32c_bitwise.restype = ctypes.c_uint32
        L.oracle_crc32c_bitwise.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc32c_shift.restype = ctypes.c_uint32
        L.oracle_crc32c_shift.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_crc32c_combine.restype = ctypes.c_uint32
        L.oracle_crc32c_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_crc32c_batch_fixed.restype = None
        L.oracle_crc32c_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_crc32c_batch_varlen.restype = None
        L.oracle_crc32c_batch_varlen.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_splitmix64_fill.restype = None
        L.oracle_splitmix64_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    return _oracle


def reference_available():
    return os.path.exists(REF_SO)


def reference():
    """The reference's own crc32c_append (contrib/crc32/crc32c.cpp:346-356)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(REF_SO + " (run `make -C oracle` where /root/reference exists)")
        _ref = _Lib(REF_SO, "crc32c_append")
    return _ref


def reference_batch_fixed(buf, stride, length, count, seed=0, out=None):
    """Single-threaded loop over the reference crc32c_append (bench cpu_baseline)."""
    L = reference().lib
    f = L.ref_batch_fixed
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                  ctypes.c_void_p]
    buf = np.ascontiguousarray(buf).view(np.uint8)
    if count:
        assert (count - 1) * stride + length <= buf.nbytes
    if out is None:
        out = np.zeros(count, dtype=np.uint32)
    f(buf.ctypes.data, stride, length, count, seed & 0xFFFFFFFF, out.ctypes.data)
    return out


def crc32c(crc, data):
    return oracle().append(crc, data)


def chained(buf, seg_offsets, seg_lengths, chain_starts, seed=0, seeds=None):
    """One CRC per chain of segments, fed in order with the running CRC as the
    next seed -- the reference's chained call sites: MutationRef checksums
    (fdbclient/include/fdbclient/CommitTransaction.h:302-304: crc = type;
    append(param1); append(param2)) and FileTransfer's whole-file CRC
    (fdbrpc/FileTransfer.cpp:29-37).  Chain c = segments [starts[c], starts[c+1])."""
    buf = np.ascontiguousarray(buf).view(np.uint8)
    n = len(chain_starts) - 1
    out = np.zeros(n, np.uint32)
    for c in range(n):
        crc = int(seeds[c]) if seeds is not None else seed
        for j in range(int(chain_starts[c]), int(chain_starts[c + 1])):
            o, ln = int(seg_offsets[j]), int(seg_lengths[j])
            crc = crc32c(crc, buf[o:o + ln])
        out[c] = crc
    return out


def crc32c_bitwise(crc, data):
    b = bytes(data)
    return oracle().lib.oracle_crc32c_bitwise(crc & 0xFFFFFFFF, b, len(b))


def shift(raw, nbytes):
    return oracle().lib.oracle_crc32c_shift(raw & 0xFFFFFFFF, nbytes)


def combine(crc_a, crc_b, len_b):
    return oracle().lib.oracle_crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def batch_fixed(buf, stride, length, count, seed=0, seeds=None, threads=None):
    buf = np.ascontiguousarray(buf).view(np.uint8)
    if count:
        assert (count - 1) * stride + length <= buf.nbytes
    out = np.zeros(count, dtype=np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    threads = threads or min(16, os.cpu_count() or 1)
    oracle().lib.oracle_crc32c_batch_fixed(buf.ctypes.data, stride, length, count, seed & 0xFFFFFFFF,
                                           None if sd is None else sd.ctypes.data, out.ctypes.data, threads)
    return out


def batch_varlen(buf, offsets, lengths, seed=0, seeds=None, threads=None):
    buf = np.ascontiguousarray(buf).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    n = offsets.size
    assert lengths.size == n
    if n:
        assert int((offsets + lengths).max()) <= buf.nbytes
    out = np.zeros(n, dtype=np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    threads = threads or min(16, os.cpu_count() or 1)
    oracle().lib.oracle_crc32c_batch_varlen(buf.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, n,
                                            seed & 0xFFFFFFFF, None if sd is None else sd.ctypes.data,
                                            out.ctypes.data, threads)
    return out


def splitmix64(nwords, state):
    out = np.empty(nwords, dtype=np.uint64)
    oracle().lib.oracle_splitmix64_fill(out.ctypes.data, nwords, state)
    return out


# ---------------------------------------------------------------- XXH3-64 / lookup3
# liboracle_xxh3.so: our restatement (xxh3_oracle.c); _ref/libxxhash_ref.so:
# the reference's flow/xxhash.c + flow/Hash3.c compiled unmodified.
XXH3_SO = os.path.join(_HERE, "liboracle_xxh3.so")
XXH3_REF_SO = os.path.join(_HERE, "_ref", "libxxhash_ref.so")
PAGECHECK_REF_SO = os.path.join(_HERE, "_ref", "libpagecheck_ref.so")
_x = None
_xref = None


def _xxh3():
    global _x
    if _x is None:
        if not os.path.exists(XXH3_SO):
            build()
        L = ctypes.CDLL(XXH3_SO)
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.oracle_xxh3_64.restype = u64
        L.oracle_xxh3_64.argtypes = [vp, ctypes.c_size_t, u64]
        L.oracle_hashlittle2.restype = None
        L.oracle_hashlittle2.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_xxh3_batch_fixed.restype = None
        L.oracle_xxh3_batch_fixed.argtypes = [vp, u64, u64, u64, u64, vp, vp, ctypes.c_int]
        L.oracle_xxh3_batch_varlen.restype = None
        L.oracle_xxh3_batch_varlen.argtypes = [vp, vp, vp, u64, u64, vp, vp, ctypes.c_int]
        _x = L
    return _x


def _as_bytes(data):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8)
        return a, a.ctypes.data, a.nbytes
    b = bytes(data)
    return b, b, len(b)


def xxh3_64(data, seed=0):
    keep, p, n = _as_bytes(data)
    return _xxh3().oracle_xxh3_64(p, n, seed & 0xFFFFFFFFFFFFFFFF)


def hashlittle2(data, pc, pb):
    keep, p, n = _as_bytes(data)
    c, b = ctypes.c_uint32(pc), ctypes.c_uint32(pb)
    _xxh3().oracle_hashlittle2(p, n, ctypes.byref(c), ctypes.byref(b))
    return c.value, b.value


def xxh3_batch_fixed(buf, stride, length, count, seed=0, seeds=None, threads=None):
    buf = np.ascontiguousarray(buf).view(np.uint8)
    if count:
        assert (count - 1) * stride + length <= buf.nbytes
    out = np.zeros(count, dtype=np.uint64)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint64)
    threads = threads or min(16, os.cpu_count() or 1)
    _xxh3().oracle_xxh3_batch_fixed(buf.ctypes.data, stride, length, count, seed & 0xFFFFFFFFFFFFFFFF,
                                    None if sd is None else sd.ctypes.data, out.ctypes.data, threads)
    return out


def xxh3_batch_varlen(buf, offsets, lengths, seed=0, seeds=None, threads=None):
    buf = np.ascontiguousarray(buf).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    n = offsets.size
    if n:
        assert int((offsets + lengths).max()) <= buf.nbytes
    out = np.zeros(n, dtype=np.uint64)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint64)
    threads = threads or min(16, os.cpu_count() or 1)
    _xxh3().oracle_xxh3_batch_varlen(buf.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, n,
                                     seed & 0xFFFFFFFFFFFFFFFF, None if sd is None else sd.ctypes.data,
                                     out.ctypes.data, threads)
    return out


def xxh3_reference_available():
    return os.path.exists(XXH3_REF_SO)


def xxh3_reference():
    """The reference's XXH3_64bits / XXH3_64bits_withSeed / hashlittle2 (compiled unmodified)."""
    global _xref
    if _xref is None:
        if not os.path.exists(XXH3_REF_SO):
            raise FileNotFoundError(XXH3_REF_SO + " (run `make -C oracle` where /root/reference exists)")
        L = ctypes.CDLL(XXH3_REF_SO)
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.XXH3_64bits.restype = u64
        L.XXH3_64bits.argtypes = [vp, ctypes.c_size_t]
        L.XXH3_64bits_withSeed.restype = u64
        L.XXH3_64bits_withSeed.argtypes = [vp, ctypes.c_size_t, u64]
        L.hashlittle2.restype = None
        L.hashlittle2.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        _xref = L
    return _xref


def ref_xxh3_64(data, seed=0):
    keep, p, n = _as_bytes(data)
    L = xxh3_reference()
    return L.XXH3_64bits(p, n) if seed == 0 else L.XXH3_64bits_withSeed(p, n, seed & 0xFFFFFFFFFFFFFFFF)


def ref_hashlittle2(data, pc, pb):
    keep, p, n = _as_bytes(data)
    c, b = ctypes.c_uint32(pc), ctypes.c_uint32(pb)
    xxh3_reference().hashlittle2(p, n, ctypes.byref(c), ctypes.byref(b))
    return c.value, b.value


def ref_xxh3_batch_varlen(buf, offsets, lengths):
    """Single-threaded C loop over the reference XXH3_64bits, one packet per
    (offset, length) (ref_bench_xxh3.c; bench cpu_baseline)."""
    buf = np.ascontiguousarray(buf).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    if offsets.size:
        assert int((offsets + lengths).max()) <= buf.nbytes
    f = xxh3_reference().ref_xxh3_batch_varlen
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    out = np.zeros(offsets.size, np.uint64)
    f(buf.ctypes.data, offsets.ctypes.data, lengths.ctypes.data, offsets.size, out.ctypes.data)
    return out


def ref_xxh3_batch_fixed(buf, stride, length, count, seed=0):
    """Single-threaded C loop over the reference XXH3_64bits (ref_bench_xxh3.c; bench cpu_baseline)."""
    buf = np.ascontiguousarray(buf).view(np.uint8)
    if count:
        assert (count - 1) * stride + length <= buf.nbytes
    L = xxh3_reference()
    f = L.ref_xxh3_batch_fixed
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    out = np.zeros(count, dtype=np.uint64)
    f(buf.ctypes.data, stride, length, count, seed & 0xFFFFFFFFFFFFFFFF, out.ctypes.data)
    return out


# ------------------------------------------------- page checks, reference-composed
_pcref = None


def pagecheck_reference_available():
    return os.path.exists(PAGECHECK_REF_SO)


def pagecheck_reference():
    """oracle/ref_pagecheck.c over the reference's own crc32c_append, XXH3_64bits
    and hashlittle2 (oracle/_ref/libpagecheck_ref.so): the SQLite and DiskQueue
    page checks as FoundationDB runs them, one page at a time."""
    global _pcref
    if _pcref is None:
        if not os.path.exists(PAGECHECK_REF_SO):
            raise FileNotFoundError(PAGECHECK_REF_SO + " (run `make -C oracle` where /root/reference exists)")
        L = ctypes.CDLL(PAGECHECK_REF_SO)
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.ref_sqlite_verify_pages.restype = u64
        L.ref_sqlite_verify_pages.argtypes = [vp, u64, u64, ctypes.c_uint32, vp]
        L.ref_diskqueue_check_pages.restype = u64
        L.ref_diskqueue_check_pages.argtypes = [vp, u64, vp]
        L.ref_sqlite_seal_pages.restype = None
        L.ref_sqlite_seal_pages.argtypes = [vp, u64, u64, ctypes.c_uint32]
        L.ref_diskqueue_seal_pages.restype = None
        L.ref_diskqueue_seal_pages.argtypes = [vp, u64]
        L.ref_redwood_verify_pages.restype = u64
        L.ref_redwood_verify_pages.argtypes = [vp, u64, u64, vp, ctypes.c_uint32, vp]
        L.ref_redwood_seal_pages.restype = None
        L.ref_redwood_seal_pages.argtypes = [vp, u64, u64, vp, ctypes.c_uint32, vp]
        _pcref = L
    return _pcref


def ref_sqlite_verify_pages(pages, page_size, count, first_pgno=1):
    """(status per page, bad count) from the reference primitives (single thread)."""
    pages = np.ascontiguousarray(pages).view(np.uint8)
    assert count * page_size <= pages.nbytes
    st = np.zeros(count, np.uint8)
    bad = pagecheck_reference().ref_sqlite_verify_pages(pages.ctypes.data, page_size, count, first_pgno,
                                                        st.ctypes.data)
    return st, int(bad)


def ref_diskqueue_check_pages(pages, count):
    pages = np.ascontiguousarray(pages).view(np.uint8)
    assert count * 4096 <= pages.nbytes
    ok = np.zeros(count, np.uint8)
    bad = pagecheck_reference().ref_diskqueue_check_pages(pages.ctypes.data, count, ok.ctypes.data)
    return ok, int(bad)


def _seal_target(pages, inplace):
    if inplace:
        assert isinstance(pages, np.ndarray) and pages.dtype == np.uint8 and pages.flags.c_contiguous
        return pages.reshape(-1)
    return np.array(np.ascontiguousarray(pages).view(np.uint8).reshape(-1), copy=True)


def ref_sqlite_seal_pages(pages, page_size, count, first_pgno=1, inplace=False):
    """A sealed copy of `pages` (or `pages` itself with inplace): the codec's page
    writes (op 6 / 7) composed from the reference's XXH3_64bits (oracle/ref_pagecheck.c)."""
    out = _seal_target(pages, inplace)
    assert count * page_size <= out.nbytes
    pagecheck_reference().ref_sqlite_seal_pages(out.ctypes.data, page_size, count, first_pgno)
    return out


def ref_diskqueue_seal_pages(pages, count, inplace=False):
    """A sealed copy of `pages` (or `pages` itself with inplace): Page::updateHash
    by version from the reference primitives."""
    out = _seal_target(pages, inplace)
    assert count * 4096 <= out.nbytes
    pagecheck_reference().ref_diskqueue_seal_pages(out.ctypes.data, count)
    return out


def _ids_ptr(ids):
    if ids is None:
        return None, None
    a = np.ascontiguousarray(ids, dtype=np.uint32)
    return a, a.ctypes.data


def ref_redwood_verify_pages(pages, page_size, count, ids=None, first_id=0, inplace=False):
    """(status per page, bad count): postReadHeader + postReadPayload composed
    from the reference's XXH3_64bits / XXH3_64bits_withSeed (oracle/ref_pagecheck.c).
    The reference zeroes and restores the checksum field in place, so the
    pages come back unchanged; without `inplace` a copy is checked."""
    buf = _seal_target(pages, inplace)
    st = np.zeros(count, np.uint8)
    keep, ip = _ids_ptr(ids)
    bad = pagecheck_reference().ref_redwood_verify_pages(buf.ctypes.data, page_size, count, ip, first_id,
                                                         st.ctypes.data)
    return st, int(bad)


def ref_redwood_seal_pages(pages, page_size, count, ids=None, first_id=0, inplace=False):
    """(sealed copy -- or `pages` itself with inplace --, status per page):
    preWrite(pageID) from the reference primitives."""
    out = _seal_target(pages, inplace)
    st = np.zeros(count, np.uint8)
    keep, ip = _ids_ptr(ids)
    pagecheck_reference().ref_redwood_seal_pages(out.ctypes.data, page_size, count, ip, first_id, st.ctypes.data)
    return out, st


# ---------------------------------------------------------------- page formats
# Restatements of the reference's page checksum logic on top of the pinned
# primitives above (checker side only).

def sqlite_trailer_crc(page):
    """Legacy writer: part1 = 0, part2 = crc32c_append(0xfdbeefdb, data) (KeyValueStoreSQLite.cpp:119-128)."""
    data = bytes(page[:-8])
    return (0).to_bytes(4, "little") + crc32c(0xFDBEEFDB, data).to_bytes(4, "little")


def sqlite_trailer_xxh3(page):
    """Current writer, KeyValueStoreSQLite.cpp:106-116."""
    h = xxh3_64(bytes(page[:-8]))
    return ((h >> 32) & 0x00FFFFFF).to_bytes(4, "little") + (h & 0xFFFFFFFF).to_bytes(4, "little")


def sqlite_trailer_hl2(page, pgno):
    c, b = hashlittle2(bytes(page[:-8]), pgno, 0x5CA1AB1E)
    return c.to_bytes(4, "little") + b.to_bytes(4, "little")


def sqlite_verify_page(page, pgno):
    """PageChecksumCodec::checksum(write=false), KeyValueStoreSQLite.cpp:118-158: 1 CRC, 2 XXH3, 3 hashlittle2, 0 bad."""
    page = bytes(page)
    data, t = page[:-8], page[-8:]
    part1, part2 = int.from_bytes(t[:4], "little"), int.from_bytes(t[4:], "little")
    if part1 == 0 and part2 == crc32c(0xFDBEEFDB, data):
        return 1
    if (part1 >> 24) == 0:
        h = xxh3_64(data)
        if part1 == ((h >> 32) & 0x00FFFFFF) and part2 == (h & 0xFFFFFFFF):
            return 2
    c, b = hashlittle2(data, pgno, 0x5CA1AB1E)
    return 3 if (c, b) == (part1, part2) else 0


def sqlite_codec_page(page, pgno, reserve_size, op):
    """PageChecksumCodec::codec (KeyValueStoreSQLite.cpp:203-244) on one page:
    returns (status, page') -- status 0 where codec() returns nullptr, else
    the accepting check (op 3) or 2 (ops 6 / 7, the page sealed)."""
    assert op in (3, 6, 7)
    page = np.array(np.frombuffer(bytes(page), np.uint8), copy=True)
    if pgno != 1 and reserve_size != 8:  # :225-237
        return 0, page
    if op == 3:
        return sqlite_verify_page(page, pgno), page
    return 2, sqlite_seal_pages(page, page.size, 1, first_pgno=pgno)


def diskqueue_hash(page, version):
    """Page::updateHash (DiskQueue.cpp:1089-1106): the 16-byte hash field for `version`."""
    page = bytes(page)
    if version == 0:
        c, b = hashlittle2(page[16:], 0x12345678, 0xBEEFABCD)
        return ((c << 32) | b).to_bytes(8, "little") + (0xFDB).to_bytes(8, "little")
    if version == 1:
        return crc32c(0xFDBEEFDB, page[4:]).to_bytes(4, "little") + page[4:16]
    return xxh3_64(page[8:]).to_bytes(8, "little") + page[8:16]


def sqlite_seal_pages(pages, page_size, count, first_pgno=1):
    """The codec's page writes (KeyValueStoreSQLite.cpp:203-244) on a copy of
    `pages`, from our XXH3 restatement: page 1 with page_size > 1024
    (SQLITE_DEFAULT_PAGE_SIZE) first sealed as a 1024-byte page (:221-224),
    then every page's trailer = sqlite_trailer_xxh3 (checksum(write = true), :107-116)."""
    out = np.array(np.ascontiguousarray(pages).view(np.uint8).reshape(-1)[:count * page_size], copy=True)
    for i in range(count):
        pg = out[i * page_size:(i + 1) * page_size]
        if first_pgno + i == 1 and page_size > 1024:
            pg[1016:1024] = np.frombuffer(sqlite_trailer_xxh3(pg[:1024]), np.uint8)
        pg[-8:] = np.frombuffer(sqlite_trailer_xxh3(pg), np.uint8)
    return out


def diskqueue_seal_pages(pages, count):
    """Page::updateHash (DiskQueue.cpp:1089-1105) on a copy of `pages` by
    implementationVersion; versions other than 0 and 1 take XXH3 (the switch's default)."""
    out = np.array(np.ascontiguousarray(pages).view(np.uint8).reshape(-1)[:count * 4096], copy=True)
    for i in range(count):
        pg = out[i * 4096:(i + 1) * 4096]
        ver = int.from_bytes(bytes(pg[10:12]), "little")
        pg[:16] = np.frombuffer(diskqueue_hash(pg, ver if ver <= 1 else 2), np.uint8)
    return out


def diskqueue_check_page(page):
    """Page::checkHash (DiskQueue.cpp:1107-1120)."""
    page = bytes(page)
    ver = int.from_bytes(page[10:12], "little")
    if ver == 0:
        c, b = hashlittle2(page[16:], 0x12345678, 0xBEEFABCD)
        return int(page[:8] == ((c << 32) | b).to_bytes(8, "little") and page[8:16] == (0xFDB).to_bytes(8, "little"))
    if ver == 1:
        return int(int.from_bytes(page[:4], "little") == crc32c(0xFDBEEFDB, page[4:]))
    if ver == 2:
        return int(int.from_bytes(page[:8], "little") == xxh3_64(page[8:]))
    return 0


# Redwood pages (fdbserver/kvstore/IPager.h:246-331, 480-565): the byte layout
# of header version 1 and the XXHash64 encoding.
REDWOOD_HEADER = 51  # PageHeader (4) + RedwoodHeaderV1 (39) + XXHashEncoder::Header (8)


def redwood_init_page(page, page_id, page_type=2, sub_type=1, write_version=1, write_time=0.0):
    """ArenaPage::init(XXHash64, pageType, pageSubType) (:448-470) and
    setWriteInfo(pageID, version) (:496-502) on a page buffer (in place):
    header version 1, encoding header at 43, payload at 51."""
    import struct
    page[0:4] = np.frombuffer(bytes([1, 0, 43, REDWOOD_HEADER]), np.uint8)
    hdr = struct.pack("<BBBQIIIdq", page_type, sub_type, 0, 0, page_id, 0xFFFFFFFF, 0xFFFFFFFF, write_time,
                      write_version)
    page[4:43] = np.frombuffer(hdr, np.uint8)
    return page


def redwood_seal_page(page, page_id):
    """preWrite(pageID) (:500-525) on a copy: (status, page')."""
    pg = np.array(np.frombuffer(bytes(page), np.uint8), copy=True)
    enc, eho, po = int(pg[1]), int(pg[2]), int(pg[3])
    if enc != 0:
        return 4, pg
    pg[eho:eho + 8] = np.frombuffer(xxh3_64(bytes(pg[po:]), page_id).to_bytes(8, "little"), np.uint8)
    if pg[0] != 1:
        return 1, pg
    pg[7:15] = 0
    pg[7:15] = np.frombuffer(xxh3_64(bytes(pg[:po])).to_bytes(8, "little"), np.uint8)
    return 0, pg


def redwood_verify_page(page, page_id):
    """postReadHeader(pageID, verify = true) then postReadPayload(pageID):
    0, or the first failure (1 version, 2 header checksum, 3 page ID, 4 encoding, 5 decoding)."""
    pg = bytearray(bytes(page))
    ver, enc, eho, po = pg[0], pg[1], pg[2], pg[3]
    if ver != 1:
        return 1
    saved = int.from_bytes(pg[7:15], "little")
    pg[7:15] = bytes(8)
    calc = xxh3_64(bytes(pg[:po]))
    pg[7:15] = saved.to_bytes(8, "little")
    if saved != calc:
        return 2
    if int.from_bytes(pg[15:19], "little") != page_id:
        return 3
    if enc != 0:
        return 4
    if int.from_bytes(pg[eho:eho + 8], "little") != xxh3_64(bytes(pg[po:]), page_id):
        return 5
    return 0


# ---- FlowTransport receive checks (packets_oracle.c) --------------------------
PACKETS_SO = os.path.join(_HERE, "liboracle_packets.so")
PACKETS_REF_SO = os.path.join(_HERE, "_ref", "libpackets_ref.so")
_pk = {}


def _packets_lib(ref):
    path = PACKETS_REF_SO if ref else PACKETS_SO
    if path not in _pk:
        if not os.path.exists(path):
            if ref:
                raise FileNotFoundError(path + " (run `make -C oracle` where /root/reference exists)")
            build()
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        L.oracle_packets_verify.restype = None
        L.oracle_packets_verify.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, vp, vp, vp]
        _pk[path] = L
    return _pk[path]


def packets_reference_available():
    return os.path.exists(PACKETS_REF_SO)


def packets_verify(buf, buf_offsets, buf_lengths, checksum=True, packet_limit=100 << 20, ref=False):
    """scanPackets' outcome per receive buffer (FlowTransport.cpp:1260-1366):
    (consumed u64, frames u32, status i32) arrays.  ref=True hashes with the
    reference's own flow/xxhash.c instead of our XXH3 restatement."""
    buf = np.ascontiguousarray(buf).view(np.uint8)
    bo = np.ascontiguousarray(buf_offsets, dtype=np.uint64)
    bl = np.ascontiguousarray(buf_lengths, dtype=np.uint64)
    n = bo.size
    if n:
        assert int((bo + bl).max()) <= buf.nbytes
    consumed = np.zeros(n, np.uint64)
    frames = np.zeros(n, np.uint32)
    status = np.zeros(n, np.int32)
    _packets_lib(ref).oracle_packets_verify(buf.ctypes.data, bo.ctypes.data, bl.ctypes.data, n, 1 if checksum else 0,
                                            packet_limit, consumed.ctypes.data, frames.ctypes.data,
                                            status.ctypes.data)
    return consumed, frames, status
