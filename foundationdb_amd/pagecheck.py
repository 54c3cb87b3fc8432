"""Python host mirror of the batched page verifiers and sealers (include/fdb_pagecheck.h).

Reference interfaces: PageChecksumCodec::checksum(pgno, page, pageLen,
write=false/true) (fdbserver/kvstore/KeyValueStoreSQLite.cpp:100-201, the
codec's page writes :203-244) and DiskQueue Page::checkHash / updateHash
(fdbserver/kvstore/DiskQueue.cpp:1047-1120), run over whole batches of
device-resident pages.  No CPU fallback.
"""
import ctypes

import torch

from .crc32c import CRC32CError, _check, _require_device, _stream_handle, lib

_bound = False

STATUS_BAD, STATUS_CRC32C, STATUS_XXH3, STATUS_HASHLITTLE2 = 0, 1, 2, 3


def _lib():
    global _bound
    L = lib()
    if not _bound:
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        L.fdb_sqlite_verify_pages.restype = ctypes.c_int
        L.fdb_sqlite_verify_pages.argtypes = [vp, u64, u64, u32, vp, vp, vp]
        L.fdb_diskqueue_check_pages.restype = ctypes.c_int
        L.fdb_diskqueue_check_pages.argtypes = [vp, u64, vp, vp, vp]
        L.fdb_pagecheck_workspace_bytes.restype = u64
        L.fdb_pagecheck_workspace_bytes.argtypes = [u64]
        L.fdb_sqlite_seal_pages.restype = ctypes.c_int
        L.fdb_sqlite_seal_pages.argtypes = [vp, u64, u64, u32, vp]
        L.fdb_diskqueue_seal_pages.restype = ctypes.c_int
        L.fdb_diskqueue_seal_pages.argtypes = [vp, u64, vp]
        L.fdb_sqlite_codec_pages.restype = ctypes.c_int
        L.fdb_sqlite_codec_pages.argtypes = [vp, u64, u32, u64, u32, ctypes.c_int, vp, vp]
        _bound = True
    return L


def _vp(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _outputs(pages, count, status, bad, who):
    """Caller-owned output tensors (no allocation or fill per call), or new
    ones.  The library stores the bad count (it does not accumulate into it),
    so neither needs initialising."""
    if status is None:
        status = torch.empty(count, dtype=torch.uint8, device=pages.device)
    _require_device(status, f"{who}: status", pages.device, (torch.uint8,), count)
    if bad is None:
        bad = torch.empty(1, dtype=torch.uint64, device=pages.device)
    _require_device(bad, f"{who}: bad", pages.device, (torch.uint64, torch.int64), 1)
    return status, bad


def sqlite_verify_pages(pages, page_size, count=None, first_pgno=1, stream=None, status=None, bad=None):
    """Returns (status uint8 tensor, bad-page count tensor) for a batch of SQLite
    pages.  `status` (uint8, >= count) and `bad` (one 64-bit word) may be
    caller-owned device tensors, reused across calls."""
    _require_device(pages, "pages")
    nbytes = pages.numel() * pages.element_size()
    count = nbytes // page_size if count is None else int(count)
    if count * page_size > nbytes:
        raise CRC32CError("sqlite_verify_pages: pages extend past the tensor")
    status, bad = _outputs(pages, count, status, bad, "sqlite_verify_pages")
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_sqlite_verify_pages(_vp(pages), page_size, count, first_pgno, _vp(status), _vp(bad),
                                            _stream_handle(stream))
    _check(rc, "fdb_sqlite_verify_pages")
    return status, bad


def diskqueue_check_pages(pages, count=None, stream=None, ok=None, bad=None):
    """Returns (ok uint8 tensor, bad-page count tensor) for a batch of 4 KiB
    DiskQueue pages (`ok` and `bad` may be caller-owned, as above)."""
    _require_device(pages, "pages")
    nbytes = pages.numel() * pages.element_size()
    count = nbytes // 4096 if count is None else int(count)
    if count * 4096 > nbytes:
        raise CRC32CError("diskqueue_check_pages: pages extend past the tensor")
    ok, bad = _outputs(pages, count, ok, bad, "diskqueue_check_pages")
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_diskqueue_check_pages(_vp(pages), count, _vp(ok), _vp(bad), _stream_handle(stream))
    _check(rc, "fdb_diskqueue_check_pages")
    return ok, bad


def _page_count(pages, page_size, count, who):
    _require_device(pages, "pages")
    nbytes = pages.numel() * pages.element_size()
    count = nbytes // page_size if count is None else int(count)
    if count * page_size > nbytes:
        raise CRC32CError(f"{who}: pages extend past the tensor")
    return count


def sqlite_seal_pages(pages, page_size, count=None, first_pgno=1, stream=None):
    """Seals a batch of SQLite pages in place as the codec's page writes do
    (checksum(write = true): the XXH3 trailer; page 1 also at 1024 bytes when
    page_size > 1024).  Asynchronous on `stream`."""
    count = _page_count(pages, page_size, count, "sqlite_seal_pages")
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_sqlite_seal_pages(_vp(pages), page_size, count, first_pgno, _stream_handle(stream))
    _check(rc, "fdb_sqlite_seal_pages")
    return pages


def diskqueue_seal_pages(pages, count=None, stream=None):
    """Page::updateHash over a batch of 4 KiB DiskQueue pages, in place, by
    each page's implementationVersion.  Asynchronous on `stream`."""
    count = _page_count(pages, 4096, count, "diskqueue_seal_pages")
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_diskqueue_seal_pages(_vp(pages), count, _stream_handle(stream))
    _check(rc, "fdb_diskqueue_seal_pages")
    return pages


CODEC_READ, CODEC_WRITE_DB, CODEC_WRITE_JOURNAL = 3, 6, 7


def sqlite_codec_pages(pages, page_size, op, reserve_size=8, count=None, first_pgno=1, stream=None, status=None):
    """The pager's codec hook (PageChecksumCodec::codec, KeyValueStoreSQLite.cpp:203-244)
    over a batch of pages, in place: op 3 verifies, ops 6 / 7 seal.  Returns
    the status tensor: 0 where codec() returns nullptr, else the check that
    accepted the page (reads) or 2 (writes).  Other ops raise CRC32CError, as
    the reference asserts."""
    count = _page_count(pages, page_size, count, "sqlite_codec_pages")
    if status is None:
        status = torch.empty(max(count, 1), dtype=torch.uint8, device=pages.device)
    _require_device(status, "sqlite_codec_pages: status", pages.device, (torch.uint8,), count)
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_sqlite_codec_pages(_vp(pages), page_size, reserve_size, count, first_pgno, op, _vp(status),
                                           _stream_handle(stream))
    _check(rc, "fdb_sqlite_codec_pages")
    return status[:count]
