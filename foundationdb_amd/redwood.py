"""Python host mirror of the batched Redwood page checks (include/fdb_redwood.h).

Reference interfaces: ArenaPage::postReadHeader(pageID) / postReadPayload(pageID)
and ArenaPage::preWrite(pageID) (fdbserver/kvstore/IPager.h:500-565), run by
the Redwood pager one page at a time (VersionedBTree.cpp:2842-2844, 2595),
here over whole batches of device-resident pages.  The per-page outcome is the
error the reference would throw first (STATUS_*), or OK.  No CPU fallback.
"""
import ctypes

import torch

from .crc32c import CRC32CError, _check, _require_device, _stream_handle, lib

(STATUS_OK, STATUS_HEADER_VERSION_NOT_SUPPORTED, STATUS_HEADER_CHECKSUM_FAILED, STATUS_HEADER_WRONG_PAGE_ID,
 STATUS_ENCODING_NOT_SUPPORTED, STATUS_DECODING_FAILED) = range(6)

_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        L.fdb_redwood_verify_pages.restype = ctypes.c_int
        L.fdb_redwood_verify_pages.argtypes = [vp, u64, u64, vp, u32, vp, vp, vp]
        L.fdb_redwood_seal_pages.restype = ctypes.c_int
        L.fdb_redwood_seal_pages.argtypes = [vp, u64, u64, vp, u32, vp, vp]
        L.fdb_redwood_workspace_bytes.restype = u64
        L.fdb_redwood_workspace_bytes.argtypes = [u64, u64]
        L.fdb_redwood_verify_pages_ws.restype = ctypes.c_int
        L.fdb_redwood_verify_pages_ws.argtypes = [vp, u64, u64, vp, u32, vp, vp, vp, u64, vp]
        L.fdb_redwood_seal_pages_ws.restype = ctypes.c_int
        L.fdb_redwood_seal_pages_ws.argtypes = [vp, u64, u64, vp, u32, vp, vp, u64, vp]
        _bound = True
    return L


def _vp(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _args(pages, page_size, count, page_ids, who):
    _require_device(pages, "pages")
    nbytes = pages.numel() * pages.element_size()
    count = nbytes // page_size if count is None else int(count)
    if count * page_size > nbytes:
        raise CRC32CError(f"{who}: pages extend past the tensor")
    if page_ids is not None:
        _require_device(page_ids, f"{who}: page_ids", pages.device, (torch.int32, torch.uint32), count)
    return count


def verify_pages(pages, page_size, count=None, page_ids=None, first_page_id=0, stream=None, status=None, bad=None):
    """(status uint8 tensor, bad-page count tensor) for a batch of Redwood pages:
    page i is checked against PhysicalPageID page_ids[i] (an int32 / uint32
    device tensor) or first_page_id + i.  `status` and `bad` may be
    caller-owned device tensors reused across calls."""
    count = _args(pages, page_size, count, page_ids, "redwood verify_pages")
    if status is None:
        status = torch.empty(max(count, 1), dtype=torch.uint8, device=pages.device)
    _require_device(status, "redwood verify_pages: status", pages.device, (torch.uint8,), count)
    if bad is None:
        bad = torch.empty(1, dtype=torch.uint64, device=pages.device)
    _require_device(bad, "redwood verify_pages: bad", pages.device, (torch.uint64, torch.int64), 1)
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_redwood_verify_pages(_vp(pages), page_size, count, _vp(page_ids), first_page_id, _vp(status),
                                             _vp(bad), _stream_handle(stream))
    _check(rc, "fdb_redwood_verify_pages")
    return status[:count], bad


def seal_pages(pages, page_size, count=None, page_ids=None, first_page_id=0, stream=None, status=None):
    """ArenaPage::preWrite(pageID) over a batch, in place; returns the status
    tensor (OK, ENCODING_NOT_SUPPORTED: page untouched, or
    HEADER_VERSION_NOT_SUPPORTED: payload checksum written, header not)."""
    count = _args(pages, page_size, count, page_ids, "redwood seal_pages")
    if status is None:
        status = torch.empty(max(count, 1), dtype=torch.uint8, device=pages.device)
    _require_device(status, "redwood seal_pages: status", pages.device, (torch.uint8,), count)
    with torch.cuda.device(pages.device):
        rc = _lib().fdb_redwood_seal_pages(_vp(pages), page_size, count, _vp(page_ids), first_page_id, _vp(status),
                                           _stream_handle(stream))
    _check(rc, "fdb_redwood_seal_pages")
    return status[:count]


def workspace_bytes(count, page_size):
    return int(_lib().fdb_redwood_workspace_bytes(count, page_size))
