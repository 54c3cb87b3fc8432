"""Python host mirror of the batched lost-write checker (include/fdb_writechecker.h),
the engine's form of fdbrpc/AsyncFileWriteChecker.h: same page history, budget
and verification rules; all full pages of an I/O are checksummed as one batch
(host CRC, the pinned GPU pipeline, or an asynchronous device batch)."""
import ctypes

import numpy as np

from .crc32c import CRC32CError, lib

_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        u32, u64, i64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p
        P = ctypes.POINTER
        sig = {
            "fdb_wc_create": ([P(vp), i64], ctypes.c_int),
            "fdb_wc_destroy": ([vp], None),
            "fdb_wc_reset_budget": ([], None),
            "fdb_wc_budget": ([], i64),
            "fdb_wc_set_gpu_threshold": ([vp, u64], ctypes.c_int),
            "fdb_wc_write": ([vp, vp, i64, i64, u64, vp, u64, P(u64)], ctypes.c_int),
            "fdb_wc_write_done": ([vp, vp, u64], ctypes.c_int),
            "fdb_wc_read": ([vp, vp, i64, i64, P(u64)], ctypes.c_int),
            "fdb_wc_sync": ([vp, u64], ctypes.c_int),
            "fdb_wc_truncate": ([vp, i64], ctypes.c_int),
            "fdb_wc_write_device": ([vp, vp, i64, i64, u64, P(u64)], ctypes.c_int),
            "fdb_wc_read_device": ([vp, vp, i64, i64, P(u64)], ctypes.c_int),
            "fdb_wc_poll": ([vp, P(u64)], ctypes.c_int),
            "fdb_wc_wait": ([vp, u64], ctypes.c_int),
            "fdb_wc_stats": ([vp, P(u64), P(u64), P(u64), P(u64)], ctypes.c_int),
            "fdb_wc_history": ([vp, u32, P(u32), P(u64)], ctypes.c_int),
            "fdb_wc_sweep_pages": ([vp, vp, u64, P(u64)], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _bound = True
    return L


def _check(rc, what):
    if rc != 0:
        raise CRC32CError(f"{what} failed with status {rc}: {lib().crc32c_gpu_last_error().decode()}")


def reset_budget():
    _lib().fdb_wc_reset_budget()


def budget():
    return int(_lib().fdb_wc_budget())


def _host_ptr(buf):
    a = np.ascontiguousarray(buf).view(np.uint8)
    return a, a.ctypes.data, a.nbytes


class WriteChecker:
    def __init__(self, history_budget=1 << 20, gpu_threshold=None):
        L = _lib()
        h = ctypes.c_void_p()
        _check(L.fdb_wc_create(ctypes.byref(h), history_budget), "fdb_wc_create")
        self.h = h
        if gpu_threshold is not None:
            _check(L.fdb_wc_set_gpu_threshold(h, gpu_threshold), "fdb_wc_set_gpu_threshold")

    def close(self):
        if self.h:
            _lib().fdb_wc_destroy(self.h)
            self.h = None

    def write(self, buf, offset, now_ms):
        a, p, n = _host_ptr(buf)
        out = np.zeros(n // 4096 + 2, np.uint32)
        cnt = ctypes.c_uint64()
        _check(_lib().fdb_wc_write(self.h, p, n, offset, now_ms, out.ctypes.data, out.size, ctypes.byref(cnt)),
               "fdb_wc_write")
        return [int(x) for x in out[:cnt.value]]

    def write_done(self, pages):
        a = np.asarray(pages, np.uint32)
        _check(_lib().fdb_wc_write_done(self.h, a.ctypes.data, a.size), "fdb_wc_write_done")

    def read(self, buf, offset):
        a, p, n = _host_ptr(buf)
        f = ctypes.c_uint64()
        _check(_lib().fdb_wc_read(self.h, p, n, offset, ctypes.byref(f)), "fdb_wc_read")
        return f.value

    def sync(self, now_ms):
        _check(_lib().fdb_wc_sync(self.h, now_ms), "fdb_wc_sync")

    def truncate(self, size):
        _check(_lib().fdb_wc_truncate(self.h, size), "fdb_wc_truncate")

    def write_device(self, d_buf, offset, now_ms):
        t = ctypes.c_uint64()
        _check(_lib().fdb_wc_write_device(self.h, ctypes.c_void_p(d_buf.data_ptr()), d_buf.numel(), offset, now_ms,
                                          ctypes.byref(t)), "fdb_wc_write_device")
        return t.value

    def read_device(self, d_buf, offset):
        t = ctypes.c_uint64()
        _check(_lib().fdb_wc_read_device(self.h, ctypes.c_void_p(d_buf.data_ptr()), d_buf.numel(), offset,
                                         ctypes.byref(t)), "fdb_wc_read_device")
        return t.value

    def poll(self):
        a = ctypes.c_uint64()
        _check(_lib().fdb_wc_poll(self.h, ctypes.byref(a)), "fdb_wc_poll")
        return a.value

    def wait(self, ticket=(1 << 64) - 1):
        _check(_lib().fdb_wc_wait(self.h, ticket), "fdb_wc_wait")

    def stats(self):
        v = [ctypes.c_uint64() for _ in range(4)]
        _check(_lib().fdb_wc_stats(self.h, *[ctypes.byref(x) for x in v]), "fdb_wc_stats")
        return {"succeed": v[0].value, "fail": v[1].value, "history": v[2].value, "writing": v[3].value}

    def sweep_pages(self, cap=1024):
        """Pages the reference's sweep actor should re-read next (fdb_wc_sweep_pages)."""
        buf = np.zeros(max(cap, 1), np.uint32)
        n = ctypes.c_uint64()
        _check(_lib().fdb_wc_sweep_pages(self.h, buf.ctypes.data, cap, ctypes.byref(n)), "fdb_wc_sweep_pages")
        return [int(x) for x in buf[:n.value]]

    def history_entry(self, page):
        c, t = ctypes.c_uint32(), ctypes.c_uint64()
        r = _lib().fdb_wc_history(self.h, page, ctypes.byref(c), ctypes.byref(t))
        return (c.value, t.value) if r == 1 else None
