"""Python host mirror of the C ABI in include/fdb_crc32c.h.

Reference interface being mirrored: ``crc32c_append(crc, input, length)``
(contrib/crc32/include/crc32/crc32c.h:36-39, contrib/crc32/crc32c.cpp:346-356)
-- same argument meaning and total behaviour: length 0 returns the seed, any
alignment, no errors.  The batched functions are the engine's additions; they
take device (HBM) tensors and run the hand-written gfx950 kernels.  There is
no CPU fallback behind them: if the shared library or a GPU is missing they
raise.

torch is used only as plumbing (device memory, streams).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDBCRC_LIB") or os.path.join(_HERE, "lib", "libfdb_crc32c.so")
TESTUTIL_LIB_PATH = os.path.join(_HERE, "lib", "libfdb_crc32c_testutil.so")


class CRC32CError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libfdb_crc32c.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CRC32CError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        L.crc32c_append.restype = u32
        L.crc32c_append.argtypes = [u32, vp, ctypes.c_size_t]
        L.crc32c_shift.restype = u32
        L.crc32c_shift.argtypes = [u32, u64]
        L.crc32c_combine.restype = u32
        L.crc32c_combine.argtypes = [u32, u32, u64]
        L.crc32c_append_zeros.restype = u32
        L.crc32c_append_zeros.argtypes = [u32, u64]
        L.crc32c_gpu_init.restype = ctypes.c_int
        L.crc32c_gpu_init.argtypes = []
        L.crc32c_gpu_batch_fixed.restype = ctypes.c_int
        L.crc32c_gpu_batch_fixed.argtypes = [vp, u64, u64, u64, u32, vp, vp, vp]
        L.crc32c_gpu_batch_varlen.restype = ctypes.c_int
        L.crc32c_gpu_batch_varlen.argtypes = [vp, vp, vp, u64, u32, vp, vp, vp]
        L.crc32c_gpu_varlen_workspace_bytes.restype = u64
        L.crc32c_gpu_varlen_workspace_bytes.argtypes = [u64]
        L.crc32c_gpu_batch_varlen_ws.restype = ctypes.c_int
        L.crc32c_gpu_batch_varlen_ws.argtypes = [vp, vp, vp, u64, u32, vp, vp, vp, u64, vp]
        L.crc32c_gpu_last_error.restype = ctypes.c_char_p
        L.crc32c_gpu_last_error.argtypes = []
        L.crc32c_gpu_version.restype = ctypes.c_char_p
        L.crc32c_gpu_version.argtypes = []
        L.crc32c_pipeline_create.restype = ctypes.c_int
        L.crc32c_pipeline_create.argtypes = [ctypes.POINTER(vp), u64, ctypes.c_int]
        L.crc32c_pipeline_destroy.restype = None
        L.crc32c_pipeline_destroy.argtypes = [vp]
        L.crc32c_pipeline_varlen.restype = ctypes.c_int
        L.crc32c_pipeline_varlen.argtypes = [vp, vp, vp, vp, u64, u32, vp, vp]
        L.crc32c_pipeline_fixed.restype = ctypes.c_int
        L.crc32c_pipeline_fixed.argtypes = [vp, vp, u64, u64, u64, u32, vp, vp]
        L.crc32c_pipeline_submit_varlen.restype = ctypes.c_int
        L.crc32c_pipeline_submit_varlen.argtypes = [vp, vp, vp, vp, u64, u32, vp, vp, ctypes.POINTER(u64)]
        L.crc32c_pipeline_submit_fixed.restype = ctypes.c_int
        L.crc32c_pipeline_submit_fixed.argtypes = [vp, vp, u64, u64, u64, u32, vp, vp, ctypes.POINTER(u64)]
        L.crc32c_pipeline_poll.restype = ctypes.c_int
        L.crc32c_pipeline_poll.argtypes = [vp, u64]
        L.crc32c_pipeline_wait.restype = ctypes.c_int
        L.crc32c_pipeline_wait.argtypes = [vp, u64]
        L.fdb_sqlite_verify_pages_host.restype = ctypes.c_int
        L.fdb_sqlite_verify_pages_host.argtypes = [vp, vp, u64, u64, u32, vp, vp]
        L.fdb_sqlite_verify_pages_host_submit.restype = ctypes.c_int
        L.fdb_sqlite_verify_pages_host_submit.argtypes = [vp, vp, u64, u64, u32, vp, vp, ctypes.POINTER(u64)]
        L.fdb_diskqueue_check_pages_host.restype = ctypes.c_int
        L.fdb_diskqueue_check_pages_host.argtypes = [vp, vp, u64, vp, vp]
        L.fdb_diskqueue_check_pages_host_submit.restype = ctypes.c_int
        L.fdb_diskqueue_check_pages_host_submit.argtypes = [vp, vp, u64, vp, vp, ctypes.POINTER(u64)]
        L.crc32c_gpu_batch_chained.restype = ctypes.c_int
        L.crc32c_gpu_batch_chained.argtypes = [vp, vp, vp, u64, vp, u64, u32, vp, vp, vp]
        L.crc32c_gpu_chained_workspace_bytes.restype = u64
        L.crc32c_gpu_chained_workspace_bytes.argtypes = [u64]
        L.crc32c_gpu_batch_chained_ws.restype = ctypes.c_int
        L.crc32c_gpu_batch_chained_ws.argtypes = [vp, vp, vp, u64, vp, u64, u32, vp, vp, vp, u64, vp]
        L.crc32c_host_impl.restype = ctypes.c_char_p
        L.crc32c_host_impl.argtypes = []
        L.crc32c_gpu_release_stream.restype = ctypes.c_int
        L.crc32c_gpu_release_stream.argtypes = [vp]
        L.crc32c_gpu_stream_bytes.restype = u64
        L.crc32c_gpu_stream_bytes.argtypes = [vp]
        L.crc32c_gpu_stream_status.restype = ctypes.c_int
        L.crc32c_gpu_stream_status.argtypes = [vp]
        L.crc32c_gpu_workspace_status.restype = ctypes.c_int
        L.crc32c_gpu_workspace_status.argtypes = [vp, vp]
        L.crc32c_host_register.restype = ctypes.c_int
        L.crc32c_host_register.argtypes = [vp, u64]
        L.crc32c_host_unregister.restype = ctypes.c_int
        L.crc32c_host_unregister.argtypes = [vp]
        _lib = L
    return _lib


_tlib = None


def testutil_lib():
    """libfdb_crc32c_testutil.so: synthetic data and LDS poisoning for tests
    and bench.py (a separate library; nothing in the product links it)."""
    global _tlib
    if _tlib is None:
        if not os.path.exists(TESTUTIL_LIB_PATH):
            raise CRC32CError(f"{TESTUTIL_LIB_PATH} missing: run `make`")
        L = ctypes.CDLL(TESTUTIL_LIB_PATH)
        L.crc32c_testutil_fill_splitmix64.restype = ctypes.c_int
        L.crc32c_testutil_fill_splitmix64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                      ctypes.c_void_p]
        L.crc32c_testutil_poison_lds.restype = ctypes.c_int
        L.crc32c_testutil_poison_lds.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        _tlib = L
    return _tlib


# ---------------------------------------------------------------- host scalar

def crc32c_append(crc, data):
    """Same semantics as the reference crc32c_append (host, synchronous)."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data)
        return lib().crc32c_append(crc & 0xFFFFFFFF, b, len(b))
    import numpy as np
    a = np.ascontiguousarray(data).view(np.uint8)
    return lib().crc32c_append(crc & 0xFFFFFFFF, a.ctypes.data, a.nbytes)


def crc32c_shift(reg, nbytes):
    return lib().crc32c_shift(reg & 0xFFFFFFFF, nbytes)


def crc32c_combine(crc_a, crc_b, len_b):
    return lib().crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def crc32c_append_zeros(crc, nzeros):
    return lib().crc32c_append_zeros(crc & 0xFFFFFFFF, nzeros)


# ---------------------------------------------------------------- device batch

def _check(rc, what):
    if rc != 0:
        msg = lib().crc32c_gpu_last_error().decode()
        raise CRC32CError(f"{what} failed with status {rc}: {msg}")


def _stream_handle(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _require_device(t, name, device=None, dtypes=None, min_numel=None):
    """Every tensor handed to the C ABI: on the GPU (on `device` if given),
    contiguous (the kernels read flat memory), of an accepted dtype, and at
    least `min_numel` elements (the kernels write out[0..count) and read
    seeds[0..count) without bounds)."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise CRC32CError(f"{name} must be a device (HBM) tensor")
    if device is not None and t.device != device:
        raise CRC32CError(f"{name} is on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise CRC32CError(f"{name} must be contiguous")
    if dtypes is not None and t.dtype not in dtypes:
        raise CRC32CError(f"{name} has dtype {t.dtype}, expected one of {[str(d) for d in dtypes]}")
    if min_numel is not None and t.numel() < min_numel:
        raise CRC32CError(f"{name} has {t.numel()} elements, needs at least {min_numel}")


U32 = (torch.uint32, torch.int32)
I64 = (torch.int64, torch.uint64)
U64 = (torch.uint64, torch.int64)


def gpu_init():
    _check(lib().crc32c_gpu_init(), "crc32c_gpu_init")


def batch_fixed(buf, stride, length, count, seed=0, seeds=None, out=None, stream=None, byte_offset=0):
    """CRC of buffer i = bytes [byte_offset + i*stride, +length) of device tensor `buf`.

    Returns a uint32 device tensor of `count` checksums (bit-identical to
    crc32c_append(seed or seeds[i], ...)).  Asynchronous on `stream`.
    """
    _require_device(buf, "buf")
    count, stride, length, byte_offset = int(count), int(stride), int(length), int(byte_offset)
    if min(count, stride, length, byte_offset) < 0:
        raise CRC32CError("batch_fixed: negative count/stride/length/byte_offset")
    if count and byte_offset + (count - 1) * stride + length > buf.numel() * buf.element_size():
        raise CRC32CError("batch_fixed: buffers extend past the end of `buf`")
    if out is None:
        out = torch.empty(count, dtype=torch.uint32, device=buf.device)
    _require_device(out, "out", buf.device, U32, count)
    sp = None
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U32, count)
        sp = ctypes.c_void_p(seeds.data_ptr())
    with torch.cuda.device(buf.device):
        rc = lib().crc32c_gpu_batch_fixed(ctypes.c_void_p(buf.data_ptr() + byte_offset), stride, length, count,
                                          seed & 0xFFFFFFFF, sp, ctypes.c_void_p(out.data_ptr()),
                                          _stream_handle(stream))
    _check(rc, "crc32c_gpu_batch_fixed")
    return out


def varlen_workspace_bytes(count):
    return int(lib().crc32c_gpu_varlen_workspace_bytes(int(count)))


def batch_varlen(buf, offsets, lengths, seed=0, seeds=None, out=None, stream=None, workspace=None):
    """CRC of buffer i = bytes [offsets[i], offsets[i]+lengths[i]) of device tensor `buf`.

    `workspace`: optional uint8 device tensor of at least varlen_workspace_bytes(count)
    bytes (caller-owned planning workspace; otherwise the library's per-stream one).
    """
    _require_device(buf, "buf")
    _require_device(offsets, "offsets", buf.device, I64)
    _require_device(lengths, "lengths", buf.device, I64)
    count = offsets.numel()
    if lengths.numel() != count:
        raise CRC32CError("offsets and lengths differ in size")
    if out is None:
        out = torch.empty(count, dtype=torch.uint32, device=buf.device)
    _require_device(out, "out", buf.device, U32, count)
    sp = None
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U32, count)
        sp = ctypes.c_void_p(seeds.data_ptr())
    with torch.cuda.device(buf.device):
        if workspace is None:
            rc = lib().crc32c_gpu_batch_varlen(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
                                               ctypes.c_void_p(lengths.data_ptr()), count, seed & 0xFFFFFFFF, sp,
                                               ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
        else:
            _require_device(workspace, "workspace", buf.device)
            rc = lib().crc32c_gpu_batch_varlen_ws(
                ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
                ctypes.c_void_p(lengths.data_ptr()), count, seed & 0xFFFFFFFF, sp, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(workspace.data_ptr()), workspace.numel() * workspace.element_size(),
                _stream_handle(stream))
    _check(rc, "crc32c_gpu_batch_varlen")
    return out


def batch_chained(buf, seg_offsets, seg_lengths, chain_starts, seed=0, seeds=None, out=None, stream=None):
    """One CRC per chain of segments (crc32c_gpu_batch_chained): chain c is
    segments [chain_starts[c], chain_starts[c+1]) of (seg_offsets, seg_lengths)
    into device tensor `buf`, fed in order with the running CRC as the next
    seed -- e.g. MutationRef's crc = type; append(param1); append(param2)."""
    _require_device(buf, "buf")
    _require_device(seg_offsets, "seg_offsets", buf.device, I64)
    _require_device(seg_lengths, "seg_lengths", buf.device, I64)
    _require_device(chain_starts, "chain_starts", buf.device, I64)
    nsegs = seg_offsets.numel()
    if seg_lengths.numel() != nsegs:
        raise CRC32CError("seg_offsets and seg_lengths differ in size")
    nchains = max(chain_starts.numel() - 1, 0)
    if out is None:
        out = torch.empty(nchains, dtype=torch.uint32, device=buf.device)
    _require_device(out, "out", buf.device, U32, nchains)
    sp = None
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U32, nchains)
        sp = ctypes.c_void_p(seeds.data_ptr())
    with torch.cuda.device(buf.device):
        rc = lib().crc32c_gpu_batch_chained(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(seg_offsets.data_ptr()),
                                            ctypes.c_void_p(seg_lengths.data_ptr()), nsegs,
                                            ctypes.c_void_p(chain_starts.data_ptr()), nchains, seed & 0xFFFFFFFF, sp,
                                            ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
    _check(rc, "crc32c_gpu_batch_chained")
    return out


def host_impl():
    """"sse4.2" or "sliced": the implementation behind the host crc32c_append."""
    return lib().crc32c_host_impl().decode()


def release_stream(stream):
    """Free the library's per-stream state (workspace, page counters) before
    the stream is destroyed (crc32c_gpu_release_stream)."""
    _check(lib().crc32c_gpu_release_stream(_stream_handle(stream)), "crc32c_gpu_release_stream")


def stream_status(stream=None):
    """Wait for `stream`; raise CRC32CError (EINVAL) if a varlen/chained batch
    on it was refused on the device since the last check (crc32c_gpu_stream_status)."""
    _check(lib().crc32c_gpu_stream_status(_stream_handle(stream)), "crc32c_gpu_stream_status")


def workspace_status(workspace, stream=None):
    """Wait for `stream`; raise CRC32CError (EINVAL) if the last batch planned in
    the caller-owned `workspace` was refused (crc32c_gpu_workspace_status)."""
    _require_device(workspace, "workspace")
    _check(lib().crc32c_gpu_workspace_status(ctypes.c_void_p(workspace.data_ptr()), _stream_handle(stream)),
           "crc32c_gpu_workspace_status")


def stream_bytes(stream=None):
    """Device bytes the library holds for `stream` (crc32c_gpu_stream_bytes)."""
    return int(lib().crc32c_gpu_stream_bytes(_stream_handle(stream)))


def poison_lds(pattern=0xA5A5A5A5, blocks=2048, stream=None):
    """Test utility: leave garbage in every CU's LDS (testutil/fdb_crc32c_testutil.h)."""
    _check(testutil_lib().crc32c_testutil_poison_lds(pattern & 0xFFFFFFFF, blocks, _stream_handle(stream)),
           "poison_lds")


def fill_splitmix64(buf, state, stream=None):
    """Test/bench utility: fill a device tensor with the BASELINE.md splitmix64 word stream."""
    _require_device(buf, "buf")
    nbytes = buf.numel() * buf.element_size()
    if nbytes % 8:
        raise CRC32CError("fill_splitmix64 needs a multiple of 8 bytes")
    with torch.cuda.device(buf.device):
        rc = testutil_lib().crc32c_testutil_fill_splitmix64(ctypes.c_void_p(buf.data_ptr()), nbytes // 8, state,
                                                            _stream_handle(stream))
    _check(rc, "crc32c_testutil_fill_splitmix64")
    return buf


# ---------------------------------------------------------------- host pipeline

class Pipeline:
    """Host-resident batches: pinned H2D -> kernel -> D2H over `nstreams` streams.

    Arguments are host buffers (numpy arrays or pinned torch CPU tensors);
    results come back in host memory.  Mirrors crc32c_pipeline_* in
    include/fdb_crc32c.h.
    """

    def __init__(self, segment_bytes=64 << 20, nstreams=4, device=None):
        import numpy as np  # noqa: F401
        self._p = ctypes.c_void_p()
        # ticket -> (host arrays the C job points into, results): held until
        # poll/wait reports the job done (or close()), whether or not the
        # caller keeps its PipelineJob -- the C side keeps raw pointers to all
        # of them and touches them from any later submit/poll/wait
        self._live = {}
        ctx = torch.cuda.device(device) if device is not None else _NullCtx()
        with ctx:
            _check(lib().crc32c_pipeline_create(ctypes.byref(self._p), segment_bytes, nstreams),
                   "crc32c_pipeline_create")

    def close(self):
        if self._p:
            lib().crc32c_pipeline_destroy(self._p)  # synchronises every lane first
            self._p = ctypes.c_void_p()
        self._live.clear()

    def _job(self, ticket, result, keep):
        self._live[ticket] = (keep, result)
        if len(self._live) > 64:  # drop what finished behind the caller's back (jobs never polled)
            for t in [t for t in self._live if t != ticket]:
                if lib().crc32c_pipeline_poll(self._p, t) != 0:
                    self._live.pop(t, None)
        return PipelineJob(self, ticket, result)

    def _retired(self, ticket):
        self._live.pop(ticket, None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _addr(a):
        if isinstance(a, torch.Tensor):
            if a.is_cuda:
                raise CRC32CError("Pipeline takes host buffers")
            return a.data_ptr()
        return a.ctypes.data

    # The host arrays of a submitted job must stay alive until it completes:
    # the pipeline keeps references to them per ticket (self._live).
    def _varlen_args(self, buf, offsets, lengths, seeds, out):
        import numpy as np
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        n = offsets.size
        if lengths.size != n:
            raise CRC32CError("offsets and lengths differ in size")
        if n and int((offsets + lengths).max()) > _nbytes(buf):
            raise CRC32CError("pipeline varlen: buffers extend past the end of `buf`")
        out = _host_out(out, n, np.uint32)
        sd = None if seeds is None else _host_seeds(seeds, n)
        return offsets, lengths, n, sd, out

    def _fixed_args(self, buf, stride, length, count, seeds, out):
        import numpy as np
        if count and (count - 1) * stride + length > _nbytes(buf):
            raise CRC32CError("pipeline fixed: buffers extend past the end of `buf`")
        return _host_out(out, count, np.uint32), None if seeds is None else _host_seeds(seeds, count)

    def submit_varlen(self, buf, offsets, lengths, seed=0, seeds=None, out=None):
        """Queue a host-resident varlen batch; returns a PipelineJob (poll()/wait())."""
        offsets, lengths, n, sd, out = self._varlen_args(buf, offsets, lengths, seeds, out)
        t = ctypes.c_uint64()
        _check(lib().crc32c_pipeline_submit_varlen(self._p, ctypes.c_void_p(self._addr(buf)), offsets.ctypes.data,
                                                   lengths.ctypes.data, n, seed & 0xFFFFFFFF, _np_ptr(sd),
                                                   ctypes.c_void_p(self._addr(out)), ctypes.byref(t)),
               "crc32c_pipeline_submit_varlen")
        return self._job(t.value, out, keep=(buf, offsets, lengths, sd))

    def submit_fixed(self, buf, stride, length, count, seed=0, seeds=None, out=None):
        out, sd = self._fixed_args(buf, stride, length, count, seeds, out)
        t = ctypes.c_uint64()
        _check(lib().crc32c_pipeline_submit_fixed(self._p, ctypes.c_void_p(self._addr(buf)), stride, length, count,
                                                  seed & 0xFFFFFFFF, _np_ptr(sd), ctypes.c_void_p(self._addr(out)),
                                                  ctypes.byref(t)), "crc32c_pipeline_submit_fixed")
        return self._job(t.value, out, keep=(buf, sd))

    def varlen(self, buf, offsets, lengths, seed=0, seeds=None, out=None):
        offsets, lengths, n, sd, out = self._varlen_args(buf, offsets, lengths, seeds, out)
        _check(lib().crc32c_pipeline_varlen(self._p, ctypes.c_void_p(self._addr(buf)), offsets.ctypes.data,
                                            lengths.ctypes.data, n, seed & 0xFFFFFFFF, _np_ptr(sd),
                                            ctypes.c_void_p(self._addr(out))), "crc32c_pipeline_varlen")
        return out

    def fixed(self, buf, stride, length, count, seed=0, seeds=None, out=None):
        out, sd = self._fixed_args(buf, stride, length, count, seeds, out)
        _check(lib().crc32c_pipeline_fixed(self._p, ctypes.c_void_p(self._addr(buf)), stride, length, count,
                                           seed & 0xFFFFFFFF, _np_ptr(sd), ctypes.c_void_p(self._addr(out))),
               "crc32c_pipeline_fixed")
        return out

    # ---- host-resident page verifiers (include/fdb_pagecheck.h)
    def sqlite_verify_pages(self, pages, page_size, count=None, first_pgno=1, submit=False):
        """Status byte per page (pagecheck.STATUS_*) and the bad-page count for
        host-resident SQLite pages; submit=True returns a PipelineJob whose
        result is (status, bad)."""
        import numpy as np
        count = _nbytes(pages) // page_size if count is None else int(count)
        if count * page_size > _nbytes(pages):
            raise CRC32CError("sqlite_verify_pages: pages extend past the buffer")
        status = np.empty(count, np.uint8)
        bad = np.zeros(1, np.uint64)
        if submit:
            t = ctypes.c_uint64()
            _check(lib().fdb_sqlite_verify_pages_host_submit(self._p, ctypes.c_void_p(self._addr(pages)), page_size,
                                                             count, first_pgno, status.ctypes.data, bad.ctypes.data,
                                                             ctypes.byref(t)), "fdb_sqlite_verify_pages_host_submit")
            return self._job(t.value, (status, bad), keep=(pages,))
        _check(lib().fdb_sqlite_verify_pages_host(self._p, ctypes.c_void_p(self._addr(pages)), page_size, count,
                                                  first_pgno, status.ctypes.data, bad.ctypes.data),
               "fdb_sqlite_verify_pages_host")
        return status, bad

    def diskqueue_check_pages(self, pages, count=None, submit=False):
        import numpy as np
        count = _nbytes(pages) // 4096 if count is None else int(count)
        if count * 4096 > _nbytes(pages):
            raise CRC32CError("diskqueue_check_pages: pages extend past the buffer")
        ok = np.empty(count, np.uint8)
        bad = np.zeros(1, np.uint64)
        if submit:
            t = ctypes.c_uint64()
            _check(lib().fdb_diskqueue_check_pages_host_submit(self._p, ctypes.c_void_p(self._addr(pages)), count,
                                                               ok.ctypes.data, bad.ctypes.data, ctypes.byref(t)),
                   "fdb_diskqueue_check_pages_host_submit")
            return self._job(t.value, (ok, bad), keep=(pages,))
        _check(lib().fdb_diskqueue_check_pages_host(self._p, ctypes.c_void_p(self._addr(pages)), count,
                                                    ok.ctypes.data, bad.ctypes.data), "fdb_diskqueue_check_pages_host")
        return ok, bad


class PipelineJob:
    """A submitted host-resident batch (crc32c_pipeline_poll / _wait)."""

    def __init__(self, pipe, ticket, result):
        self.pipe, self.ticket, self.result = pipe, ticket, result
        self.done = False

    def poll(self):
        """Non-blocking: True once the job's results are in place."""
        if not self.done:
            rc = lib().crc32c_pipeline_poll(self.pipe._p, self.ticket)
            if rc < 0:
                self.pipe._retired(self.ticket)  # finished (failed): the C side no longer touches its arrays
                _check(rc, "crc32c_pipeline_poll")
            self.done = rc == 1
            if self.done:
                self.pipe._retired(self.ticket)
        return self.done

    def wait(self):
        if not self.done:
            rc = lib().crc32c_pipeline_wait(self.pipe._p, self.ticket)
            self.pipe._retired(self.ticket)  # finished either way
            _check(rc, "crc32c_pipeline_wait")
            self.done = True
        return self.result


def _nbytes(a):
    if isinstance(a, torch.Tensor):
        return a.numel() * a.element_size()
    return a.nbytes


def _np_ptr(a):
    return None if a is None else a.ctypes.data


def _host_out(out, n, dtype):
    import numpy as np
    if out is None:
        return np.empty(n, dtype=dtype)
    if isinstance(out, torch.Tensor):
        if out.is_cuda or not out.is_contiguous() or out.numel() < n or out.element_size() != 4:
            raise CRC32CError("out must be a contiguous host array of >= count 32-bit elements")
        return out
    if not out.flags.c_contiguous or out.size < n or out.dtype.itemsize != 4:
        raise CRC32CError("out must be a contiguous host array of >= count 32-bit elements")
    return out


def _host_seeds(seeds, n):
    import numpy as np
    sd = np.ascontiguousarray(seeds, dtype=np.uint32)
    if sd.size < n:
        raise CRC32CError("seeds has fewer than count elements")
    return sd


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
