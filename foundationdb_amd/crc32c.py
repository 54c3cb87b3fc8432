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
        L.crc32c_host_register.restype = ctypes.c_int
        L.crc32c_host_register.argtypes = [vp, u64]
        L.crc32c_host_unregister.restype = ctypes.c_int
        L.crc32c_host_unregister.argtypes = [vp]
        L.crc32c_testutil_fill_splitmix64.restype = ctypes.c_int
        L.crc32c_testutil_fill_splitmix64.argtypes = [vp, u64, u64, vp]
        L.crc32c_testutil_poison_lds.restype = ctypes.c_int
        L.crc32c_testutil_poison_lds.argtypes = [u32, ctypes.c_int, vp]
        _lib = L
    return _lib


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


def _require_device(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise CRC32CError(f"{name} must be a device (HBM) tensor")


def gpu_init():
    _check(lib().crc32c_gpu_init(), "crc32c_gpu_init")


def batch_fixed(buf, stride, length, count, seed=0, seeds=None, out=None, stream=None, byte_offset=0):
    """CRC of buffer i = bytes [byte_offset + i*stride, +length) of device tensor `buf`.

    Returns a uint32 device tensor of `count` checksums (bit-identical to
    crc32c_append(seed or seeds[i], ...)).  Asynchronous on `stream`.
    """
    _require_device(buf, "buf")
    count = int(count)
    if count and byte_offset + (count - 1) * stride + length > buf.numel() * buf.element_size():
        raise CRC32CError("batch_fixed: buffers extend past the end of `buf`")
    if out is None:
        out = torch.empty(count, dtype=torch.uint32, device=buf.device)
    _require_device(out, "out")
    sp = None
    if seeds is not None:
        _require_device(seeds, "seeds")
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
    _require_device(offsets, "offsets")
    _require_device(lengths, "lengths")
    if offsets.dtype not in (torch.int64, torch.uint64) or lengths.dtype not in (torch.int64, torch.uint64):
        raise CRC32CError("offsets/lengths must be 64-bit integer tensors")
    count = offsets.numel()
    if lengths.numel() != count:
        raise CRC32CError("offsets and lengths differ in size")
    if out is None:
        out = torch.empty(count, dtype=torch.uint32, device=buf.device)
    sp = None
    if seeds is not None:
        _require_device(seeds, "seeds")
        sp = ctypes.c_void_p(seeds.data_ptr())
    with torch.cuda.device(buf.device):
        if workspace is None:
            rc = lib().crc32c_gpu_batch_varlen(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
                                               ctypes.c_void_p(lengths.data_ptr()), count, seed & 0xFFFFFFFF, sp,
                                               ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
        else:
            _require_device(workspace, "workspace")
            rc = lib().crc32c_gpu_batch_varlen_ws(
                ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
                ctypes.c_void_p(lengths.data_ptr()), count, seed & 0xFFFFFFFF, sp, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(workspace.data_ptr()), workspace.numel() * workspace.element_size(),
                _stream_handle(stream))
    _check(rc, "crc32c_gpu_batch_varlen")
    return out


def poison_lds(pattern=0xA5A5A5A5, blocks=2048, stream=None):
    """Test utility: leave garbage in every CU's LDS (see fdb_crc32c_testutil.h)."""
    _check(lib().crc32c_testutil_poison_lds(pattern & 0xFFFFFFFF, blocks, _stream_handle(stream)), "poison_lds")


def fill_splitmix64(buf, state, stream=None):
    """Fill a device tensor with the BASELINE.md splitmix64 word stream."""
    _require_device(buf, "buf")
    nbytes = buf.numel() * buf.element_size()
    if nbytes % 8:
        raise CRC32CError("fill_splitmix64 needs a multiple of 8 bytes")
    with torch.cuda.device(buf.device):
        rc = lib().crc32c_testutil_fill_splitmix64(ctypes.c_void_p(buf.data_ptr()), nbytes // 8, state,
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
        ctx = torch.cuda.device(device) if device is not None else _NullCtx()
        with ctx:
            _check(lib().crc32c_pipeline_create(ctypes.byref(self._p), segment_bytes, nstreams),
                   "crc32c_pipeline_create")

    def close(self):
        if self._p:
            lib().crc32c_pipeline_destroy(self._p)
            self._p = ctypes.c_void_p()

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

    def varlen(self, buf, offsets, lengths, seed=0, seeds=None, out=None):
        import numpy as np
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        n = offsets.size
        if out is None:
            out = np.empty(n, dtype=np.uint32)
        sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
        _check(lib().crc32c_pipeline_varlen(self._p, ctypes.c_void_p(self._addr(buf)), offsets.ctypes.data,
                                            lengths.ctypes.data, n, seed & 0xFFFFFFFF,
                                            None if sd is None else sd.ctypes.data, ctypes.c_void_p(self._addr(out))),
               "crc32c_pipeline_varlen")
        return out

    def fixed(self, buf, stride, length, count, seed=0, seeds=None, out=None):
        import numpy as np
        if out is None:
            out = np.empty(count, dtype=np.uint32)
        sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
        _check(lib().crc32c_pipeline_fixed(self._p, ctypes.c_void_p(self._addr(buf)), stride, length, count,
                                           seed & 0xFFFFFFFF, None if sd is None else sd.ctypes.data,
                                           ctypes.c_void_p(self._addr(out))), "crc32c_pipeline_fixed")
        return out


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
