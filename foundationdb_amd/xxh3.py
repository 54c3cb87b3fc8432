"""Python host mirror of the batched XXH3-64 C ABI (include/fdb_xxh3.h).

Reference interface: ``XXH3_64bits(data, len)`` and
``XXH3_64bits_withSeed(data, len, seed)`` (flow/include/flow/xxhash.h:456,465,
xxHash v0.8.0) -- same results for every input, length and seed.  Device
(HBM) tensors in, uint64 digests out, asynchronous on a HIP stream; there is
no CPU fallback: a missing library or GPU raises.
"""
import ctypes

import torch

from .crc32c import I64, U64, CRC32CError, _check, _require_device, _stream_handle, lib

_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.xxh3_gpu_batch_fixed.restype = ctypes.c_int
        L.xxh3_gpu_batch_fixed.argtypes = [vp, u64, u64, u64, u64, vp, vp, vp]
        L.xxh3_gpu_batch_varlen.restype = ctypes.c_int
        L.xxh3_gpu_batch_varlen.argtypes = [vp, vp, vp, u64, u64, vp, vp, vp]
        L.xxh3_gpu_varlen_workspace_bytes.restype = u64
        L.xxh3_gpu_varlen_workspace_bytes.argtypes = [u64]
        L.xxh3_gpu_varlen_workspace_bytes_for.restype = u64
        L.xxh3_gpu_varlen_workspace_bytes_for.argtypes = [u64, u64]
        L.xxh3_gpu_batch_varlen_ws.restype = ctypes.c_int
        L.xxh3_gpu_batch_varlen_ws.argtypes = [vp, vp, vp, u64, u64, vp, vp, vp, u64, vp]
        L.xxh3_gpu_batch_chained.restype = ctypes.c_int
        L.xxh3_gpu_batch_chained.argtypes = [vp, vp, vp, u64, vp, u64, u64, u64, vp, vp, vp]
        _bound = True
    return L


def _vp(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def batch_fixed(buf, stride, length, count, seed=0, seeds=None, out=None, stream=None, byte_offset=0):
    """XXH3-64 of bytes [byte_offset + i*stride, +length) of device tensor `buf`, i < count."""
    _require_device(buf, "buf")
    count, stride, length, byte_offset = int(count), int(stride), int(length), int(byte_offset)
    if min(count, stride, length, byte_offset) < 0:
        raise CRC32CError("xxh3 batch_fixed: negative count/stride/length/byte_offset")
    if count and byte_offset + (count - 1) * stride + length > buf.numel() * buf.element_size():
        raise CRC32CError("xxh3 batch_fixed: buffers extend past the end of `buf`")
    if out is None:
        out = torch.empty(count, dtype=torch.uint64, device=buf.device)
    _require_device(out, "out", buf.device, U64, count)
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U64, count)
    with torch.cuda.device(buf.device):
        rc = _lib().xxh3_gpu_batch_fixed(ctypes.c_void_p(buf.data_ptr() + byte_offset), stride, length, count,
                                         seed & 0xFFFFFFFFFFFFFFFF, _vp(seeds), _vp(out), _stream_handle(stream))
    _check(rc, "xxh3_gpu_batch_fixed")
    return out


def varlen_workspace_bytes(count, total_bytes=None):
    """Workspace bytes for batch_varlen(workspace=...) of `count` buffers; with
    `total_bytes` (>= the sum of the lengths), room for the split route of
    buffers longer than 16 KiB as well."""
    if total_bytes is None:
        return int(_lib().xxh3_gpu_varlen_workspace_bytes(int(count)))
    return int(_lib().xxh3_gpu_varlen_workspace_bytes_for(int(count), int(total_bytes)))


def batch_varlen(buf, offsets, lengths, seed=0, seeds=None, out=None, stream=None, workspace=None):
    """XXH3-64 of bytes [offsets[i], +lengths[i]) of device tensor `buf` (int64 device tensors)."""
    _require_device(buf, "buf")
    _require_device(offsets, "offsets", buf.device, I64)
    _require_device(lengths, "lengths", buf.device, I64)
    n = offsets.numel()
    if lengths.numel() != n:
        raise CRC32CError("xxh3 batch_varlen: offsets and lengths differ in size")
    if out is None:
        out = torch.empty(n, dtype=torch.uint64, device=buf.device)
    _require_device(out, "out", buf.device, U64, n)
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U64, n)
    with torch.cuda.device(buf.device):
        if workspace is None:
            rc = _lib().xxh3_gpu_batch_varlen(_vp(buf), _vp(offsets), _vp(lengths), n, seed & 0xFFFFFFFFFFFFFFFF,
                                              _vp(seeds), _vp(out), _stream_handle(stream))
        else:
            _require_device(workspace, "workspace", buf.device)
            rc = _lib().xxh3_gpu_batch_varlen_ws(_vp(buf), _vp(offsets), _vp(lengths), n, seed & 0xFFFFFFFFFFFFFFFF,
                                                 _vp(seeds), _vp(out), _vp(workspace),
                                                 workspace.numel() * workspace.element_size(), _stream_handle(stream))
    _check(rc, "xxh3_gpu_batch_varlen")
    return out


def batch_chained(buf, seg_offsets, seg_lengths, chain_starts, total_bytes=None, seed=0, seeds=None, out=None,
                  stream=None):
    """XXH3-64 of each chain of segments (xxh3_gpu_batch_chained): chain c is the
    concatenation of segments [chain_starts[c], chain_starts[c+1]) -- a packet
    over a PacketBuffer chain (fdbrpc/FlowTransport.cpp:2025-2068).
    `total_bytes` bounds the sum of the segment lengths (default: computed,
    which synchronises the stream once)."""
    _require_device(buf, "buf")
    _require_device(seg_offsets, "seg_offsets", buf.device, I64)
    _require_device(seg_lengths, "seg_lengths", buf.device, I64)
    _require_device(chain_starts, "chain_starts", buf.device, I64)
    nsegs = seg_offsets.numel()
    if seg_lengths.numel() != nsegs:
        raise CRC32CError("seg_offsets and seg_lengths differ in size")
    nchains = max(chain_starts.numel() - 1, 0)
    if total_bytes is None:
        total_bytes = int(seg_lengths.sum().item()) if nsegs else 0
    if out is None:
        out = torch.empty(nchains, dtype=torch.uint64, device=buf.device)
    _require_device(out, "out", buf.device, U64, nchains)
    if seeds is not None:
        _require_device(seeds, "seeds", buf.device, U64, nchains)
    with torch.cuda.device(buf.device):
        rc = _lib().xxh3_gpu_batch_chained(_vp(buf), _vp(seg_offsets), _vp(seg_lengths), nsegs, _vp(chain_starts),
                                           nchains, int(total_bytes), seed & 0xFFFFFFFFFFFFFFFF, _vp(seeds), _vp(out),
                                           _stream_handle(stream))
    _check(rc, "xxh3_gpu_batch_chained")
    return out
