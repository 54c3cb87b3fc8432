"""Python host mirror of the batched FlowTransport receive verification
(include/fdb_packets.h).

Reference interface: scanPackets (fdbrpc/FlowTransport.cpp:1260-1366), which
walks one connection's receive buffer of [u32 len][u64 XXH3][payload] frames
and throws checksum_failed / platform_error at the first bad frame; here many
connections' device-resident buffers are verified at once and the outcome of
each is returned instead of thrown.  No CPU fallback.
"""
import ctypes

import numpy as np
import torch

from .crc32c import CRC32CError, _check, _require_device, _stream_handle, lib

OK, CHECKSUM_FAILED, LIMIT_EXCEEDED, TOO_SMALL, ECAPACITY = 0, 1, 2, 3, 4
PACKET_LIMIT = 100 << 20  # FLOW_KNOBS->PACKET_LIMIT (flow/Knobs.cpp:237)

RESULT_DTYPE = np.dtype([("consumed", np.uint64), ("frames", np.uint32), ("status", np.int32)])
FRAME_DTYPE = np.dtype([("offset", np.uint64), ("length", np.uint64), ("checksum", np.uint64),
                        ("buffer", np.uint32), ("ordinal", np.uint32)])

_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        u32, u64, vp, ci = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
        L.fdb_packets_workspace_bytes.restype = u64
        L.fdb_packets_workspace_bytes.argtypes = [u64, u64, u64]
        L.fdb_packets_verify_ws.restype = ci
        L.fdb_packets_verify_ws.argtypes = [vp, vp, vp, u64, u64, ci, u32, u64, vp, vp, u64, vp]
        L.fdb_packets_verify.restype = ci
        L.fdb_packets_verify.argtypes = [vp, vp, vp, u64, u64, ci, u32, u64, vp, vp]
        L.fdb_packets_frames.restype = ci
        L.fdb_packets_frames.argtypes = [vp, u64, u64, vp, u64, vp, vp]
        _bound = True
    return L


def _vp(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def workspace_bytes(nbuf, max_frames, total_bytes):
    return int(_lib().fdb_packets_workspace_bytes(nbuf, max_frames, total_bytes))


class PacketVerifier:
    """Caller-owned workspace for batches of up to `nbuf` receive buffers,
    `max_frames` frames and `total_bytes` bytes (fdb_packets_verify_ws): no
    allocation per call, and the frame list of the last batch stays readable."""

    def __init__(self, device, nbuf, max_frames, total_bytes):
        self.device = torch.device(device)
        self.nbuf, self.max_frames, self.total_bytes = int(nbuf), int(max_frames), int(total_bytes)
        n = workspace_bytes(self.nbuf, self.max_frames, self.total_bytes)
        if n == 0:
            raise CRC32CError("fdb_packets_workspace_bytes failed: " + lib().crc32c_gpu_last_error().decode())
        self.ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.results = torch.empty(self.nbuf * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self._n = 0
        self._stream = None

    def verify(self, data, buf_offsets, buf_lengths, checksum=True, packet_limit=PACKET_LIMIT, stream=None):
        """Starts the verification of receive buffers [data + off, + len) on
        `stream`; returns the device tensor of results (RESULT_DTYPE records,
        use results_numpy())."""
        _require_device(data, "packets: data")
        _require_device(buf_offsets, "packets: buf_offsets", data.device, (torch.int64, torch.uint64))
        _require_device(buf_lengths, "packets: buf_lengths", data.device, (torch.int64, torch.uint64))
        n = buf_offsets.numel()
        if n > self.nbuf or buf_lengths.numel() != n:
            raise CRC32CError("packets: more buffers than the verifier was sized for, or mismatched arrays")
        self._n = n
        self._stream = stream  # frames_numpy() reads the frame list on the same stream
        with torch.cuda.device(data.device):
            rc = _lib().fdb_packets_verify_ws(_vp(data), _vp(buf_offsets), _vp(buf_lengths), n, self.total_bytes,
                                              1 if checksum else 0, packet_limit, self.max_frames,
                                              _vp(self.results), _vp(self.ws), self.ws.numel(),
                                              _stream_handle(stream))
        _check(rc, "fdb_packets_verify_ws")
        return self.results[: n * RESULT_DTYPE.itemsize]

    def results_numpy(self):
        torch.cuda.synchronize(self.device)
        return self.results[: self._n * RESULT_DTYPE.itemsize].cpu().numpy().view(RESULT_DTYPE)

    def frames_numpy(self, stream=None):
        """The last batch's frame list (FRAME_DTYPE records, in no particular
        order), read on the stream verify() ran on unless `stream` is given."""
        if stream is None:
            stream = self._stream
        out = torch.empty(max(self.max_frames, 1) * FRAME_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        cnt = torch.zeros(1, dtype=torch.uint64, device=self.device)
        with torch.cuda.device(self.device):
            rc = _lib().fdb_packets_frames(_vp(self.ws), self._n, self.max_frames, _vp(out), self.max_frames,
                                           _vp(cnt), _stream_handle(stream))
        _check(rc, "fdb_packets_frames")
        torch.cuda.synchronize(self.device)
        k = int(cnt.cpu().numpy().view(np.uint64)[0])
        if k == (1 << 64) - 1:
            raise CRC32CError("fdb_packets_frames: the workspace does not hold a batch of this shape")
        k = min(k, self.max_frames)
        return out[: k * FRAME_DTYPE.itemsize].cpu().numpy().view(FRAME_DTYPE)


def verify_packets(data, buf_offsets, buf_lengths, checksum=True, packet_limit=PACKET_LIMIT, max_frames=None,
                   total_bytes=None, stream=None):
    """One-shot form (library workspace): returns the RESULT_DTYPE records as
    numpy after the stream completes.  max_frames defaults to the bound no
    batch can exceed (every delivered frame holds at least 28 bytes with
    checksums, 20 without)."""
    n = buf_offsets.numel()
    if total_bytes is None:
        total_bytes = int(buf_lengths.sum().item()) if n else 0
    if max_frames is None:
        max_frames = total_bytes // (28 if checksum else 20) + n
    res = torch.empty(max(n, 1) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=data.device)
    with torch.cuda.device(data.device):
        rc = _lib().fdb_packets_verify(_vp(data), _vp(buf_offsets), _vp(buf_lengths), n, total_bytes,
                                       1 if checksum else 0, packet_limit, max_frames, _vp(res),
                                       _stream_handle(stream))
    _check(rc, "fdb_packets_verify")
    torch.cuda.synchronize(data.device)
    return res[: n * RESULT_DTYPE.itemsize].cpu().numpy().view(RESULT_DTYPE)
