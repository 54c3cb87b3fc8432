"""Batch shapes of the BASELINE.json variable-length configs, torch-free so the
golden-vector script (tests/golden/make_golden.py), the GPU tests and
bench_workloads.py all build the very same batches.

configs[2]  Zipf packet sizes 64 B - 16 KiB        zipf_lengths(),  offsets 256 B aligned
configs[4]  log-uniform 4 KiB - 1 MiB backup chunks chunk_lengths(), offsets 4 KiB aligned

Data bytes are the splitmix64 stream (BASELINE.md generator, state 0x5EED)
laid over the whole padded extent, so buffer i is bytes
[offsets[i], offsets[i] + lengths[i]) of that stream.
"""
import hashlib

import numpy as np

STATE = 0x5EED
ZIPF_ALIGN = 256
CHUNK_ALIGN = 4096
GOLDEN_GAMMA = 0x9E3779B97F4A7C15
SHARD_BYTES = 4 << 30  # one rank's page batch: 1 Mi x 4 KiB or 512 Ki x 8 KiB pages


def shard_state(shard, state=STATE):
    """splitmix64 state whose stream starts at byte shard * SHARD_BYTES of the
    global stream (word k = mix(state + (k+1)*gamma), so a jump of n words adds
    n*gamma): BASELINE configs[3]'s whole-file scan, rank r checksumming bytes
    [r*4 GiB, (r+1)*4 GiB) of one file, each rank generating its own shard."""
    return (state + shard * (SHARD_BYTES // 8) * GOLDEN_GAMMA) & 0xFFFFFFFFFFFFFFFF


def zipf_lengths(total_bytes=1 << 30, seed=1):
    """Packet sizes: bucket k in 1..256 with P(k) ~ 1/k (Zipf, exponent 1.0),
    length = clip(64*k - u, 64, 16384) with u uniform in [0, 63]."""
    rng = np.random.default_rng(seed)
    k = np.arange(1, 257)
    p = (1.0 / k) / (1.0 / k).sum()
    mean = float((p * (64 * k - 31.5)).sum())
    n = int(total_bytes / mean)
    ks = rng.choice(k, size=n, p=p)
    u = rng.integers(0, 64, n)
    return np.clip(64 * ks - u, 64, 16384).astype(np.uint64)


def chunk_lengths(total_bytes=1 << 30, seed=5):
    """Backup-sized chunks, log-uniform on [4 KiB, 1 MiB]."""
    rng = np.random.default_rng(seed)
    out, tot = [], 0
    while tot < total_bytes:
        L = int(np.exp(rng.uniform(np.log(4096), np.log(1 << 20))))
        out.append(L)
        tot += L
    return np.array(out, dtype=np.uint64)


def layout(lengths, align):
    """Back-to-back buffers, each starting at a multiple of `align`.
    Returns (offsets u64, extent in bytes rounded up to 8)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    padded = (lengths + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offsets = np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.uint64)
    total = int(offsets[-1] + padded[-1]) if lengths.size else 0
    return offsets, (total + 7) // 8 * 8


def scattered_layout(lengths, align, seed=9):
    """The same buffers laid out in a shuffled order (packets gathered from many
    connections' receive buffers, fdbrpc/FlowTransport.cpp:1260): buffer i's
    offset is not ascending in i, so the extent route's packing check refuses
    the batch and it takes the general window route.  Same extent as layout()."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    padded = (lengths + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    perm = np.random.default_rng(seed).permutation(lengths.size)
    pos = np.concatenate([[0], np.cumsum(padded[perm])[:-1]]).astype(np.uint64)
    offsets = np.empty(lengths.size, np.uint64)
    offsets[perm] = pos
    total = int(padded.sum()) if lengths.size else 0
    return offsets, (total + 7) // 8 * 8


def lengths_digest(lengths):
    """sha256 of the little-endian u64 length list: pins the shape across numpy versions."""
    return hashlib.sha256(np.ascontiguousarray(lengths, dtype="<u8").tobytes()).hexdigest()


SHAPES = {
    "zipf": (zipf_lengths, ZIPF_ALIGN),
    "chunks": (chunk_lengths, CHUNK_ALIGN),
    # configs[2]'s packets, scattered: the general (window) route's batch
    "zipf-scattered": (zipf_lengths, ZIPF_ALIGN),
}


def shape(name):
    """(lengths, offsets, extent_bytes) of the named configs batch."""
    fn, align = SHAPES[name]
    lengths = fn()
    offsets, extent = (scattered_layout if name.endswith("-scattered") else layout)(lengths, align)
    return lengths, offsets, extent


def xxh3_seeds(n):
    """Per-buffer seeds of the seeded exact-batch XXH3 digests (Redwood's
    XXH3_64bits_withSeed call sites, fdbserver/kvstore/IPager.h:325-361)."""
    i = np.arange(n, dtype=np.uint64)
    return (i * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0xFDBEEFDB)


def array_sha256(a, dtype):
    """sha256 of the whole result array as little-endian words: any single
    wrong value (or two that cancel in xor and sum) changes it."""
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dtype).tobytes()).hexdigest()


def digest(crcs):
    """xor, sum and sha256 of a CRC-32C result array (the full-size golden pins)."""
    crcs = np.asarray(crcs, dtype=np.uint32)
    return {"xor": int(np.bitwise_xor.reduce(crcs)) if crcs.size else 0, "sum": int(crcs.astype(np.uint64).sum()),
            "sha256": array_sha256(crcs, "<u4")}


def pinned(entry):
    """The digest fields of a golden entry (every full-size entry carries all three)."""
    return {k: entry[k] for k in ("xor", "sum", "sha256")}


def digest64(h):
    """The same for XXH3-64 result arrays (hex strings, as xxh3_golden.json holds them)."""
    h = np.asarray(h, dtype=np.uint64)
    return {"xor": "%016x" % (int(np.bitwise_xor.reduce(h)) if h.size else 0), "sum": "%016x" % int(h.sum(dtype=np.uint64)),
            "sha256": array_sha256(h, "<u8")}
