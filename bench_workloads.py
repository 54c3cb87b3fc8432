"""Workloads for bench.py (BASELINE.json configs), each a synthetic input of
the named shape generated directly in HBM (or pinned host memory), plus the
CPU-baseline sample and a parity check of the last device result.

configs[0]  CPU contrib/crc32 on 65536 x 4 KiB pages        -> cpu_baseline of pages4k
configs[1]  1 Mi x 4 KiB pages, 1 GPU                        -> "pages4k" (default)
configs[2]  Zipf 64 B - 16 KiB packets, 1 GPU                -> "zipf"
configs[3]  8 KiB sqlite pages, sharded per GPU              -> "pages8k"
configs[4]  4 KiB - 1 MiB chunks; device-only rate           -> "chunks"
            (the host-to-host pipelined rate: "chunks-host")
"""
import json
import os

import numpy as np
import torch

import bench_shapes as S
import foundationdb_amd as F

ROOT = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")
STATE = S.STATE


def _golden():
    with open(GOLDEN) as fh:
        return json.load(fh)


def pmc_record(workload):
    """The committed rocprofv3 --pmc summary of a workload (profiles/pmc_<w>.json), if any."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary, if any."""
    d = pmc_record(workload)
    return None if d is None else d.get("hbm_bytes_per_launch")


def pmc_commit(workload):
    """The commit whose code the committed --pmc summary measured: the bench
    line carries it next to `traffic`, so a reader can tell whether the
    counter figure is from the code being benched."""
    d = pmc_record(workload)
    return None if d is None else d.get("commit")


class CpuSample:
    def __init__(self, desc, nbytes, buf, stride=None, length=None, count=None, offsets=None, lengths=None, seed=0,
                 ref=None, port=None, port_only=False, ref_available=None):
        self.desc, self.nbytes, self.buf = desc, nbytes, buf
        self.port_only = port_only  # no compiled reference for this path: time the oracle restatement
        self.stride, self.length, self.count = stride, length, count
        self.offsets, self.lengths, self.seed = offsets, lengths, seed
        self.ref, self.port = ref, port  # optional callables(O) for non-CRC workloads
        self.ref_available = ref_available  # optional callable(O): is `ref` built (oracle/_ref)?

    def available(self, O):
        if self.port_only:
            return False
        if self.ref_available:
            return self.ref_available(O)
        return O.xxh3_reference_available() if self.ref else O.reference_available()

    def run_reference(self, O):
        if self.ref:
            return self.ref(O)
        if self.offsets is None:
            return O.reference_batch_fixed(self.buf, self.stride, self.length, self.count, seed=self.seed)
        L = O.reference().lib
        import ctypes
        f = L.ref_batch_varlen
        f.restype = None
        f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
        out = np.zeros(self.offsets.size, np.uint32)
        f(self.buf.ctypes.data, self.offsets.ctypes.data, self.lengths.ctypes.data, self.offsets.size, self.seed,
          out.ctypes.data)
        return out

    def run_port(self, O):
        if self.port:
            return self.port(O)
        if self.offsets is None:
            return O.batch_fixed(self.buf, self.stride, self.length, self.count, seed=self.seed, threads=1)
        return O.batch_varlen(self.buf, self.offsets, self.lengths, seed=self.seed, threads=1)


class Pages:
    """configs[1] (4 KiB) and configs[3]'s per-GPU shard (8 KiB SQLite pages).
    `shard` r is bytes [r*4 GiB, (r+1)*4 GiB) of one global splitmix64 file
    (bench_shapes.shard_state): rank r of an N-GPU run checksums shard r."""

    def __init__(self, dev, shard, page_bytes=4096, count=1 << 20, seed=0):
        self.dev, self.page_bytes, self.count, self.seed, self.shard = dev, page_bytes, count, seed, shard
        self.kernel_name = "fdbcrc::k_pages4k<2>" if page_bytes == 4096 else "fdbcrc::k_pages4k<2, PAIR> (8 KiB pages as block pairs)"
        if page_bytes != 4096:
            self.metric = f"device-resident CRC32C GiB/s on {page_bytes // 1024} KiB page batches; % of HBM-read peak"
        sharded = count * page_bytes == S.SHARD_BYTES
        self.state = S.shard_state(shard) if sharded else STATE
        self.buf = torch.empty(count * page_bytes, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(self.buf, self.state)
        self.out = torch.empty(count, dtype=torch.uint32, device=dev)
        self.bytes_per_step = count * page_bytes
        self.algorithmic_bytes_per_step = count * (page_bytes + 4)
        where = f"shard {shard} (bytes [{shard}*4 GiB, +4 GiB) of one file) of " if sharded else ""
        self.data_desc = (f"synthetic: {where}the splitmix64 stream (state 0x{STATE:X}) generated in HBM, "
                          f"{count} pages x {page_bytes} B, seed 0x{seed:08x}")
        self.config = {"workload": f"{count} x {page_bytes} B pages, device-resident, fixed stride",
                       "pages": count, "page_bytes": page_bytes, "seed": seed, "stride": page_bytes}

    def step(self, stream):
        F.batch_fixed(self.buf, self.page_bytes, self.page_bytes, self.count, seed=self.seed, out=self.out,
                      stream=stream)

    def verify(self):
        got = self.out.cpu().numpy()
        d = shard_digest(self.page_bytes, self.count, self.seed, self.state)
        if d is not None:  # the reference's own digest of this exact shard (xor, sum, sha256 of every checksum)
            return S.digest(got) == S.pinned(d)
        return _spot_check(self.buf, np.arange(self.count, dtype=np.uint64) * self.page_bytes,
                           np.full(self.count, self.page_bytes, np.uint64), self.seed, got)

    def cpu_sample(self):
        from oracle import oracle as O
        n = 65536 if self.page_bytes == 4096 else 32768
        buf = O.splitmix64(n * self.page_bytes // 8, self.state).view(np.uint8)
        return CpuSample(f"{n} x {self.page_bytes} B pages (configs[0] sample of the same stream)",
                         n * self.page_bytes, buf, stride=self.page_bytes, length=self.page_bytes, count=n,
                         seed=self.seed)


def shard_digest(page_bytes, count, seed, state):
    """{xor, sum, sha256} the reference produced for this page batch (tests/golden:
    pages_full for the state 0x5EED batch, pages_shards for rank shards), or None."""
    g = _golden()
    full = g["pages_full"]
    if state == STATE and page_bytes == 4096 and count == full["count"]:
        for d in full["digests"]:
            if d["seed"] == seed:
                return d
    if state == STATE and page_bytes == 8192 and seed == 0xFDBEEFDB and count == full["digest_8k_fdbeefdb"]["count"]:
        return full["digest_8k_fdbeefdb"]
    sh = g.get("pages_shards", {})
    for name in ("pages4k", "pages8k"):
        for d in sh.get(name, []):
            if (d["state"], d["page_bytes"], d["count"], d["seed"]) == (state, page_bytes, count, seed):
                return d
    return None


def _varlen_digest(shape, lengths, seed):
    """{xor, sum, sha256} the reference produced for this exact batch (tests/golden,
    make_golden.py --varlen), or None if the batch is not a pinned one."""
    ent = _golden().get("varlen_full", {}).get(shape) if shape else None
    if ent is None or ent["lengths_sha256"] != S.lengths_digest(lengths):
        return None
    for d in ent["digests"]:
        if d["seed"] == seed:
            return S.pinned(d)
    return None


def _spot_check(buf, offsets, lengths, seed, got, n=512):
    """Recheck n random buffers with the library's independent host path."""
    rng = np.random.default_rng(0)
    idx = rng.choice(offsets.size, size=min(n, offsets.size), replace=False)
    for i in idx:
        o, l = int(offsets[i]), int(lengths[i])
        data = buf[o:o + l].cpu().numpy()
        if F.crc32c_append(seed, data) != int(got[i]):
            return False
    return True


class VarLen:
    kernel_name = ("varlen engine, the batch's route: extent (k_v7count + k_xgrab + k_xfin), "
                   "blocks (k_v7prep_b + k_bigblocks) or windows (k_v7prep_w + k_varlen7)")

    def __init__(self, dev, rank, lengths, align, desc, seed=0, metric=None, shape=None):
        self.dev, self.seed = dev, seed
        self.metric, self.shape = metric, shape
        lengths = np.asarray(lengths, dtype=np.uint64)
        offsets, extent = (S.scattered_layout if shape and shape.endswith("-scattered") else S.layout)(lengths, align)
        self.h_offsets, self.h_lengths = offsets, lengths
        self.buf = torch.empty(extent, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(self.buf, STATE)
        self.offsets = torch.from_numpy(offsets.astype(np.int64)).to(dev)
        self.lengths = torch.from_numpy(lengths.astype(np.int64)).to(dev)
        self.out = torch.empty(lengths.size, dtype=torch.uint32, device=dev)
        n = lengths.size
        self.bytes_per_step = int(lengths.sum())
        # data + u64 offset + u64 length + u32 checksum per buffer
        self.algorithmic_bytes_per_step = self.bytes_per_step + 20 * n
        self.data_desc = f"synthetic: splitmix64 stream (state 0x{STATE:X}) in HBM; {desc}"
        self.config = {"workload": desc, "buffers": int(n), "total_bytes": self.bytes_per_step,
                       "mean_len": round(self.bytes_per_step / n, 1), "align": align, "seed": seed}

    def step(self, stream):
        F.batch_varlen(self.buf, self.offsets, self.lengths, seed=self.seed, out=self.out, stream=stream)

    def verify(self):
        got = self.out.cpu().numpy()
        want = _varlen_digest(self.shape, self.h_lengths, self.seed)
        if want is not None:  # the exact configs batch: the reference's own digest of every buffer
            return S.digest(got) == want
        return _spot_check(self.buf, self.h_offsets, self.h_lengths, self.seed, got)

    def cpu_sample(self):
        from oracle import oracle as O
        # a prefix of the same buffer list of about 256 MiB
        csum = np.cumsum(self.h_lengths)
        k = int(np.searchsorted(csum, 256 << 20)) + 1
        k = min(k, self.h_lengths.size)
        # (the bytes up to the furthest of them: a scattered layout's offsets are not ascending)
        end = int((self.h_offsets[:k] + self.h_lengths[:k]).max())
        buf = O.splitmix64((end + 7) // 8, STATE).view(np.uint8)
        return CpuSample(f"first {k} buffers ({int(csum[k - 1]) >> 20} MiB) of the same list", int(csum[k - 1]), buf,
                         offsets=self.h_offsets[:k].copy(), lengths=self.h_lengths[:k].copy(), seed=self.seed)


zipf_lengths, chunk_lengths = S.zipf_lengths, S.chunk_lengths


class HostChunks:
    """configs[4], host-to-host: backup chunks in pinned host memory, checksummed
    through the pinned H2D -> kernel -> D2H pipeline (4 streams, 64 MiB segments).
    The rate includes both PCIe copies; it is PCIe-bound by design."""
    kernel_name = "host pipeline (H2D + varlen engine + D2H)"
    metric = "host-to-host CRC32C GiB/s on 4 KiB-1 MiB chunk batches (pinned H2D + kernel + D2H); % of PCIe peak"
    host_timed = True
    pcie_peak_gbs = 63.0  # PCIe Gen5 x16 per direction, MI355X_MICROARCH.md

    def __init__(self, dev, rank, seed=0):
        lengths, offsets, total = S.shape("chunks")
        self.buf = torch.empty(total, dtype=torch.uint8).pin_memory()
        dbuf = torch.empty(total, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(dbuf, STATE)
        self.buf.copy_(dbuf)
        del dbuf
        self.h_offsets, self.h_lengths, self.seed = offsets, lengths.astype(np.uint64), seed
        self.out = torch.empty(lengths.size, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
        self.pipe = F.Pipeline(segment_bytes=64 << 20, nstreams=4)
        self.bytes_per_step = int(lengths.sum())
        self.algorithmic_bytes_per_step = self.bytes_per_step + 20 * lengths.size
        self.data_desc = (f"synthetic: splitmix64 stream (state 0x{STATE:X}) in PINNED HOST memory; "
                          "log-uniform 4 KiB - 1 MiB backup chunks, ~1 GiB per batch, host-to-host")
        self.config = {"workload": "log-uniform 4 KiB - 1 MiB chunks, host-resident, pinned H2D/D2H overlapped "
                                   "(4 streams x 64 MiB segments)", "buffers": int(lengths.size),
                       "total_bytes": self.bytes_per_step, "seed": seed}

    def step(self, stream):
        self.pipe.varlen(self.buf, self.h_offsets, self.h_lengths, seed=self.seed, out=self.out)

    def verify(self):
        want = _varlen_digest("chunks", self.h_lengths, self.seed)
        if want is not None:
            return S.digest(self.out) == want
        host = self.buf.numpy()
        rng = np.random.default_rng(0)
        for i in rng.choice(self.h_offsets.size, size=256, replace=False):
            o, l = int(self.h_offsets[i]), int(self.h_lengths[i])
            if F.crc32c_append(self.seed, host[o:o + l]) != int(self.out[i]):
                return False
        return True

    def cpu_sample(self):
        from oracle import oracle as O
        csum = np.cumsum(self.h_lengths)
        k = min(int(np.searchsorted(csum, 256 << 20)) + 1, self.h_lengths.size)
        end = int((self.h_offsets[:k] + self.h_lengths[:k]).max())
        buf = self.buf.numpy()[:end]
        return CpuSample(f"first {k} buffers ({int(csum[k - 1]) >> 20} MiB) of the same list", int(csum[k - 1]), buf,
                         offsets=self.h_offsets[:k].copy(), lengths=self.h_lengths[:k].copy(), seed=self.seed)


class HostPages(HostChunks):
    """configs[1] shape, host-to-host: 1 Mi x 4 KiB pages in pinned host memory
    (pages as read from disk), checksummed through the pinned H2D -> page kernel
    -> D2H pipeline (4 streams, 64 MiB segments).  PCIe-bound by design; the
    device-resident rate of the same batch is the `pages4k` workload."""
    kernel_name = "host pipeline (H2D + fdbcrc::k_pages4k + D2H)"
    metric = "host-to-host CRC32C GiB/s on 4 KiB page batches (pinned H2D + kernel + D2H); % of PCIe peak"

    def __init__(self, dev, rank, count=1 << 20, seed=0):
        self.count, self.seed = count, seed
        self.buf = torch.empty(count * 4096, dtype=torch.uint8).pin_memory()
        dbuf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(dbuf, STATE)
        self.buf.copy_(dbuf)
        del dbuf
        self.out = torch.empty(count, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
        self.pipe = F.Pipeline(segment_bytes=64 << 20, nstreams=4)
        self.bytes_per_step = count * 4096
        self.algorithmic_bytes_per_step = count * 4100
        self.data_desc = (f"synthetic: splitmix64 stream (state 0x{STATE:X}) in PINNED HOST memory; "
                          f"{count} x 4096 B pages, host-to-host")
        self.config = {"workload": f"{count} x 4 KiB pages, host-resident, pinned H2D/D2H overlapped "
                                   "(4 streams x 64 MiB segments)", "buffers": count,
                       "total_bytes": self.bytes_per_step, "seed": seed}

    def step(self, stream):
        self.pipe.fixed(self.buf, 4096, 4096, self.count, seed=self.seed, out=self.out)

    def verify(self):
        got = self.out
        if self.count == 1 << 20:
            d = [d for d in _golden()["pages_full"]["digests"] if d["seed"] == self.seed][0]
            return S.digest(got) == S.pinned(d)
        host = self.buf.numpy()
        rng = np.random.default_rng(0)
        return all(F.crc32c_append(self.seed, host[i * 4096:(i + 1) * 4096]) == int(got[i])
                   for i in rng.choice(self.count, size=256, replace=False))

    def cpu_sample(self):
        from oracle import oracle as O
        n = 65536
        buf = self.buf.numpy()[:n * 4096]
        return CpuSample(f"first {n} x 4096 B pages of the same batch", n * 4096, buf, stride=4096, length=4096,
                         count=n, seed=self.seed)


class DryCpuPages:
    """--dry-cpu: exercises bench.py's multi-rank harness on CPU with the
    library's host crc32c_append over a small page batch.  Not a measurement."""
    kernel_name = "host crc32c_append (dry run)"
    host_timed = True
    pcie_peak_gbs = 1.0

    def __init__(self, rank, count=2048):
        self.count = count
        rng = np.random.default_rng(rank)
        self.buf = rng.integers(0, 256, count * 4096, dtype=np.uint8)
        self.out = np.zeros(count, dtype=np.uint32)
        self.bytes_per_step = count * 4096
        self.algorithmic_bytes_per_step = count * 4100
        self.data_desc = "dry run"
        self.config = {"workload": f"dry run: {count} x 4096 B pages on CPU"}

    def step(self, stream):
        for i in range(self.count):
            self.out[i] = F.crc32c_append(0, self.buf[4096 * i:4096 * (i + 1)])

    def verify(self):
        return int(self.out[0]) == F.crc32c_append(0, self.buf[:4096].tobytes())


class Xxh3Pages:
    """Batched XXH3-64 over 4 KiB pages in the SQLite page-checksum layout:
    XXH3_64bits(page, 4088) per page (fdbserver/kvstore/KeyValueStoreSQLite.cpp:112),
    1 Mi pages resident in HBM."""
    metric = "device-resident XXH3-64 GiB/s on 4 KiB page batches (4088 B hashed per page); % of HBM-read peak"
    kernel_name = "fdbxxh::k_xxh3_rows<false>"

    def __init__(self, dev, rank, count=1 << 20, length=4088, seed=0):
        import foundationdb_amd.xxh3 as X
        self.X, self.dev, self.count, self.length, self.seed = X, dev, count, length, seed
        self.buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(self.buf, STATE)
        self.out = torch.empty(count, dtype=torch.uint64, device=dev)
        self.bytes_per_step = count * length
        self.algorithmic_bytes_per_step = count * (length + 8)
        self.data_desc = (f"synthetic: splitmix64 stream (state 0x{STATE:X}) generated in HBM, {count} pages x "
                          f"4096 B, XXH3-64 of the first {length} B of each (seed {seed})")
        self.config = {"workload": f"{count} x 4096 B pages, XXH3-64 over {length} B each, device-resident",
                       "pages": count, "page_bytes": 4096, "hashed_bytes": length, "seed": seed}

    def step(self, stream):
        self.X.batch_fixed(self.buf, 4096, self.length, self.count, seed=self.seed, out=self.out, stream=stream)

    def verify(self):
        with open(os.path.join(ROOT, "tests", "golden", "xxh3_golden.json")) as fh:
            g = json.load(fh)["pages_full"]
        a = self.out.cpu().numpy().view(np.uint64)
        return S.digest64(a) == S.pinned(g)

    def cpu_sample(self):
        from oracle import oracle as O
        n = 65536
        buf = O.splitmix64(n * 4096 // 8, STATE).view(np.uint8)
        return CpuSample(f"{n} x 4096 B pages, XXH3_64bits over {self.length} B each (reference flow/xxhash.c)",
                         n * self.length, buf, ref=lambda O: O.ref_xxh3_batch_fixed(buf, 4096, self.length, n),
                         port=lambda O: O.xxh3_batch_fixed(buf, 4096, self.length, n, threads=1))


def _sqlite_pages_on_device(dev, count, kinds_per=16):
    """1 Mi SQLite pages of 4 KiB in HBM, the mix a database written by several
    FoundationDB versions holds: trailers from the current writer (XXH3,
    KeyValueStoreSQLite.cpp:106-116) on 12 of every 16 pages, from the legacy
    writer (CRC-32C, :119-128) on 3, and a corrupt trailer on 1.  Every page is
    first sealed by the engine's own write side (fdb_sqlite_seal_pages, page 1
    also at 1024 B), then the legacy CRC trailers come from the CRC batch kernel;
    verify() re-checks a sample with the CPU oracle, so nothing here is circular."""
    import foundationdb_amd.pagecheck as PC
    buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
    F.fill_splitmix64(buf, STATE)
    pages = buf.view(count, 4096)
    PC.sqlite_seal_pages(buf, 4096, count, first_pgno=1)
    c = F.batch_fixed(buf, 4096, 4088, count, seed=0xFDBEEFDB)
    kind = torch.arange(count, device=dev) % kinds_per
    tr = pages[:, 4088:4096].contiguous().view(torch.int32).view(count, 2)
    cr = (kind >= 12) & (kind < 15)
    bad = kind == 15
    tr[:, 0] = torch.where(cr, torch.zeros_like(tr[:, 0]), torch.where(bad, torch.full_like(tr[:, 0], 0x7E000001),
                                                                          tr[:, 0]))
    tr[:, 1] = torch.where(cr, c.view(torch.int32), torch.where(bad, tr[:, 1] ^ 0x5A5A5A5A, tr[:, 1]))
    pages[:, 4088:4096] = tr.view(torch.uint8).view(count, 8)
    expect = torch.where(kind < 12, 2, torch.where(cr, 1, 0)).to(torch.uint8)
    return buf, expect


class SqliteVerify:
    """SQLite whole-file page verification (SQLiteDB::checkAllPageChecksums,
    KeyValueStoreSQLite.cpp:1378-1470 -> PageChecksumCodec::checksum(write=false),
    :100-201): 1 Mi mixed 4 KiB pages, device-resident (fdb_sqlite_verify_pages)."""
    metric = "device-resident SQLite page verification GiB/s (1 Mi mixed 4 KiB pages); % of HBM-read peak"
    kernel_name = "fdb_sqlite_verify_pages (classify + k_pages4k list + k_xxh3_rows list + compare)"

    def __init__(self, dev, rank, count=1 << 20):
        import foundationdb_amd.pagecheck as PC
        self.PC, self.count = PC, count
        self.buf, self.expect = _sqlite_pages_on_device(dev, count)
        self.bytes_per_step = count * 4096
        self.algorithmic_bytes_per_step = count * (4096 + 1)
        self.data_desc = (f"synthetic: splitmix64 pages (state 0x{STATE:X}) in HBM with XXH3 / CRC-32C / corrupt "
                          "trailers 12:3:1")
        self.config = {"workload": f"{count} x 4 KiB SQLite pages, mixed trailers, device-resident", "pages": count}
        # caller-owned outputs: no allocation or fill inside the timed steps
        self.status = torch.empty(count, dtype=torch.uint8, device=dev)
        self.bad = torch.empty(1, dtype=torch.uint64, device=dev)

    def step(self, stream):
        self.PC.sqlite_verify_pages(self.buf, 4096, self.count, first_pgno=1, stream=stream, status=self.status,
                                    bad=self.bad)

    def verify(self):
        from oracle import oracle as O
        if not torch.equal(self.status, self.expect):
            return False
        if int(self.bad.cpu().numpy().view(np.uint64)[0]) != self.count // 16:
            return False
        h = self.buf.view(self.count, 4096)
        st = self.status.cpu().numpy()
        for i in np.random.default_rng(0).choice(self.count, 128, replace=False):
            if O.sqlite_verify_page(h[i].cpu().numpy(), int(i) + 1) != int(st[i]):
                return False
        return True

    def cpu_sample(self):
        n = 65536
        host = self.buf[:n * 4096].cpu().numpy()
        return CpuSample(f"first {n} pages of the batch through PageChecksumCodec::checksum(write=false) "
                         "(KeyValueStoreSQLite.cpp:118-155) composed from the reference's own crc32c_append, "
                         "XXH3_64bits and hashlittle2 compiled unmodified (oracle/ref_pagecheck.c), one page per call",
                         n * 4096, host, ref=lambda O_: O_.ref_sqlite_verify_pages(host, 4096, n, 1),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: [O_.sqlite_verify_page(host[4096 * i:4096 * (i + 1)], i + 1)
                                          for i in range(n)])


class SqliteVerifyHost(SqliteVerify):
    """The same 1 Mi pages starting in pinned host memory (as read from disk):
    fdb_sqlite_verify_pages_host through the pipeline (PCIe-bound by design)."""
    metric = "host-to-host SQLite page verification GiB/s (1 Mi mixed 4 KiB pages); % of PCIe peak"
    kernel_name = "host pipeline (H2D + fdb_sqlite_verify_pages + D2H of status bytes)"
    host_timed = True
    pcie_peak_gbs = 63.0

    def __init__(self, dev, rank, count=1 << 20):
        super().__init__(dev, rank, count)
        dbuf = self.buf
        self.buf = torch.empty(count * 4096, dtype=torch.uint8).pin_memory()
        self.buf.copy_(dbuf)
        self.expect = self.expect.cpu()
        del dbuf
        self.pipe = F.Pipeline(segment_bytes=64 << 20, nstreams=4)
        self.config = {"workload": f"{count} x 4 KiB SQLite pages, mixed trailers, host-resident, pinned pipeline "
                                   "(4 streams x 64 MiB)", "pages": count}

    def step(self, stream):
        st, bad = self.pipe.sqlite_verify_pages(self.buf, 4096, self.count, first_pgno=1)
        self.status, self.bad = torch.from_numpy(st), torch.from_numpy(bad.view(np.int64))


def _diskqueue_headers(dev, count, state):
    """Unsealed DiskQueue pages (fdbserver/kvstore/DiskQueue.cpp:1047-1120):
    splitmix64 bytes with magic + implementationVersion V2 (XXH3-64 of [8, 4096),
    the current TLog format) on 13 of every 16 pages, V1 (CRC-32C of [4, 4096),
    TLogVersion V3..V6) on 3, and V0 (hashlittle2) on every 4099th page."""
    buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
    F.fill_splitmix64(buf, state)
    pages = buf.view(count, 4096)
    kind = torch.arange(count, device=dev) % 16
    ver = torch.where((kind >= 12) & (kind < 15), 1, 2).to(torch.int16)
    v0 = torch.arange(7, count, 4099, device=dev)
    ver[v0] = 0
    hdr = torch.stack([torch.full_like(ver, 0x4D51), ver], 1)  # magic, implementationVersion
    pages[:, 8:12] = hdr.view(torch.uint8).view(count, 4)
    return buf, kind, ver


def _diskqueue_pages_on_device(dev, count):
    """1 Mi DiskQueue pages of 4 KiB in HBM, sealed by the engine's own write side
    (fdb_diskqueue_seal_pages, Page::updateHash by version), then one V2 page of
    every 16 given a wrong hash.  verify() re-checks a sample with the reference
    composition."""
    import foundationdb_amd.pagecheck as PC
    buf, kind, ver = _diskqueue_headers(dev, count, STATE ^ 0xD15C)
    PC.diskqueue_seal_pages(buf, count)
    pages = buf.view(count, 4096)
    bad = (kind == 15) & (ver == 2)
    h64 = pages[:, 0:8].contiguous().view(torch.int64).view(count)
    pages[:, 0:8] = torch.where(bad[:, None], (h64 ^ 0x5A5A).view(torch.uint8).view(count, 8), pages[:, 0:8])
    expect = torch.where(bad, 0, 1).to(torch.uint8)
    return buf, expect


class DiskQueueVerify:
    """DiskQueue page verification (Page::checkHash over a contiguous run of
    pages, DiskQueue.cpp:1230-1290 / recovery :1342-1360): 1 Mi mixed 4 KiB
    pages, device-resident (fdb_diskqueue_check_pages)."""
    metric = "device-resident DiskQueue page verification GiB/s (1 Mi mixed 4 KiB pages); % of HBM-read peak"
    kernel_name = "fdb_diskqueue_check_pages (classify + k_xxh3_rows list + k_pages4k list + lookup3 + compare)"

    def __init__(self, dev, rank, count=1 << 20):
        import foundationdb_amd.pagecheck as PC
        self.PC, self.count = PC, count
        self.buf, self.expect = _diskqueue_pages_on_device(dev, count)
        self.bytes_per_step = count * 4096
        self.algorithmic_bytes_per_step = count * (4096 + 1)
        self.data_desc = (f"synthetic: splitmix64 pages in HBM, DiskQueue V2 / V1 / corrupt 12:3:1 plus V0 pages")
        self.config = {"workload": f"{count} x 4 KiB DiskQueue pages, mixed implementationVersion, device-resident",
                       "pages": count}
        self.ok = torch.empty(count, dtype=torch.uint8, device=dev)
        self.bad = torch.empty(1, dtype=torch.uint64, device=dev)

    def step(self, stream):
        self.PC.diskqueue_check_pages(self.buf, self.count, stream=stream, ok=self.ok, bad=self.bad)

    def verify(self):
        from oracle import oracle as O
        if not torch.equal(self.ok, self.expect):
            return False
        if int(self.bad.cpu().numpy().view(np.uint64)[0]) != int((self.expect == 0).sum()):
            return False
        idx = np.random.default_rng(0).choice(self.count, 256, replace=False)
        host = self.buf.view(self.count, 4096)[torch.from_numpy(idx).to(self.buf.device)].cpu().numpy()
        ok = self.ok.cpu().numpy()
        return all(O.diskqueue_check_page(host[j]) == int(ok[i]) for j, i in enumerate(idx))

    def cpu_sample(self):
        n = 65536
        host = self.buf[:n * 4096].cpu().numpy()
        return CpuSample(f"first {n} pages through Page::checkHash (DiskQueue.cpp:1077-1120) composed from the "
                         "reference's own crc32c_append / XXH3_64bits / hashlittle2 (oracle/ref_pagecheck.c)",
                         n * 4096, host, ref=lambda O_: O_.ref_diskqueue_check_pages(host, n),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: [O_.diskqueue_check_page(host[4096 * i:4096 * (i + 1)])
                                          for i in range(n)])


class SqliteSeal:
    """SQLite page writes (the codec's op 6 / op 7, KeyValueStoreSQLite.cpp:203-244
    -> PageChecksumCodec::checksum(write=true), :107-116) over a batch: 1 Mi
    4 KiB pages sealed in place each step (fdb_sqlite_seal_pages)."""
    metric = "device-resident SQLite page sealing GiB/s (1 Mi 4 KiB pages, XXH3 trailers); % of HBM-read peak"
    kernel_name = "fdb_sqlite_seal_pages (k_xxh3_rows over the pages + k_sq_seal trailer write)"

    def __init__(self, dev, rank, count=1 << 20):
        import foundationdb_amd.pagecheck as PC
        self.PC, self.count = PC, count
        self.buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
        F.fill_splitmix64(self.buf, STATE ^ 0x5EA1)
        self.sample = np.concatenate([[0], np.random.default_rng(1).choice(np.arange(1, count), 63, replace=False)])
        self.orig = self.buf.view(count, 4096)[torch.from_numpy(self.sample).to(dev)].cpu().numpy()
        self.bytes_per_step = count * 4096
        # each page: 4088 B hashed + the 8-byte trailer written (page 1's 1024 B pass aside)
        self.algorithmic_bytes_per_step = count * 4096
        self.data_desc = f"synthetic: splitmix64 pages (state 0x{STATE ^ 0x5EA1:X}) in HBM, sealed in place"
        self.config = {"workload": f"{count} x 4 KiB SQLite pages sealed in place (page 1 also at 1024 B), "
                                   "device-resident", "pages": count}

    def step(self, stream):
        self.PC.sqlite_seal_pages(self.buf, 4096, self.count, first_pgno=1, stream=stream)

    def verify(self):
        from oracle import oracle as O
        st, bad = self.PC.sqlite_verify_pages(self.buf, 4096, self.count, first_pgno=1)
        if not bool((st == 2).all()) or int(bad.cpu().numpy().view(np.uint64)[0]) != 0:
            return False
        # page 1 also verifies as a 1024-byte page, as the codec guarantees
        st1, _ = self.PC.sqlite_verify_pages(self.buf[:1024], 1024, 1, first_pgno=1)
        if int(st1.cpu()[0]) != 2:
            return False
        got = self.buf.view(self.count, 4096)[torch.from_numpy(self.sample).to(self.buf.device)].cpu().numpy()
        seal = O.ref_sqlite_seal_pages if O.pagecheck_reference_available() else O.sqlite_seal_pages
        for j, i in enumerate(self.sample):
            want = seal(self.orig[j], 4096, 1, first_pgno=int(i) + 1)
            if not np.array_equal(got[j], want):
                return False
        return True

    def cpu_sample(self):
        from oracle import oracle as O
        n = 65536
        host = O.splitmix64(n * 4096 // 8, STATE ^ 0x5EA1).view(np.uint8)
        return CpuSample(f"{n} pages sealed in place by the codec's checksum(write=true) composed from the "
                         "reference's own XXH3_64bits compiled unmodified (oracle/ref_pagecheck.c)",
                         n * 4096, host, ref=lambda O_: O_.ref_sqlite_seal_pages(host, 4096, n, 1, inplace=True),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: O_.sqlite_seal_pages(host, 4096, n, 1))


class DiskQueueSeal:
    """DiskQueue commit-time hashing (Page::updateHash, DiskQueue.cpp:1089-1105,
    called for every page of a commit, :955-965): 1 Mi 4 KiB pages of mixed
    implementationVersion sealed in place each step (fdb_diskqueue_seal_pages)."""
    metric = ("device-resident DiskQueue page sealing GiB/s (1 Mi 4 KiB pages, V2 / V1 / V0 by version); "
              "% of HBM-read peak")
    kernel_name = "fdb_diskqueue_seal_pages (classify + k_xxh3_rows list + k_pages4k list + hash write)"

    def __init__(self, dev, rank, count=1 << 20):
        import foundationdb_amd.pagecheck as PC
        self.PC, self.count = PC, count
        self.buf, _, _ = _diskqueue_headers(dev, count, STATE ^ 0x5EA2)
        self.sample = np.concatenate([[7, 4106], np.random.default_rng(2).choice(count, 62, replace=False)])
        self.orig = self.buf.view(count, 4096)[torch.from_numpy(self.sample).to(dev)].cpu().numpy()
        self.bytes_per_step = count * 4096
        self.algorithmic_bytes_per_step = count * 4096
        self.data_desc = "synthetic: splitmix64 pages in HBM, implementationVersion V2 / V1 13:3 plus V0 pages"
        self.config = {"workload": f"{count} x 4 KiB DiskQueue pages sealed in place by implementationVersion, "
                                   "device-resident", "pages": count}

    def step(self, stream):
        self.PC.diskqueue_seal_pages(self.buf, self.count, stream=stream)

    def verify(self):
        from oracle import oracle as O
        ok, bad = self.PC.diskqueue_check_pages(self.buf, self.count)
        if not bool((ok == 1).all()) or int(bad.cpu().numpy().view(np.uint64)[0]) != 0:
            return False
        got = self.buf.view(self.count, 4096)[torch.from_numpy(self.sample).to(self.buf.device)].cpu().numpy()
        seal = O.ref_diskqueue_seal_pages if O.pagecheck_reference_available() else O.diskqueue_seal_pages
        return all(np.array_equal(got[j], seal(self.orig[j], 1)) for j in range(self.sample.size))

    def cpu_sample(self):
        n = 65536
        host = self.buf[:n * 4096].cpu().numpy()
        return CpuSample(f"first {n} pages through Page::updateHash (DiskQueue.cpp:1089-1105) composed from the "
                         "reference's own crc32c_append / XXH3_64bits / hashlittle2 (oracle/ref_pagecheck.c), in place",
                         n * 4096, host, ref=lambda O_: O_.ref_diskqueue_seal_pages(host, n, inplace=True),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: O_.diskqueue_seal_pages(host, n))


def _redwood_pages_on_device(dev, count, ps, first_id, state):
    """Redwood BTree pages in HBM as ArenaPage::init(XXHash64, BTreeNode, 1) +
    setWriteInfo(pageID, version) leave them (fdbserver/kvstore/IPager.h:448-502):
    header version 1, encoding header at 43, payload at 51, firstPhysicalPageID
    first_id + i; splitmix64 payloads.  Not sealed."""
    from oracle import oracle as O
    buf = torch.empty(count * ps, dtype=torch.uint8, device=dev)
    F.fill_splitmix64(buf, state)
    tmpl = np.zeros(O.REDWOOD_HEADER, np.uint8)
    O.redwood_init_page(tmpl, 0, page_type=2, sub_type=1, write_version=1)
    pages = buf.view(count, ps)
    pages[:, :43] = torch.from_numpy(tmpl[:43]).to(dev)
    ids = (first_id + torch.arange(count, device=dev, dtype=torch.int64)).to(torch.int32)
    pages[:, 15:19] = ids.view(torch.uint8).view(count, 4)
    return buf


class RedwoodVerify:
    """Redwood page reads (ArenaPage::postReadHeader + postReadPayload,
    fdbserver/kvstore/IPager.h:527-565, run per page by the pager at
    VersionedBTree.cpp:2842-2844) over a batch: 512 Ki BTree pages of the
    default 8 KiB (REDWOOD_DEFAULT_PAGE_SIZE, fdbserver/core/ServerKnobs.cpp:1332),
    sealed by the engine's own preWrite batch, one in 16 with a flipped payload
    byte (fdb_redwood_verify_pages)."""
    metric = ("device-resident Redwood page verification GiB/s (512 Ki 8 KiB BTree pages: header XXH3 + seeded "
              "payload XXH3); % of HBM-read peak")
    kernel_name = "fdb_redwood_verify_pages (k_rw_head + XXH3 planner + k_xxh3_vrows (seeded) + k_rw_verify_fin)"
    PS, FIRST = 8192, 1000

    def __init__(self, dev, rank, count=1 << 19):
        import foundationdb_amd.redwood as RW
        self.RW, self.count = RW, count
        ps = self.PS
        self.buf = _redwood_pages_on_device(dev, count, ps, self.FIRST, STATE ^ 0x4ED0)
        st = RW.seal_pages(self.buf, ps, count, first_page_id=self.FIRST)
        assert bool((st == 0).all())
        pages = self.buf.view(count, ps)
        bad = torch.arange(count, device=dev) % 16 == 5
        col = 51 + (torch.arange(count, device=dev) * 131) % (ps - 51)
        rows = torch.nonzero(bad).view(-1)
        pages[rows, col[rows]] ^= 0x20
        self.expect = torch.where(bad, 5, 0).to(torch.uint8)
        self.bytes_per_step = count * ps
        # every page read once (header + payload) + the status byte
        self.algorithmic_bytes_per_step = count * (ps + 1)
        self.data_desc = (f"synthetic: splitmix64 payloads (state 0x{STATE ^ 0x4ED0:X}) in HBM, Redwood header "
                          "version 1 / XXHash64 encoding, sealed by fdb_redwood_seal_pages, 1 in 16 payloads corrupt")
        self.config = {"workload": f"{count} x {ps >> 10} KiB Redwood BTree pages, device-resident", "pages": count,
                       "page_size": ps}
        self.status = torch.empty(count, dtype=torch.uint8, device=dev)
        self.nbad = torch.empty(1, dtype=torch.uint64, device=dev)

    def step(self, stream):
        self.RW.verify_pages(self.buf, self.PS, self.count, first_page_id=self.FIRST, stream=stream,
                             status=self.status, bad=self.nbad)

    def verify(self):
        from oracle import oracle as O
        if not torch.equal(self.status, self.expect):
            return False
        if int(self.nbad.cpu().numpy().view(np.uint64)[0]) != int((self.expect != 0).sum()):
            return False
        idx = np.random.default_rng(3).choice(self.count, 256, replace=False)
        host = self.buf.view(self.count, self.PS)[torch.from_numpy(idx).to(self.buf.device)].cpu().numpy()
        st = self.status.cpu().numpy()
        if O.pagecheck_reference_available():
            want, _ = O.ref_redwood_verify_pages(host, self.PS, idx.size, ids=(self.FIRST + idx).astype(np.uint32))
        else:
            want = [O.redwood_verify_page(host[j], self.FIRST + int(i)) for j, i in enumerate(idx)]
        return all(int(want[j]) == int(st[i]) for j, i in enumerate(idx))

    def cpu_sample(self):
        n = 32768
        host = self.buf[:n * self.PS].cpu().numpy()
        return CpuSample(f"first {n} pages through postReadHeader + postReadPayload (IPager.h:527-565) composed "
                         "from the reference's own XXH3_64bits / XXH3_64bits_withSeed compiled unmodified "
                         "(oracle/ref_pagecheck.c), one page per call",
                         n * self.PS, host,
                         ref=lambda O_: O_.ref_redwood_verify_pages(host, self.PS, n, first_id=self.FIRST, inplace=True),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: [O_.redwood_verify_page(host[self.PS * i:self.PS * (i + 1)], self.FIRST + i)
                                          for i in range(n)])


class RedwoodSeal:
    """Redwood page writes (ArenaPage::preWrite, fdbserver/kvstore/IPager.h:500-525,
    per page at VersionedBTree.cpp:2595): 512 Ki 8 KiB BTree pages sealed in
    place each step (fdb_redwood_seal_pages)."""
    metric = ("device-resident Redwood page sealing GiB/s (512 Ki 8 KiB BTree pages: seeded payload XXH3 + header "
              "XXH3); % of HBM-read peak")
    kernel_name = "fdb_redwood_seal_pages (k_rw_head + XXH3 planner + k_xxh3_vrows (seeded) + k_rw_seal_fin)"
    PS, FIRST = 8192, 77

    def __init__(self, dev, rank, count=1 << 19):
        import foundationdb_amd.redwood as RW
        self.RW, self.count = RW, count
        self.buf = _redwood_pages_on_device(dev, count, self.PS, self.FIRST, STATE ^ 0x4ED1)
        self.sample = np.random.default_rng(4).choice(count, 64, replace=False)
        self.orig = self.buf.view(count, self.PS)[torch.from_numpy(self.sample).to(dev)].cpu().numpy()
        self.status = torch.empty(count, dtype=torch.uint8, device=dev)
        self.bytes_per_step = count * self.PS
        self.algorithmic_bytes_per_step = count * self.PS  # each page read once, 16 header bytes written
        self.data_desc = f"synthetic: splitmix64 payloads (state 0x{STATE ^ 0x4ED1:X}), Redwood headers, sealed in place"
        self.config = {"workload": f"{count} x {self.PS >> 10} KiB Redwood BTree pages sealed in place, "
                                   "device-resident", "pages": count, "page_size": self.PS}

    def step(self, stream):
        self.RW.seal_pages(self.buf, self.PS, self.count, first_page_id=self.FIRST, stream=stream, status=self.status)

    def verify(self):
        from oracle import oracle as O
        if not bool((self.status == 0).all()):
            return False
        st, bad = self.RW.verify_pages(self.buf, self.PS, self.count, first_page_id=self.FIRST)
        if not bool((st == 0).all()) or int(bad.cpu().numpy().view(np.uint64)[0]) != 0:
            return False
        got = self.buf.view(self.count, self.PS)[torch.from_numpy(self.sample).to(self.buf.device)].cpu().numpy()
        for j, i in enumerate(self.sample):
            if O.pagecheck_reference_available():
                want, _ = O.ref_redwood_seal_pages(self.orig[j], self.PS, 1, first_id=self.FIRST + int(i))
            else:
                want = O.redwood_seal_page(self.orig[j], self.FIRST + int(i))[1]
            if not np.array_equal(got[j], want):
                return False
        return True

    def cpu_sample(self):
        n = 32768
        host = self.buf[:n * self.PS].cpu().numpy().copy()
        return CpuSample(f"first {n} pages sealed in place by preWrite (IPager.h:500-525) composed from the "
                         "reference's own XXH3_64bits / XXH3_64bits_withSeed (oracle/ref_pagecheck.c)",
                         n * self.PS, host,
                         ref=lambda O_: O_.ref_redwood_seal_pages(host, self.PS, n, first_id=self.FIRST, inplace=True),
                         ref_available=lambda O_: O_.pagecheck_reference_available(),
                         port=lambda O_: [O_.redwood_seal_page(host[self.PS * i:self.PS * (i + 1)], self.FIRST + i)
                                          for i in range(n)])


class Xxh3Zipf(VarLen):
    """XXH3-64 of every packet of the configs[2] Zipf batch (FlowTransport packet
    checksum, fdbrpc/FlowTransport.cpp:2025-2068), device-resident."""
    metric = "device-resident XXH3-64 GiB/s on Zipf 64 B-16 KiB packet batches; % of HBM-read peak"
    kernel_name = "fdbxxh planner (k_xplan + k_xscan + k_xassign) + k_xxh3_vrows"

    def __init__(self, dev, rank):
        import foundationdb_amd.xxh3 as X
        super().__init__(dev, rank, zipf_lengths(), S.ZIPF_ALIGN,
                         "Zipf(1.0) packet sizes 64 B - 16 KiB, ~1 GiB per batch, XXH3-64 per packet")
        self.X = X
        self.metric = Xxh3Zipf.metric
        self.out = torch.empty(self.h_lengths.size, dtype=torch.uint64, device=dev)
        self.algorithmic_bytes_per_step = self.bytes_per_step + 24 * self.h_lengths.size

    def step(self, stream):
        self.X.batch_varlen(self.buf, self.offsets, self.lengths, out=self.out, stream=stream)

    def verify(self):
        from oracle import oracle as O
        got = self.out.cpu().numpy().view(np.uint64)
        rng = np.random.default_rng(0)
        # every packet against the reference's own flow/xxhash.c over the same bytes
        want = O.ref_xxh3_batch_varlen(self.buf.cpu().numpy(), self.h_offsets, self.h_lengths)
        return bool(np.array_equal(got, want))

    def cpu_sample(self):
        from oracle import oracle as O
        k = 120000
        end = int((self.h_offsets[:k] + self.h_lengths[:k]).max())
        host = self.buf[:end].cpu().numpy()
        offs, lens = self.h_offsets[:k], self.h_lengths[:k]
        return CpuSample(f"first {k} packets ({int(lens.sum()) >> 20} MiB), reference flow/xxhash.c XXH3_64bits",
                         int(lens.sum()), host,
                         ref=lambda O_: O_.ref_xxh3_batch_varlen(host, offs, lens),
                         port=lambda O_: O_.xxh3_batch_varlen(host, offs, lens, threads=1))


class Xxh3Chunks(Xxh3Zipf):
    """XXH3-64 of every chunk of the configs[4] backup-chunk batch (4 KiB - 1 MiB,
    log-uniform), device-resident: the split route for every chunk over 16 KiB
    (xxh3_split.hip), the row kernel for the rest."""
    metric = "device-resident XXH3-64 GiB/s on 4 KiB-1 MiB chunk batches; % of HBM-read peak"
    kernel_name = "fdbxxh planner (k_xplan + k_xassign) + k_xlong (buffers over 16 KiB) + k_xxh3_vrows"

    def __init__(self, dev, rank):
        import foundationdb_amd.xxh3 as X
        VarLen.__init__(self, dev, rank, chunk_lengths(), 4096,
                        "log-uniform 4 KiB - 1 MiB backup chunks, ~1 GiB per batch, XXH3-64 per chunk")
        self.X = X
        self.metric = Xxh3Chunks.metric
        self.out = torch.empty(self.h_lengths.size, dtype=torch.uint64, device=dev)
        self.algorithmic_bytes_per_step = self.bytes_per_step + 24 * self.h_lengths.size

    def cpu_sample(self):
        from oracle import oracle as O
        csum = np.cumsum(self.h_lengths)
        k = min(int(np.searchsorted(csum, 256 << 20)) + 1, self.h_lengths.size)
        end = int((self.h_offsets[:k] + self.h_lengths[:k]).max())
        host = self.buf[:end].cpu().numpy()
        offs, lens = self.h_offsets[:k], self.h_lengths[:k]
        return CpuSample(f"first {k} chunks ({int(lens.sum()) >> 20} MiB), reference flow/xxhash.c XXH3_64bits",
                         int(lens.sum()), host,
                         ref=lambda O_: O_.ref_xxh3_batch_varlen(host, offs, lens),
                         port=lambda O_: O_.xxh3_batch_varlen(host, offs, lens, threads=1))


class Xxh3Chained:
    """XXH3-64 of packets laid over PacketBuffer chains (fdbrpc/FlowTransport.cpp:2025-2068:
    XXH3_64bits over one buffer, reset / update per buffer / digest when the
    packet spans several): the configs[2] Zipf packets serialized back to back
    into 4 KiB PacketBuffers whose slots lie in HBM in shuffled order, one
    chain of segments per packet (xxh3_gpu_batch_chained)."""
    metric = ("device-resident XXH3-64 GiB/s on Zipf packets over shuffled 4 KiB PacketBuffer chains; "
              "% of HBM-read peak")
    kernel_name = "xxh3_gpu_batch_chained (segment scan + gather of multi-segment chains + fdbxxh varlen)"

    def __init__(self, dev, rank, seg=4096):
        from oracle import oracle as O
        import foundationdb_amd.xxh3 as X
        self.X = X
        lens = zipf_lengths().astype(np.int64)
        pos = np.concatenate([[0], np.cumsum(lens)[:-1]])
        total = int(lens.sum())
        nbuf = (total + seg - 1) // seg
        stream = O.splitmix64((nbuf * seg + 7) // 8, STATE).view(np.uint8)[:nbuf * seg]
        slot = np.random.default_rng(7).permutation(nbuf).astype(np.int64)
        host = np.empty(nbuf * seg, np.uint8)
        host.reshape(nbuf, seg)[slot] = stream.reshape(nbuf, seg)  # buffer k lives at slot[k]
        # one segment per (packet, buffer) it touches
        b0, b1 = pos // seg, (pos + lens - 1) // seg
        nseg = (b1 - b0 + 1)
        pk = np.repeat(np.arange(lens.size), nseg)
        bk = np.repeat(b0, nseg) + (np.arange(nseg.sum()) - np.repeat(np.cumsum(nseg) - nseg, nseg))
        lo = np.maximum(pos[pk], bk * seg)
        hi = np.minimum(pos[pk] + lens[pk], (bk + 1) * seg)
        self.h_seg_off = slot[bk] * seg + (lo - bk * seg)
        self.h_seg_len = hi - lo
        self.h_starts = np.concatenate([[0], np.cumsum(nseg)])
        self.h_pos, self.h_lens, self.stream = pos, lens, stream
        self.buf = torch.from_numpy(host).to(dev)
        self.seg_off = torch.from_numpy(self.h_seg_off).to(dev)
        self.seg_len = torch.from_numpy(self.h_seg_len).to(dev)
        self.starts = torch.from_numpy(self.h_starts).to(dev)
        self.total = total
        self.out = torch.empty(lens.size, dtype=torch.uint64, device=dev)
        self.bytes_per_step = total
        # payload + per segment (offset, length) + per chain (start, digest)
        self.algorithmic_bytes_per_step = total + 16 * int(nseg.sum()) + 16 * lens.size
        multi = nseg > 1
        self.data_desc = (f"synthetic: splitmix64 stream (state 0x{STATE:X}) in {nbuf} shuffled {seg} B "
                          f"PacketBuffers; {lens.size} Zipf packets, {int(multi.sum())} spanning 2+ buffers "
                          f"({int(lens[multi].sum()) >> 20} MiB)")
        self.config = {"workload": f"{lens.size} Zipf(1.0) 64 B - 16 KiB packets over {seg} B PacketBuffer chains "
                                   f"({int(nseg.sum())} segments)", "packets": int(lens.size),
                       "segments": int(nseg.sum()), "total_bytes": total}

    def step(self, stream):
        self.X.batch_chained(self.buf, self.seg_off, self.seg_len, self.starts, total_bytes=self.total,
                             out=self.out, stream=stream)

    def verify(self):
        from oracle import oracle as O
        got = self.out.cpu().numpy().view(np.uint64)
        want = O.ref_xxh3_batch_varlen(self.stream, self.h_pos.astype(np.uint64), self.h_lens.astype(np.uint64)) \
            if O.xxh3_reference_available() else O.xxh3_batch_varlen(self.stream, self.h_pos, self.h_lens)
        return bool(np.array_equal(got, want))

    def cpu_sample(self):
        k = 120000
        end = int(self.h_pos[k - 1] + self.h_lens[k - 1])
        host = self.stream[:end]
        offs, lens = self.h_pos[:k].astype(np.uint64), self.h_lens[:k].astype(np.uint64)
        return CpuSample(f"first {k} packets ({int(lens.sum()) >> 20} MiB) contiguous, reference flow/xxhash.c "
                         "XXH3_64bits (the reference's chained update over the same bytes does no less work)",
                         int(lens.sum()), host,
                         ref=lambda O_: O_.ref_xxh3_batch_varlen(host, offs, lens),
                         port=lambda O_: O_.xxh3_batch_varlen(host, offs, lens, threads=1))


class PacketsVerify:
    """FlowTransport receive verification (scanPackets, fdbrpc/FlowTransport.cpp:1260-1366)
    over many connections' receive buffers at once (fdb_packets_verify, include/fdb_packets.h):
    the configs[2] Zipf packet sizes (64 B - 16 KiB payloads) framed as
    [u32 len][u64 XXH3_64bits(payload)][payload], packed back to back into
    64 KiB receive buffers (each holds whole frames).  The headers' checksums
    come from the reference's own flow/xxhash.c on the host, so verify() is a
    real check: every buffer must come back with all its frames delivered."""
    metric = ("device-resident FlowTransport receive verification GiB/s (Zipf 64 B-16 KiB packets framed in "
              "64 KiB receive buffers); % of HBM-read peak")
    kernel_name = "fdbpkt::k_pkt_walk + XXH3 planner + k_xxh3_vrows + k_pkt_check + k_pkt_final"

    def __init__(self, dev, rank, rbuf=64 << 10):
        import foundationdb_amd.packets as PK
        from oracle import oracle as O
        self.PK = PK
        lens = zipf_lengths().astype(np.int64)
        lens = np.maximum(lens, 16)  # (a frame shorter than sizeof(UID) is an error: keep every frame valid)
        frame = lens + 12
        # receive buffers: whole frames up to rbuf bytes each
        cs = np.cumsum(frame)
        bid = (np.concatenate([[0], cs[:-1]]) // rbuf).astype(np.int64)
        starts = np.concatenate([[0], cs[:-1]])
        total = int(cs[-1])
        first = np.flatnonzero(np.concatenate([[True], bid[1:] != bid[:-1]]))
        boff = starts[first]
        blen = np.diff(np.concatenate([boff, [total]]))
        host = O.splitmix64((total + 7) // 8, STATE).view(np.uint8)[:total].copy()
        poff = (starts + 12).astype(np.uint64)
        ck = O.ref_xxh3_batch_varlen(host, poff, lens.astype(np.uint64)) if O.xxh3_reference_available() else \
            O.xxh3_batch_varlen(host, poff, lens.astype(np.uint64))
        hdr = np.zeros((lens.size, 12), np.uint8)
        hdr[:, 0:4] = lens.astype("<u4").view(np.uint8).reshape(-1, 4)
        hdr[:, 4:12] = ck.astype("<u8").view(np.uint8).reshape(-1, 8)
        idx = (starts[:, None] + np.arange(12)[None, :]).reshape(-1)
        host[idx] = hdr.reshape(-1)
        self.buf = torch.from_numpy(host).to(dev)
        self.h_boff, self.h_blen, self.nframes = boff, blen, np.bincount(bid)
        self.boff = torch.from_numpy(boff.astype(np.int64)).to(dev)
        self.blen = torch.from_numpy(blen.astype(np.int64)).to(dev)
        self.V = PK.PacketVerifier(dev, boff.size, int(lens.size) + 1024, total)
        self.bytes_per_step = total
        # the receive buffers read, plus per buffer offset + length (16 B) and a 16-byte result
        self.algorithmic_bytes_per_step = total + 32 * boff.size
        self.data_desc = (f"synthetic: splitmix64 payloads (state 0x{STATE:X}), headers with the reference "
                          "flow/xxhash.c XXH3_64bits; framed Zipf packets in HBM")
        self.config = {"workload": f"{lens.size} Zipf(1.0) 64 B - 16 KiB packets framed [len][XXH3][payload] in "
                                   f"{boff.size} receive buffers of <= {rbuf >> 10} KiB",
                       "buffers": int(boff.size), "frames": int(lens.size), "total_bytes": total}
        self.host = host

    def step(self, stream):
        self.V.verify(self.buf, self.boff, self.blen, stream=stream)

    def verify(self):
        r = self.V.results_numpy()
        return bool((r["status"] == 0).all() and np.array_equal(r["frames"], self.nframes.astype(np.uint32))
                    and np.array_equal(r["consumed"], self.h_blen.astype(np.uint64)))

    def cpu_sample(self):
        k = int(np.searchsorted(np.cumsum(self.h_blen), 256 << 20)) + 1
        k = min(k, self.h_boff.size)
        end = int(self.h_boff[k - 1] + self.h_blen[k - 1])
        host = self.host[:end]
        bo, bl = self.h_boff[:k].astype(np.uint64), self.h_blen[:k].astype(np.uint64)
        return CpuSample(f"first {k} receive buffers ({end >> 20} MiB): scanPackets' checks restated in C "
                         "(oracle/packets_oracle.c) over the reference's own flow/xxhash.c XXH3_64bits", end, host,
                         ref=lambda O_: O_.packets_verify(host, bo, bl, ref=True),
                         port=lambda O_: O_.packets_verify(host, bo, bl),
                         ref_available=lambda O_: O_.packets_reference_available())


WORKLOADS = {
    "pages4k": lambda dev, rank: Pages(dev, rank, 4096, 1 << 20, 0),
    "pages8k": lambda dev, rank: Pages(dev, rank, 8192, 1 << 19, 0xFDBEEFDB),
    "zipf": lambda dev, rank: VarLen(dev, rank, zipf_lengths(), 256,
                                     "Zipf(1.0) packet sizes 64 B - 16 KiB, ~1 GiB per batch, 256 B-aligned offsets",
                                     metric="device-resident CRC32C GiB/s on Zipf 64 B-16 KiB packet batches; "
                                            "% of HBM-read peak", shape="zipf"),
    "zipf-scattered": lambda dev, rank: VarLen(dev, rank, zipf_lengths(), 256,
                                               "Zipf(1.0) packet sizes 64 B - 16 KiB, ~1 GiB per batch, 256 B-aligned, "
                                               "laid out in shuffled order (offsets not ascending: the window route)",
                                               metric="device-resident CRC32C GiB/s on scattered Zipf 64 B-16 KiB "
                                                      "packet batches; % of HBM-read peak", shape="zipf-scattered"),
    "chunks": lambda dev, rank: VarLen(dev, rank, chunk_lengths(), 4096,
                                       "log-uniform 4 KiB - 1 MiB backup chunks, ~1 GiB per batch",
                                       metric="device-resident CRC32C GiB/s on 4 KiB-1 MiB chunk batches; "
                                              "% of HBM-read peak", shape="chunks"),
    "chunks-host": lambda dev, rank: HostChunks(dev, rank),
    "pages4k-host": lambda dev, rank: HostPages(dev, rank),
    "xxh3-pages4k": lambda dev, rank: Xxh3Pages(dev, rank),
    "xxh3-zipf": lambda dev, rank: Xxh3Zipf(dev, rank),
    "xxh3-chunks": lambda dev, rank: Xxh3Chunks(dev, rank),
    "sqlite-verify": lambda dev, rank: SqliteVerify(dev, rank),
    "sqlite-verify-host": lambda dev, rank: SqliteVerifyHost(dev, rank),
    "diskqueue-verify": lambda dev, rank: DiskQueueVerify(dev, rank),
    "sqlite-seal": lambda dev, rank: SqliteSeal(dev, rank),
    "diskqueue-seal": lambda dev, rank: DiskQueueSeal(dev, rank),
    "packets-verify": lambda dev, rank: PacketsVerify(dev, rank),
    "xxh3-chained": lambda dev, rank: Xxh3Chained(dev, rank),
    "redwood-verify": lambda dev, rank: RedwoodVerify(dev, rank),
    "redwood-seal": lambda dev, rank: RedwoodSeal(dev, rank),
}
