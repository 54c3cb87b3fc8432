"""XXH3 varlen probes (development): timing on the zipf / chunks / fixed-size batches."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X
import bench_workloads as W

dev = torch.device("cuda:0")
F.gpu_init()
buf = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
ONLY = sys.argv[1:]


def run(name, lengths, align=256, reps=10):
    if ONLY and not any(o in name for o in ONLY):
        return
    lengths = np.asarray(lengths, dtype=np.int64)
    padded = (lengths + align - 1) // align * align
    offs = np.concatenate([[0], np.cumsum(padded)[:-1]])
    o = torch.from_numpy(offs).to(dev); l = torch.from_numpy(lengths).to(dev)
    out = torch.empty(lengths.size, dtype=torch.uint64, device=dev)
    for _ in range(3):
        X.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        X.batch_varlen(buf, o, l, out=out)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"xxh3 {name:28s} n={lengths.size:8d} bytes={int(lengths.sum()) / 2**20:8.1f} MiB  {ms:7.3f} ms  "
          f"{lengths.sum() / ms / 1e6:8.1f} GB/s  {lengths.size / ms / 1e3:8.1f} Mbuf/s")


run("4096 x 256K aligned", [4096] * (1 << 18), 4096)
run("1024 x 1M", [1024] * (1 << 20), 1024)
run("256 x 1M", [256] * (1 << 20), 256)
run("64 x 1M", [64] * (1 << 20), 64)
run("16384 x 64K", [16384] * (1 << 16), 256)
run("8192 x 128K", [8192] * (1 << 17), 256)
run("5000 x 200K", [5000] * 200000, 256)
_r = np.random.default_rng(4)
run("rand 4-16K", _r.integers(4097, 16385, 90000), 256)
run("alt 5000/15000", [5000, 15000] * 50000, 256)
_z = W.zipf_lengths()
run("zipf mid (>4K)", _z[_z > 4096], 256)
run("zipf low (<=4K)", _z[_z <= 4096], 256)
run("zipf short (<=240)", _z[_z <= 240], 256)
run("zipf one (241-1K)", _z[(_z > 240) & (_z <= 1024)], 256)
run("zipf few (1K-4K)", _z[(_z > 1024) & (_z <= 4096)], 256)
run("zipf", W.zipf_lengths(), 256)
run("chunks", W.chunk_lengths(), 4096)
run("zipf unaligned", W.zipf_lengths(), 1)
run("1500 x 512K unaligned", [1500] * (1 << 19), 1)
