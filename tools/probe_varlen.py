"""Varlen engine probes (development): per-config timing."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import bench_workloads as W

dev = torch.device("cuda:0")
F.gpu_init()
buf = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)


ONLY = sys.argv[1:]


def run(name, lengths, align=256, reps=int(os.environ.get("REPS", 10))):
    if ONLY and not any(o in name for o in ONLY):
        return
    lengths = np.asarray(lengths, dtype=np.int64)
    padded = (lengths + align - 1) // align * align
    offs = np.concatenate([[0], np.cumsum(padded)[:-1]])
    o = torch.from_numpy(offs).to(dev); l = torch.from_numpy(lengths).to(dev)
    out = torch.empty(lengths.size, dtype=torch.uint32, device=dev)
    for _ in range(3):
        F.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        F.batch_varlen(buf, o, l, out=out)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name:32s} n={lengths.size:8d} bytes={int(lengths.sum()) / 2**20:8.1f} MiB  {ms:7.3f} ms  "
          f"{lengths.sum() / ms / 1e6:8.1f} GB/s  {lengths.size / ms / 1e3:8.1f} Mbuf/s")


run("1 MiB x 1024", [1 << 20] * 1024, 4096)
run("4096 x 256K aligned", [4096] * (1 << 18), 4096)
run("16384 x 64K", [16384] * (1 << 16), 4096)
run("1024 x 1M", [1024] * (1 << 20), 1024)
run("256 x 1M", [256] * (1 << 20), 256)
run("64 x 1M", [64] * (1 << 20), 64)
run("4000 x 256K (ragged)", [4000] * (1 << 18), 4096)
run("zipf", W.zipf_lengths(), 256)
run("zipf a64", W.zipf_lengths(), 64)
run("zipf a16", W.zipf_lengths(), 16)
run("small: 4096 x 1000", [4096] * 1000, 4096, reps=200)
run("small: 1500 x 10000", [1500] * 10000, 2048, reps=200)
run("small: 600 x 2000", [600] * 2000, 1024, reps=200)
run("chunks", W.chunk_lengths(), 4096)
run("16 KiB x 8K", [16384] * 8192, 4096)
run("2 KiB x 16K", [2048] * 16384, 2048, reps=50)
run("one route buffer 100000", [100000], 4096, reps=200)
run("route 64 KiB x 16K", [65536] * (1 << 14), 4096)
