"""Workload driver for rocprofv3 --pmc passes (development)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import foundationdb_amd as F

mode = sys.argv[1] if len(sys.argv) > 1 else "pages4k"
dev = torch.device("cuda:0")
F.gpu_init()
n = 1 << 20
big = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(big, 0x5EED)
out = torch.empty(n, dtype=torch.uint32, device=dev)
out64 = torch.empty(n, dtype=torch.uint64, device=dev)
VARLEN = ("chunks", "zipf", "v4096", "v1024", "xchunks", "xzipf", "scattered")
if mode == "scattered":  # the zipf-scattered bench line: the same packets, shuffled non-ascending offsets
    import numpy as np
    import bench_shapes as S
    lens, offs_np, extent = S.shape("zipf-scattered")
    assert extent <= big.numel()
    offs = torch.from_numpy(offs_np.astype(np.int64)).to(dev)
    lt = torch.from_numpy(lens.astype(np.int64)).to(dev)
    vout = torch.empty(lens.size, dtype=torch.uint32, device=dev)
elif mode in VARLEN:
    import numpy as np
    import bench_workloads as W
    lens = {"chunks": W.chunk_lengths, "zipf": W.zipf_lengths, "xchunks": W.chunk_lengths, "xzipf": W.zipf_lengths, "v4096": lambda: np.full(1 << 18, 4096),
            "v1024": lambda: np.full(1 << 20, 1024)}[mode]().astype(np.int64)
    al = {"chunks": 4096, "zipf": 256, "v4096": 4096, "v1024": 1024, "xchunks": 4096, "xzipf": 256}[mode]
    padded = (lens + al - 1) // al * al
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(padded)[:-1]])).to(dev)
    lt = torch.from_numpy(lens).to(dev)
    vout = torch.empty(lens.size, dtype=torch.uint32, device=dev)
    vout64 = torch.empty(lens.size, dtype=torch.uint64, device=dev)
    import foundationdb_amd.xxh3 as X
torch.cuda.synchronize()
for it in range(5):
    if it == 1:  # (steady state: the library's room sized from the first batch's need)
        torch.cuda.synchronize()
    if mode in ("xchunks", "xzipf"):
        X.batch_varlen(big, offs, lt, out=vout64)
    elif mode in VARLEN:
        F.batch_varlen(big, offs, lt, out=vout)
    elif mode == "xxh3":
        import foundationdb_amd.xxh3 as X
        X.batch_fixed(big, 4096, 4088, n, out=out64)
    elif mode == "pages4k":
        F.batch_fixed(big, 4096, 4096, n, out=out)
    elif mode == "pages8k":
        F.batch_fixed(big, 8192, 8192, n // 2, seed=0xFDBEEFDB, out=out)
    elif mode == "stride0":
        F.batch_fixed(big, 0, 4096, n, out=out)
torch.cuda.synchronize()
print("done", mode)
