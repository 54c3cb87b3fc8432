"""development: k_xxh3_rows over 1 Mi x 4 KiB pages, 4088 bytes at +0 (16-byte
aligned form) and at +8 (the DiskQueue V2 region: 8-byte aligned form)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X

dev = torch.device("cuda:0")
n = 1 << 20
buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
out = torch.empty(n, dtype=torch.uint64, device=dev)
for rep in range(3):
    for off in (0, 8):
        for _ in range(3):
            X.batch_fixed(buf, 4096, 4088, n, out=out, byte_offset=off)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            X.batch_fixed(buf, 4096, 4088, n, out=out, byte_offset=off)
        b.record()
        torch.cuda.synchronize()
        print(f"offset {off}: {a.elapsed_time(b) / 20 * 1e3:.1f} us")
