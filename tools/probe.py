"""Ad-hoc kernel probes (development only)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import foundationdb_amd as F

dev = torch.device("cuda:0")
F.gpu_init()
n = 1 << 20
big = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(big, 0x5EED)
out = torch.empty(n, dtype=torch.uint32, device=dev)


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for name, stride, length, count in [("pages4k", 4096, 4096, n), ("pages4k stride0 (compute only)", 0, 4096, n),
                                    ("pages4k 256MiB (L3-resident)", 4096, 4096, 65536),
                                    ("pages8k", 8192, 8192, n // 2), ("pages8k stride0", 0, 8192, n // 2),
                                    ("pages1k", 1024, 1024, 4 * n), ]:
    o = torch.empty(count, dtype=torch.uint32, device=dev)
    ms = timeit(lambda: F.batch_fixed(big, stride, length, count, out=o))
    print(f"{name:34s} {ms:8.4f} ms  {count * length / ms / 1e6:8.1f} GB/s (equiv)")
