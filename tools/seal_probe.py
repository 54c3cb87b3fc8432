"""development: does writing the 8-byte trailers slow the next XXH3 pass over the pages?
Times k_xxh3_rows alone, after a torch trailer write, and the whole seal."""
import sys
import torch
sys.path.insert(0, ".")
import foundationdb_amd.crc32c as F
import foundationdb_amd.xxh3 as X
import foundationdb_amd.pagecheck as PC

count = 1 << 20
dev = torch.device("cuda:0")
buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
pages = buf.view(count, 4096)
out = torch.empty(count, dtype=torch.uint64, device=dev)
tr = torch.zeros(count, 8, dtype=torch.uint8, device=dev)


def timed(fn, pre=None, n=20):
    ts = []
    for i in range(n + 3):
        if pre:
            pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return f"{ts[len(ts) // 2]:.1f}"


xx = lambda: X.batch_fixed(buf, 4096, 4088, count, out=out)
print("xxh3 alone", timed(xx))
src = pages[:, 4032:4096].clone()
print("after zero_ 64 B", timed(xx, pre=lambda: pages[:, 4032:4096].zero_()))
print("after add_(0) 64 B", timed(xx, pre=lambda: pages[:, 4032:4096].add_(0)))
print("after copy_ 64 B", timed(xx, pre=lambda: pages[:, 4032:4096].copy_(src)))
print("after add_(0) 8 B", timed(xx, pre=lambda: pages[:, 4088:4096].add_(0)))
print("after zero_ 128 B", timed(xx, pre=lambda: pages[:, 3968:4096].zero_()))
print("after add_(0) 128 B", timed(xx, pre=lambda: pages[:, 3968:4096].add_(0)))
print("after zero_ 64 B at +0", timed(xx, pre=lambda: pages[:, 0:64].zero_()))
print("seal", timed(lambda: PC.sqlite_seal_pages(buf, 4096, count, first_pgno=0)))
print("xxh3 alone again", timed(xx))
