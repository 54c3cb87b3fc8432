"""Ad-hoc GPU check used during development (tests/ holds the real suite)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as f
from oracle import oracle as o

dev = torch.device("cuda:0")
f.gpu_init()
# 1. generator parity
buf = torch.empty(65536 * 4096, dtype=torch.uint8, device=dev)
f.fill_splitmix64(buf, 0x5EED)
torch.cuda.synchronize()
h = buf.cpu().numpy()
ref_words = o.splitmix64(512 * 65536, 0x5EED)
print("gen match", np.array_equal(h.view(np.uint64), ref_words))
# 2. pages
for seed in (0, 0xfdbeefdb):
    out = f.batch_fixed(buf, 4096, 4096, 65536, seed=seed)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    exp = o.batch_fixed(h, 4096, 4096, 65536, seed=seed)
    print("pages seed %08x: mismatches %d xor %08x sum %x" % (seed, int((got != exp).sum()), np.bitwise_xor.reduce(got), int(got.astype(np.uint64).sum())))
    if (got != exp).any():
        idx = np.nonzero(got != exp)[0][:5]
        print("  first bad", idx, [hex(x) for x in got[idx]], [hex(x) for x in exp[idx]])
# 3. general kernel via unaligned fixed
for (off, stride, length, count) in [(0, 4096, 4088, 1000), (3, 4100, 4092, 1000), (1, 100, 77, 5000), (0, 8192, 8192, 2000), (5, 1 << 20, 1 << 20, 20), (0, 16, 0, 10), (7, 33, 33, 3000)]:
    out = f.batch_fixed(buf, stride, length, count, seed=0x1234, byte_offset=off)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    exp = o.batch_fixed(h[off:], stride, length, count, seed=0x1234)
    print("fixed off=%d stride=%d len=%d: mismatches %d / %d" % (off, stride, length, int((got != exp).sum()), count))
# 4. varlen random
rng = np.random.default_rng(5)
n = 20000
lengths = rng.integers(0, 20000, n).astype(np.uint64)
offsets = rng.integers(0, h.size - 20000, n).astype(np.uint64)
seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
out = f.batch_varlen(buf, torch.from_numpy(offsets.astype(np.int64)).to(dev), torch.from_numpy(lengths.astype(np.int64)).to(dev), seeds=torch.from_numpy(seeds).to(dev))
torch.cuda.synchronize()
got = out.cpu().numpy()
exp = o.batch_varlen(h, offsets, lengths, seeds=seeds)
print("varlen mismatches", int((got != exp).sum()), "/", n)
# 5. timing, 1 Mi x 4 KiB
del buf
big = torch.empty(1 << 32, dtype=torch.uint8, device=dev)
f.fill_splitmix64(big, 0x5EED)
out = torch.empty(1 << 20, dtype=torch.uint32, device=dev)
for _ in range(3):
    f.batch_fixed(big, 4096, 4096, 1 << 20, out=out)
torch.cuda.synchronize()
reps = 20
a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    f.batch_fixed(big, 4096, 4096, 1 << 20, out=out)
b.record(); torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
print("1Mi x 4KiB: %.3f ms  %.1f GB/s  %.1f GiB/s" % (ms, (1 << 32) / ms / 1e6, (1 << 32) / ms / 1e3 / 2**30 * 1e3 / 1e3))
got = out.cpu().numpy()
print("xor %08x sum %x" % (np.bitwise_xor.reduce(got), int(got.astype(np.uint64).sum())))
