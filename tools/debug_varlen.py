"""Replays test_random_varlen_vs_oracle's inputs against the bounds-checked debug build."""
import os, sys
os.environ["FDBCRC_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "foundationdb_amd", "lib", "libfdb_crc32c_debug.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes
import numpy as np
import torch
import foundationdb_amd as F
from oracle import oracle as O

L = F.lib()
L.crc32c_debug_bounds.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
L.crc32c_debug_read.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
F.gpu_init()
rng = np.random.default_rng(2024)
h = O.splitmix64((64 << 20) // 8, 0x1234).view(np.uint8).copy()
data = torch.from_numpy(h).to(dev)
n = 30000
lengths = np.where(rng.random(n) < 0.8, rng.integers(0, 20000, n), rng.integers(0, 2 << 20, n))
offsets = rng.integers(0, h.size - lengths)
seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
dbg = torch.zeros(8, dtype=torch.int64, device=dev)
L.crc32c_debug_bounds(data.data_ptr(), data.data_ptr() + h.size)
out = F.batch_varlen(data, torch.from_numpy(offsets.astype(np.int64)).to(dev),
                     torch.from_numpy(lengths.astype(np.int64)).to(dev), seeds=torch.from_numpy(seeds).to(dev))
torch.cuda.synchronize()
L.crc32c_debug_read(dbg.data_ptr())
d = [int(x) & 0xFFFFFFFFFFFFFFFF for x in dbg.cpu().numpy()]
print("bounds", hex(d[0]), hex(d[1]), "violations", d[2], "first bad", hex(d[3]), "site", d[4])
got = out.cpu().numpy()
want = O.batch_varlen(h, offsets, lengths, seeds=seeds)
bad = np.nonzero(got != want)[0]
print("mismatches", bad.size, "of", n, bad[:10], lengths[bad[:10]], offsets[bad[:10]])
if d[2]:
    ofs = d[3] - d[0]
    print("bad address offset from data base:", ofs, "(negative => before)" )
