"""Development: per-wave timestamps of k_xxh3_rows (library built with
-DFDBXXH_TIMES, FDBCRC_LIB=...) on 1 Mi 4 KiB pages (4088 B hashed): the
workgroup generations (blockIdx / CUs) and their end times."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X

dev = torch.device("cuda:0")
F.gpu_init()
n = 1 << 20
buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
out = torch.empty(n, dtype=torch.uint64, device=dev)
for _ in range(8):
    X.batch_fixed(buf, 4096, 4088, n, out=out)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
nw = ncu * 4 * 4
t = np.zeros((nw, 4), dtype=np.uint64)
lib.fdbxxh_debug_times(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
t = t.astype(np.int64)
ok = t[:, 0] > 0
w = np.arange(nw)[ok]
t = t[ok]
t0 = t[:, 0].min()
end = (t[:, 2] - t0) / 100
dur = (t[:, 2] - t[:, 0]) / 100
pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 100))
print("waves", ok.sum(), " end", pc(end), " dur", pc(dur))
gen = (w // 4) // ncu
for g in range(gen.max() + 1):
    m = gen == g
    print(f"  gen {g}: waves {m.sum()} dur p10/50/90 {np.percentile(dur[m], 10):.1f} {np.median(dur[m]):.1f} {np.percentile(dur[m], 90):.1f}  start median {np.median((t[m, 0] - t0) / 100):.1f}")
