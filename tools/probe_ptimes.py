"""Development: per-wave timestamps of k_pages4k (library built with
-DFDBCRC_BTIMES, FDBCRC_LIB=...) on 1 Mi 4 KiB device pages."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F

dev = torch.device("cuda:0")
F.gpu_init()
n = 1 << 20
buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
out = torch.empty(n, dtype=torch.uint32, device=dev)
for _ in range(30):
    F.batch_fixed(buf, 4096, 4096, n, out=out)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
nw = ncu * 16
t = np.zeros((nw, 4), dtype=np.uint64)
lib.fdbcrc_debug_btimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
t = t.astype(np.int64)
t0 = t[:, 0].min()
end = (t[:, 1] - t0) / 100
pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 99, 100))
print("end", pc(end))
wg_end = end.reshape(ncu, 16).max(1)
print("WG end", pc(wg_end))
print("WG first wave done", pc(end.reshape(ncu, 16).min(1)))
for x in range(8):
    m = (np.arange(ncu) % 8) == x
    print(f"  xcd {x}: WG end median {np.median(wg_end[m]):.1f}")
