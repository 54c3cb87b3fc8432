"""Development: per-wave start/end timestamps of k_pages4k (library built
with -DFDBCRC_BTIMES, FDBCRC_LIB=...) on the headline batch (1 Mi x 4 KiB)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F

dev = torch.device("cuda:0")
F.gpu_init()
count = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
buf = torch.empty(count * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 12345)
out = torch.empty(count, dtype=torch.uint32, device=dev)
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
nw = ncu * 16
pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 99, 100))
for rep in range(3):
    for _ in range(10):
        F.batch_fixed(buf, 4096, 4096, count, seed=0, out=out)
    torch.cuda.synchronize()
    t = np.zeros((nw, 4), dtype=np.uint64)
    lib.fdbcrc_debug_btimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
    t = t.astype(np.int64)
    t0 = t[:, 0].min()
    end = (t[:, 1] - t0) / 100
    wg_end = end.reshape(ncu, 16).max(1)
    wg_first = end.reshape(ncu, 16).min(1)
    print(f"pages {count}: wave end {pc(end)} | mean {end.mean():.1f}")
    print(f"   WG last-wave end {pc(wg_end)} | WG first-wave end {pc(wg_first)}")
