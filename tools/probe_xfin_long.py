"""development: a packed batch with buffers of hundreds of MiB on the extent
route (300 small packets first, as tests/test_gpu_parity.py's
test_extent_route_grows_to_the_extent): time per call, by HIP events."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F

dev = torch.device("cuda:0")
buf = torch.empty(600 << 20, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x6209)
small = np.full(300, 1000, dtype=np.int64)
soffs = np.arange(300, dtype=np.int64) * 1024 + 5
base = int(soffs[-1]) + 1000 + 24
lens = np.concatenate([small, np.array([200 << 20, 3, (150 << 20) + 5, 1 << 20], dtype=np.int64)])
offs = np.concatenate([soffs, base + np.array([0, (200 << 20) + 100, (200 << 20) + 200, (350 << 20) + 1205])])
o, l = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
out = torch.empty(lens.size, dtype=torch.uint32, device=dev)
ts = []
for i in range(12):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    F.batch_varlen(buf, o, l, seed=4, out=out)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(os.environ.get("FDBCRC_LIB", "product").split("/")[-1], "ms per call:", " ".join(f"{t:.3f}" for t in ts[2:]))
