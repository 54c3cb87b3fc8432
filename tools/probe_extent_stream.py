"""development: k_xgrab's streaming rate without points -- one buffer of
`MiB` MiB on the extent route (FDBCRC_ROUTE=3), and the zipf batch, by HIP events."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import bench_workloads as W

dev = torch.device("cuda:0")
buf = torch.empty(1200 << 20, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)


def run(name, lens, offs, reps=20):
    o = torch.from_numpy(np.asarray(offs, np.int64)).to(dev)
    l = torch.from_numpy(np.asarray(lens, np.int64)).to(dev)
    out = torch.empty(len(lens), dtype=torch.uint32, device=dev)
    for _ in range(3):
        F.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        F.batch_varlen(buf, o, l, out=out)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    nb = int(np.sum(lens))
    print(f"{name:24s} {ms:.4f} ms  {nb / ms / 1e6:.1f} GB/s")


run("one buffer 1132 MB", [1131653632], [0])
run("two buffers", [565826816, 565826816], [0, 565826816])
L = W.zipf_lengths().astype(np.int64)
pad = (L + 255) // 256 * 256
run("zipf", L, np.concatenate([[0], np.cumsum(pad)[:-1]]))
