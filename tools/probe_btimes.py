"""Development: per-wave timestamps of the block-route kernel k_bigblocks
(library built with -DFDBCRC_BTIMES, FDBCRC_LIB=...) on a configs batch: start,
stream start (tables in LDS), stream end, kernel end."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import bench_shapes as S

dev = torch.device("cuda:0")
F.gpu_init()
name = sys.argv[1] if len(sys.argv) > 1 else "chunks"
lengths, offsets, extent = S.shape(name)
buf = torch.empty(extent, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, S.STATE)
o = torch.from_numpy(offsets.astype(np.int64)).to(dev)
l = torch.from_numpy(lengths.astype(np.int64)).to(dev)
out = torch.empty(lengths.size, dtype=torch.uint32, device=dev)
for _ in range(8):
    F.batch_varlen(buf, o, l, out=out)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
nw = ncu * 16
t = np.zeros((nw, 4), dtype=np.uint64)
lib.fdbcrc_debug_btimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
t = t.astype(np.int64)
t0 = t[:, 0].min()
st, end = (t[:, 0] - t0) / 100, (t[:, 1] - t0) / 100
s1, fin = (t[:, 2] - t0) / 100, (t[:, 3] - t0) / 100
pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 99, 100))
print(f"{name}: percentiles 0/10/50/90/99/100 (us)")
print(" start       ", pc(st)); print(" stream start", pc(s1)); print(" stream end  ", pc(end)); print(" kernel end  ", pc(fin))
wg_end = end.reshape(ncu, 16).max(1)
wg_first = end.reshape(ncu, 16).min(1)
print(" WG end (last wave)", pc(wg_end)); print(" WG first wave done", pc(wg_first))
if hasattr(lib, "fdbcrc_debug_btimes2") and os.environ.get("FDBCRC_NP", "1") != "0":
    t2 = np.zeros((nw, 4), dtype=np.uint64)
    lib.fdbcrc_debug_btimes2(t2.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
    t2 = (t2.astype(np.int64) - t0) / 100
    for k, nm in enumerate(["metadata in", "scan barrier", "entries barrier", "first loads issued"]):
        print(f" {nm:18s}", pc(t2[:, k]))
for x in range(8):
    m = (np.arange(ncu) % 8) == x
    print(f"  xcd {x}: WG end median {np.median(wg_end[m]):.1f}")
