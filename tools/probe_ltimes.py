"""Development: per-wave timestamps of k_xlong (library built with
-DFDBXXH_TIMES, FDBCRC_LIB=...) on the chunks batch: producers' steps and first
idle, chain waves' buffers, ring waits and ends, per CU and per XCD."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X
import bench_workloads as W

dev = torch.device("cuda:0")
F.gpu_init()
lengths = np.asarray(W.chunk_lengths(), dtype=np.int64)
padded = (lengths + 4095) // 4096 * 4096
offs = np.concatenate([[0], np.cumsum(padded)[:-1]])
buf = torch.empty(int(padded.sum()), dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
o = torch.from_numpy(offs).to(dev); l = torch.from_numpy(lengths).to(dev)
out = torch.empty(lengths.size, dtype=torch.uint64, device=dev)
for _ in range(8):
    X.batch_varlen(buf, o, l, out=out)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
LW = int(os.environ.get("LWAVES", 16)); LC = int(os.environ.get("LCHAINS", 4))
nw = ncu * LW
t = np.zeros((nw, 4), dtype=np.uint64)
lib.fdbxxh_debug_ltimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
t = t.astype(np.int64)
t0 = t[:, 0].min()
st = (t[:, 0] - t0) / 100; idle = np.where(t[:, 1] > 0, (t[:, 1] - t0) / 100, np.nan); end = (t[:, 2] - t0) / 100
cnt = t[:, 3] & 0xFFFFF; spin = t[:, 3] >> 20
wv = np.arange(nw) % LW; cu = np.arange(nw) // LW
prod = wv < LW - LC
pc = lambda a: " ".join(f"{np.nanpercentile(a, q):6.1f}" for q in (0, 10, 50, 90, 100))
print("long bytes", int(lengths[lengths > 16384].sum()) / 2**20, "MiB of", int(lengths.sum()) / 2**20)
print("start      ", pc(st))
print("prod idle  ", pc(idle[prod]), "(first time both steps empty)")
print("prod end   ", pc(end[prod]))
print("prod steps ", pc(cnt[prod].astype(float)))
print("chain lastq", pc(idle[~prod]), "(last dequeue)")
print("chain end  ", pc(end[~prod]))
print("chain bufs ", pc(cnt[~prod].astype(float)), " spins", pc(spin[~prod].astype(float)))
cend = end.reshape(ncu, LW).max(1)
print("CU end     ", pc(cend))
for x in range(8):
    m = (np.arange(ncu) % 8) == x
    print(f"  xcd {x}: CU end p50 {np.median(cend[m]):.1f} max {cend[m].max():.1f}  steps/CU {cnt.reshape(ncu, LW)[m][:, :LW - LC].sum(1).mean():.0f}")
