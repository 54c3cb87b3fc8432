"""Development: per-wave timestamps of k_xxh3_vrows (library built with
-DFDBXXH_TIMES, FDBCRC_LIB=...): start skew, row phase, short/quad tail, end."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X
import bench_workloads as W
import bench_shapes as S

dev = torch.device("cuda:0")
F.gpu_init()
name = sys.argv[1] if len(sys.argv) > 1 else "zipf"
lengths, offsets, extent = S.shape(name)
buf = torch.empty(extent, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, S.STATE)
o = torch.from_numpy(offsets.astype(np.int64)).to(dev)
l = torch.from_numpy(lengths.astype(np.int64)).to(dev)
out = torch.empty(lengths.size, dtype=torch.uint64, device=dev)
for _ in range(5):
    X.batch_varlen(buf, o, l, out=out)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
nw = torch.cuda.get_device_properties(0).multi_processor_count * 2 * 4
t = np.zeros((nw, 4), dtype=np.uint64)
rc = lib.fdbxxh_debug_times(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
t = t.astype(np.int64)
ok = t[:, 0] > 0
t = t[ok]
t0 = t[:, 0].min()
st, rows, tail, end = (t[:, 0] - t0) / 100, (t[:, 1] - t[:, 0]) / 100, (t[:, 2] - t[:, 1]) / 100, (t[:, 2] - t0) / 100
pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 99, 100))
print(f"{name}: waves {ok.sum()} (rc {rc}); percentiles 0/10/50/90/99/100, us")
print(" start ", pc(st)); print(" rows  ", pc(rows)); print(" tail  ", pc(tail)); print(" end   ", pc(end))
late = np.argsort(end)[-8:]
for i in late:
    print(f"  late wave: start {st[i]:.1f} rows {rows[i]:.1f} tail {tail[i]:.1f} end {end[i]:.1f} nbuf {t[i, 3]}")

# per-wave work from the (contiguous, ascending) ranges
nb = t[:, 3]
starts = np.concatenate([[0], np.cumsum(nb)[:-1]])
L = lengths.astype(np.int64)
rowblk = np.where(L > 1024, (L + 1023) // 1024, 0)
cb = np.concatenate([[0], np.cumsum(rowblk)])
cbytes = np.concatenate([[0], np.cumsum(L)])
blk = cb[starts + nb] - cb[starts]
byt = cbytes[starts + nb] - cbytes[starts]
print(" row blocks/wave ", pc(blk.astype(float)))
print(" bytes/wave KiB  ", pc(byt / 1024.0))
print(" corr(rows, blocks) %.3f  corr(rows, bytes) %.3f" % (np.corrcoef(rows, blk)[0, 1], np.corrcoef(rows, byt)[0, 1]))
print(" us per row block: median %.3f" % np.median(rows / np.maximum(blk, 1)))
w = np.arange(t.shape[0])
wg = w // 4
for x in range(8):
    m = (wg % 8) == x
    print(f"  xcd {x}: rows median {np.median(rows[m]):.1f}  blocks median {np.median(blk[m]):.0f}")
ncu = nw // 8
for lab, m in (("wg < ncu", wg < ncu), ("wg >= ncu", wg >= ncu)):
    print(f"  {lab}: rows p10/50/90 {np.percentile(rows[m], 10):.1f} {np.median(rows[m]):.1f} {np.percentile(rows[m], 90):.1f}")
for k in range(4):
    m = (w % 4) == k
    print(f"  wave {k} of WG: rows median {np.median(rows[m]):.1f}")
# per CU (2 WGs per CU assumed: wg and wg + ncu share a CU?) -- print rows of pairs
pa = rows[(wg < ncu)].reshape(-1, 4).mean(1)
pb = rows[(wg >= ncu)].reshape(-1, 4).mean(1)
print("  corr(WG w, WG w+ncu) %.3f" % np.corrcoef(pa, pb)[0, 1])
