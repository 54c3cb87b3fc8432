"""Development: is a wave's row-phase speed in k_xxh3_vrows a property of its
slot (CU / SIMD / dispatch order) or of the buffers it gets?  Per-wave
timestamps (library built with -DFDBXXH_TIMES, FDBCRC_LIB=...) over two zipf
batches with the same lengths in different orders: a slot-driven speed
correlates between them, a data-driven one does not."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import foundationdb_amd.xxh3 as X
import bench_shapes as S

dev = torch.device("cuda:0")
F.gpu_init()
lengths, offsets, extent = S.shape("zipf")
buf = torch.empty(extent + (1 << 20), dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, S.STATE)
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
nw = torch.cuda.get_device_properties(0).multi_processor_count * 2 * 4
rng = np.random.default_rng(5)
lens2 = lengths[rng.permutation(lengths.size)]
offs2 = np.concatenate([[0], np.cumsum((lens2 + 255) // 256 * 256)[:-1]])
batches = []
for L_, O_ in ((lengths, offsets), (lens2, offs2)):
    batches.append((L_.astype(np.int64), torch.from_numpy(O_.astype(np.int64)).to(dev),
                    torch.from_numpy(L_.astype(np.int64)).to(dev)))
out = torch.empty(lengths.size, dtype=torch.uint64, device=dev)


def run(b):
    L_, o, l = batches[b]
    X.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    t = np.zeros((nw, 4), dtype=np.uint64)
    lib.fdbxxh_debug_times(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
    t = t.astype(np.int64)
    rowblk = np.where(L_ > 1024, (L_ + 1023) // 1024, 0)
    cb = np.concatenate([[0], np.cumsum(rowblk)])
    nb = t[:, 3]
    starts = np.concatenate([[0], np.cumsum(nb)[:-1]])
    blk = cb[starts + nb] - cb[starts]
    rows = (t[:, 1] - t[:, 0]) / 100.0
    end = (t[:, 2] - t[:, 0].min()) / 100.0
    return rows / np.maximum(blk, 1), end


for b in (0, 1):
    for _ in range(4):
        run(b)
A0, eA = run(0)
A1, _ = run(0)
B0, eB = run(1)
print("end max/mean: A %.1f / %.1f   B %.1f / %.1f" % (eA.max(), eA.mean(), eB.max(), eB.mean()))
print("corr speed A vs A (same data, same slots): %.3f" % np.corrcoef(A0, A1)[0, 1])
print("corr speed A vs B (other data, same slots): %.3f" % np.corrcoef(A0, B0)[0, 1])
cv = lambda a: np.std(a) / np.mean(a)
print("speed cv: A %.3f  B %.3f  slot mean of A,B %.3f" % (cv(A0), cv(B0), cv((A0 + B0) / 2)))
