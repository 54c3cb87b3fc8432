"""Development: per-tile timestamps of the block-route prep kernel k_v7prep_b
and per-wave start/end of k_bigblocks (library built with -DFDBCRC_PTIMES
-DFDBCRC_BTIMES, FDBCRC_LIB=...) on a configs batch (default chunks)."""
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
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ntile = (lengths.size + 255) // 256
ncu = torch.cuda.get_device_properties(0).multi_processor_count
nw = ncu * 16
for rep in range(3):
    for _ in range(6):
        F.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    t = np.zeros((ntile, 4), dtype=np.uint64)
    lib.fdbcrc_debug_ptimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(ntile))
    b = np.zeros((nw, 4), dtype=np.uint64)
    lib.fdbcrc_debug_btimes(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(nw))
    t = t.astype(np.int64); b = b.astype(np.int64)
    t0 = t[:, 0].min()
    r = (t - t0) / 100.0
    print(f"{name}: {lengths.size} buffers, {ntile} tiles (us from the first tile's start)")
    pc = lambda a: " ".join(f"{np.percentile(a, q):6.2f}" for q in (0, 50, 100))
    for k, lab in enumerate(("start", "tables+chunks in", "prefixes", "entries")):
        print(f"  prep {lab:18s} min/med/max {pc(r[:, k])}")
    print("  last tile", " ".join(f"{x:6.2f}" for x in r[-1]))
    bs = (b[:, 0] - t0) / 100.0
    be = (b[:, 1] - t0) / 100.0
    print(f"  bigblocks wave start min/med/max {pc(bs)}   end {pc(be)}")
