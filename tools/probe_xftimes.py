"""Development: per-workgroup phase timestamps of the fused extent kernel
k_xgf (library built with -DFDBX_TIMES, FDBCRC_LIB=...) on a configs batch:
stream end, finishing set up, own buffers done, end (us from the first start)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
import bench_shapes as S

dev = torch.device("cuda:0")
F.gpu_init()
name = sys.argv[1] if len(sys.argv) > 1 else "zipf"
lengths, offsets, extent = S.shape(name)
buf = torch.empty(extent, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, S.STATE)
o = torch.from_numpy(offsets.astype(np.int64)).to(dev)
l = torch.from_numpy(lengths.astype(np.int64)).to(dev)
out = torch.empty(lengths.size, dtype=torch.uint32, device=dev)
lib = ctypes.CDLL(os.environ["FDBCRC_LIB"])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
for rep in range(3):
    for _ in range(8):
        F.batch_varlen(buf, o, l, out=out)
    torch.cuda.synchronize()
    t = np.zeros((ncu, 8), dtype=np.uint64)
    lib.fdbx_debug_ftimes(t.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(ncu))
    t = t.astype(np.int64)
    t0 = t[:, 0].min()
    pc = lambda a: " ".join(f"{np.percentile(a, q):6.1f}" for q in (0, 10, 50, 90, 100))
    print(f"{name} rep {rep}: percentiles 0/10/50/90/100 (us)")
    for k, nm in enumerate(["start", "stream", "setup", "own", "end"]):
        print(f"  {nm:7s}", pc((t[:, k] - t0) / 100))
    print("  setup-stream", pc((t[:, 2] - t[:, 1]) / 100), " own-setup", pc((t[:, 3] - t[:, 2]) / 100),
          " end-own", pc((t[:, 4] - t[:, 3]) / 100))
