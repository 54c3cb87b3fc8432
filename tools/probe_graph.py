"""Launch cost of small varlen batches (development): direct calls through the
convenience entry point vs one HIP graph replay of the caller-workspace form."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F

dev = torch.device("cuda:0")
F.gpu_init()
buf = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
for n, L in ((1000, 4096), (10000, 1500), (100, 100000)):
    lengths = np.full(n, L, dtype=np.int64)
    offs = torch.from_numpy(np.arange(n, dtype=np.int64) * ((L + 4095) // 4096 * 4096)).to(dev)
    lens = torch.from_numpy(lengths).to(dev)
    out = torch.empty(n, dtype=torch.uint32, device=dev)
    ws = torch.empty(F.varlen_workspace_bytes(n), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for _ in range(3):
            F.batch_varlen(buf, offs, lens, out=out, workspace=ws, stream=s)
            F.batch_varlen(buf, offs, lens, out=out, stream=s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        F.batch_varlen(buf, offs, lens, out=out, workspace=ws, stream=s)
    reps = 200
    for name, fn in (("direct", lambda: F.batch_varlen(buf, offs, lens, out=out, stream=s)), ("graph", g.replay)):
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                fn()
            b.record(s)
        torch.cuda.synchronize()
        print(f"{n:6d} x {L:6d} B  {name:6s}  {a.elapsed_time(b) / reps * 1e3:7.1f} us per batch")
