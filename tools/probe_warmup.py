"""Headline warm-up probe (development): in a FRESH process, the page kernel's
duration launch by launch (HIP events around every launch of 1 Mi x 4 KiB
pages), from the first launch after the data is generated, to find what makes
`bench.py --warmup 5` slower than a long warm-up (clock ramp, first-touch /
TLB, the stream's one-time allocations).  Prints one JSON line.

    python tools/probe_warmup.py [launches] [idle_ms]
idle_ms: sleep between generating the data and the first launch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import foundationdb_amd as F  # noqa: E402

n_launch = int(sys.argv[1]) if len(sys.argv) > 1 else 60
idle_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
dev = torch.device("cuda:0")
t0 = time.perf_counter()
F.gpu_init()
t_init = time.perf_counter() - t0
n = 1 << 20
buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
F.fill_splitmix64(buf, 0x5EED)
out = torch.empty(n, dtype=torch.uint32, device=dev)
torch.cuda.synchronize()
if idle_ms:
    time.sleep(idle_ms / 1e3)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_launch + 1)]
s = torch.cuda.current_stream()
t1 = time.perf_counter()
ev[0].record(s)
for i in range(n_launch):
    F.batch_fixed(buf, 4096, 4096, n, out=out, stream=s)
    ev[i + 1].record(s)
torch.cuda.synchronize()
host_ms = (time.perf_counter() - t1) * 1e3
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(n_launch)]
print(json.dumps({"init_s": round(t_init, 3), "idle_ms": idle_ms, "host_ms_total": round(host_ms, 3),
                  "launch_ms": [round(x, 4) for x in ms],
                  "first5_avg": round(sum(ms[:5]) / 5, 4), "next20_avg": round(sum(ms[5:25]) / 20, 4),
                  "last20_avg": round(sum(ms[-20:]) / 20, 4)}))
