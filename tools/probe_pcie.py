"""PCIe ceiling probe (development): pinned host -> device copy rate of 1 GiB
in 64 MiB pieces on 1 and 4 streams, and device -> host, for the host-to-host
pipeline's roofline."""
import time
import torch

dev = torch.device("cuda:0")
n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device=dev)
piece = 64 << 20


def run(nstreams, h2d=True, reps=5):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        for k, o in enumerate(range(0, n, piece)):
            with torch.cuda.stream(streams[k % nstreams]):
                if h2d:
                    d[o:o + piece].copy_(h[o:o + piece], non_blocking=True)
                else:
                    h[o:o + piece].copy_(d[o:o + piece], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, n / (time.perf_counter() - t0) / 1e9)
    return best


for s in (1, 4):
    print(f"H2D {s} stream(s): {run(s):.1f} GB/s   D2H {s} stream(s): {run(s, False):.1f} GB/s")
