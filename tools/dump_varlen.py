"""Development: run the golden threshold batch through the varlen engine and
dump the device results (gpurun_out/dump_thresholds.npy) for CPU-side diagnosis."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
from oracle import oracle as O
g = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "crc32c_golden.json")))
t = g["threshold"]
h = O.splitmix64((t["nbytes"] + 7) // 8, t["state"]).view(np.uint8)[:t["nbytes"]].copy()
d = torch.from_numpy(h).to("cuda:0")
c = t["cases"]
o = torch.tensor([x[0] for x in c], dtype=torch.int64, device="cuda:0")
l = torch.tensor([x[1] for x in c], dtype=torch.int64, device="cuda:0")
s = torch.tensor([x[2] for x in c], dtype=torch.int64).to(torch.uint32).to("cuda:0")
res = []
for k in range(3):
    res.append(F.batch_varlen(d, o, l, seeds=s).cpu().numpy())
res.append(F.batch_varlen(d, o, l, seed=0).cpu().numpy())
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/dump_thresholds.npy", np.stack(res))
want = np.array([x[3] for x in c], np.uint32)
print("mismatches per run:", [int((r != want).sum()) for r in res[:3]])
