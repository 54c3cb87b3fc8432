import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import foundationdb_amd as F
from oracle import oracle as O
g = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/crc32c_golden.json")))
t = g["threshold"]
h = O.splitmix64((t["nbytes"] + 7) // 8, t["state"]).view(np.uint8)[:t["nbytes"]].copy()
dev = torch.device("cuda:0")
data = torch.from_numpy(h).to(dev)
cases = t["cases"]
offs = torch.tensor([c[0] for c in cases], dtype=torch.int64, device=dev)
lens = torch.tensor([c[1] for c in cases], dtype=torch.int64, device=dev)
sds = torch.tensor(np.array([c[2] for c in cases], dtype=np.uint32), device=dev)
got = F.batch_varlen(data, offs, lens, seeds=sds).cpu().numpy()
want = np.array([c[3] for c in cases], dtype=np.uint32)
bad = np.nonzero(got != want)[0]
print("bad", bad.size, "of", len(cases))
for i in bad[:30]:
    print(cases[i][:3])
# same cases one at a time (no splitting across waves)
bad1 = []
for i in bad[:10]:
    o, l, s, w = cases[i]
    r = F.batch_varlen(data, torch.tensor([o], dtype=torch.int64, device=dev), torch.tensor([l], dtype=torch.int64, device=dev), seed=s).cpu().numpy()[0]
    bad1.append((o, l, int(r) == w))
print("single:", bad1)
