"""Development: which buffers of the route test's mixed batch differ from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import foundationdb_amd as F
from oracle import oracle as O
dev = torch.device("cuda:0"); F.gpu_init()
rng = np.random.default_rng(77)
h = O.splitmix64((96 << 20) // 8, 0x70E).view(np.uint8)
d = torch.from_numpy(h.copy()).to(dev)
for name, lengths in [("mixed", np.where(rng.random(3000) < 0.5, rng.integers(0, 2000, 3000), rng.integers(16384, 300000, 3000))),
                      ("big", rng.integers(16384, 300000, 3000))]:
    offsets = rng.integers(0, h.size - lengths)
    seeds = rng.integers(0, 2**32, lengths.size, dtype=np.uint64).astype(np.uint32)
    want = O.batch_varlen(h, offsets, lengths, seeds=seeds)
    for it in range(3):
        got = F.batch_varlen(d, torch.from_numpy(offsets.astype(np.int64)).to(dev), torch.from_numpy(lengths.astype(np.int64)).to(dev),
                             seeds=torch.from_numpy(seeds.astype(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        print(name, it, "bad", bad.size, "first", bad[:10], "lens", lengths[bad[:10]])
