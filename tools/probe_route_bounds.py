"""development: the route-bounds batches of tests/test_gpu_parity.py, one line per batch."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
from oracle import oracle as O
dev = torch.device("cuda:0")
rng = np.random.default_rng(31)
for lens in ([5000], [5000, 9000], [4096] * 3, [4096, 4097, 70000], [123457] * 5, [4096] * 257):
    lens = np.array(lens, dtype=np.int64)
    k0 = int(rng.integers(0, 16))
    offs = np.concatenate([[k0], k0 + np.cumsum(lens)[:-1] + 16]).astype(np.int64)
    total = int(offs[-1] + lens[-1])
    h = rng.integers(0, 256, total, dtype=np.uint8)
    data = torch.from_numpy(h).to(dev)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = F.batch_varlen(data, torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev),
                         seeds=torch.from_numpy(seeds).to(dev)).cpu().numpy()
    want = O.batch_varlen(h, offs, lens, seeds=seeds)
    bad = np.flatnonzero(got != want)
    print(len(lens), lens[0], "bad", bad[:8].tolist())
