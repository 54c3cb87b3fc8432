"""Replays test_random_varlen_vs_oracle's inputs on the RELEASE build (after the earlier parity tests' calls)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import foundationdb_amd as F
from oracle import oracle as O
dev = torch.device("cuda:0")
F.gpu_init()
rng = np.random.default_rng(2024)
h = O.splitmix64((64 << 20) // 8, 0x1234).view(np.uint8).copy()
data = torch.from_numpy(h).to(dev)
n = 30000
lengths = np.where(rng.random(n) < 0.8, rng.integers(0, 20000, n), rng.integers(0, 2 << 20, n))
offsets = rng.integers(0, h.size - lengths)
seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
out = F.batch_varlen(data, torch.from_numpy(offsets.astype(np.int64)).to(dev),
                     torch.from_numpy(lengths.astype(np.int64)).to(dev), seeds=torch.from_numpy(seeds).to(dev))
torch.cuda.synchronize()
got = out.cpu().numpy()
want = O.batch_varlen(h, offsets, lengths, seeds=seeds)
print("release replay mismatches", int((got != want).sum()))
