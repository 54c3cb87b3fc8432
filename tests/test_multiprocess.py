"""N>1 paths on CPU: world_size-2 gloo process groups exercising the sharding
helpers and bench.py's multi-rank aggregation (no GPU)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import foundationdb_amd as F
    from foundationdb_amd import parallel as P
    from oracle import oracle as O
    data = O.splitmix64(512 * 1000, 0x5EED).view(np.uint8)
    # fixed pages
    b, e = P.shard_bounds(1000, rank, world)
    local = torch.tensor([F.crc32c_append(0xAB12FD93, data[4096 * i:4096 * (i + 1)]) for i in range(b, e)],
                         dtype=torch.int64)
    counts = [P.shard_bounds(1000, r, world)[1] - P.shard_bounds(1000, r, world)[0] for r in range(world)]
    full = P.gather_checksums(local, counts).numpy().astype(np.uint32)
    ok_fixed = np.array_equal(full, O.batch_fixed(data, 4096, 4096, 1000, seed=0xAB12FD93))
    # byte-balanced varlen shards + whole-stream fold
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 9000, 300).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    b, e = P.shard_bounds_by_bytes(lens, rank, world)
    seg = data[int(offs[b]):int(offs[b] + lens[b:e].sum())] if e > b else data[:0]
    part = torch.tensor([F.crc32c_append(0, seg), int(lens[b:e].sum())], dtype=torch.int64)
    parts = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(parts, part)
    crc = P.fold_stream([int(p[0]) for p in parts], [int(p[1]) for p in parts], seed=7)
    ok_stream = crc == O.crc32c(7, data[:int(lens.sum())])
    out_q.put((rank, bool(ok_fixed), bool(ok_stream)))
    dist.destroy_process_group()


def test_gloo_world2_shards_gather_and_fold():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] and r[2] for r in res), res


def test_shard_bounds_cover():
    from foundationdb_amd import parallel as P
    for count in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [P.shard_bounds(count, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == count
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    lens = np.random.default_rng(0).integers(0, 1 << 20, 5000)
    for world in (1, 2, 8):
        spans = [P.shard_bounds_by_bytes(lens, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == lens.size
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _bench(args, env=None, timeout=300):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=dict(os.environ, OMP_NUM_THREADS="1", **(env or {})))


def test_bench_gpus2_launches_two_ranks():
    """`python bench.py --gpus 2` exactly as the driver calls it (no outer
    launcher): bench.py starts two ranks itself, every rank checks the world
    size, and rank 0's single line aggregates both (barrier, max time over
    ranks, byte sum, per-rank kernel times).  --dry-cpu: gloo + host checksums."""
    r = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-cpu"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["scaling"] == "weak" and rec["parity_ok"]
    assert [p["rank"] for p in rec["per_rank"]] == [0, 1]
    assert [p["shard"] for p in rec["per_rank"]] == [0, 1] and rec["collective"] == "gloo"
    assert sum(p["bytes_per_step"] for p in rec["per_rank"]) * 3 / rec["value"] / (1 << 30) == \
        pytest.approx(max(p["elapsed_s"] for p in rec["per_rank"]), rel=0.02)
    assert rec["value"] > 0 and rec["steps"] == 3


def test_bench_under_outer_launcher():
    """The same harness under an outer torch.distributed.run (ranks from the env)."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["parity_ok"] and len(rec["per_rank"]) == 2


def test_bench_refuses_world_size_mismatch():
    """A world size that disagrees with --gpus is an error, never a mislabelled line."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--dry-cpu"],
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "world size 1 != --gpus 2" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_force_pg_world1_and_shard_base():
    """--force-pg initialises the process group at world size 1 (the collective
    path runs with one rank) and --shard-base K moves rank 0 to shard K."""
    r = _bench(["--gpus", "1", "--steps", "2", "--warmup", "1", "--dry-cpu", "--force-pg", "--shard-base", "5"],
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(_free_port())}, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["world_size"] == 1 and rec["collective"] == "gloo" and rec["per_rank"][0]["shard"] == 5


@pytest.mark.gpu
def test_bench_rccl_path_on_one_gpu():
    """bench.py's multi-GPU path on the one-GPU box: torch.distributed.run
    --nproc-per-node 1 with --force-pg initialises RCCL (init_process_group
    "nccl", device_id) and gathers the per-rank stats with an RCCL all_gather,
    as every rank of the driver's 8-GPU run does; --shard-base 5 makes the rank
    checksum shard 5 of the global 8 KiB-page file (configs[3]) and check it
    against the reference's digest of that shard (tests/golden pages_shards)."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--workload", "pages8k", "--steps", "3", "--warmup", "1", "--force-pg",
           "--shard-base", "5", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["world_size"] == 1 and rec["collective"] == "nccl", rec
    assert rec["parity_ok"] and rec["per_rank"][0]["shard"] == 5 and rec["per_rank"][0]["parity_ok"]
    assert "shard 5" in rec["data"] and rec["value"] > 0
