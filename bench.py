#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC-32C on MI355X.

Default workload = BASELINE.json configs[1]: 1 Mi x 4 KiB pages resident in
HBM, one checksum per page, bit-exact with contrib/crc32.  A "step" is one
pass of the engine over the whole batch (one kernel launch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload pages4k|pages8k|zipf|chunks]

N > 1: one rank per GPU.  Started as `python bench.py --gpus N` (no
WORLD_SIZE in the environment) it launches `torch.distributed.run
--nproc-per-node N` on itself as a child process, before anything touches the
GPU, and exits with the child's status; under an outer launcher it uses the
launcher's ranks.  Every rank checks that the world size equals --gpus.
Pages shard trivially (the whole-file scan of
fdbserver/kvstore/KeyValueStoreSQLite.cpp:1378-1470 split by page range):
rank r checksums shard r of one global splitmix64 file -- bytes
[r*4 GiB, (r+1)*4 GiB), generated in its own HBM by jumping the generator --
and checks it against the reference's digest of that shard
(tests/golden, make_golden.py --shards): weak scaling, no data-path
collective.  RCCL (all_gather over xGMI) is used only to take the max elapsed
time over ranks and to gather the per-rank byte counts, parity flags and
kernel times.  --force-pg initialises the process group at world size 1 too,
so one GPU exercises the whole multi-GPU path; --shard-base K makes rank r
checksum shard K + r.

Rank 0 prints ONE JSON line.  `value` is GiB/s of buffer bytes read, whole
job, from the host clock around the K timed steps.  `roofline.achieved` is the
dominant kernel's algorithmic bytes per launch (buffer bytes + 4 B checksum
per buffer [+ per-buffer metadata]) / its average launch duration measured
with HIP events on the launch stream.  `cpu_baseline` times the reference's
own crc32c.cpp (oracle/_ref) single-threaded on a bounded sample of the same
workload on this host.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import foundationdb_amd as F  # noqa: E402
import bench_workloads as W  # noqa: E402

METRIC = "device-resident CRC32C GiB/s on 4 KiB page batches; % of HBM-read peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5, help="untimed steps (the driver's setting)")
    p.add_argument("--workload", default="pages4k", choices=sorted(W.WORKLOADS))
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 disables)")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--dry-cpu", action="store_true",
                   help="test the multi-rank harness on CPU (gloo, host checksums); not a measurement")
    p.add_argument("--force-pg", action="store_true",
                   help="initialise the RCCL process group even at world size 1 (exercises the multi-GPU path)")
    p.add_argument("--shard-base", type=int, default=0,
                   help="rank r checksums shard shard_base + r of the global batch (page workloads)")
    return p.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(wl, seconds):
    """Reference crc32c_append (oracle/_ref), 1 thread pinned to one core."""
    from oracle import oracle as O
    sample = wl.cpu_sample()
    kind = "reference" if sample.available(O) else "port"
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        def once():
            t = time.perf_counter()
            if kind == "reference":
                sample.run_reference(O)
            else:
                sample.run_port(O)
            return time.perf_counter() - t
        once()  # warm
        best, total, reps = 1e30, 0.0, 0
        while total < seconds or reps < 3:
            dt = once()
            best = min(best, dt)
            total += dt
            reps += 1
    finally:
        os.sched_setaffinity(0, old)
    return {"value": round(sample.nbytes / best / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"{sample.desc}; best of {reps} passes ({total:.1f} s of CPU work), 1 thread pinned to "
                      f"core {core} of {len(old)} allowed; host CPU: {cpu_model()}"}


def cpu_baseline_threads(wl, seconds, threads=16):
    """Context only: the reference crc32c_append over the same sample split
    across `threads` host threads (the GPU box's CPU share is 16 cores per
    GPU); ctypes releases the GIL, so the slices run in parallel.  Fixed-stride
    samples only; None otherwise."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    sample = wl.cpu_sample()
    if sample.offsets is not None or sample.ref or not sample.available(O):
        return None
    n = max(1, min(threads, len(os.sched_getaffinity(0))))
    cuts = [sample.count * k // n for k in range(n + 1)]
    parts = [(sample.buf[cuts[k] * sample.stride:], cuts[k + 1] - cuts[k]) for k in range(n)]

    def once(pool):
        t = time.perf_counter()
        list(pool.map(lambda bc: O.reference_batch_fixed(bc[0], sample.stride, sample.length, bc[1],
                                                         seed=sample.seed), parts))
        return time.perf_counter() - t

    with ThreadPoolExecutor(n) as pool:
        once(pool)
        best, total, reps = 1e30, 0.0, 0
        while total < seconds or reps < 3:
            dt = once(pool)
            best, total, reps = min(best, dt), total + dt, reps + 1
    return {"value": round(sample.nbytes / best / GIB, 3), "unit": "GiB/s", "cores": n, "kind": "reference",
            "sample": f"{sample.desc}; {n} threads over contiguous slices, best of {reps} passes"}


def launch_ranks(args):
    """`--gpus N` without an outer launcher: run torch.distributed.run on this
    script as a child process (never an exec: nothing here has touched the GPU
    yet, and the parent never does) and return its exit status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: world size {world} != --gpus {args.gpus}")
    dry = args.dry_cpu
    use_pg = world > 1 or args.force_pg  # the collective path (RCCL, or gloo for --dry-cpu)
    shard = args.shard_base + rank        # this rank's shard of the global batch
    if dry:
        dev = torch.device("cpu")
        if use_pg:
            dist.init_process_group("gloo")
            assert dist.get_world_size() == args.gpus
        wl = W.DryCpuPages(shard)
        sync = lambda: None  # noqa: E731
        stream = None
    else:
        if use_pg:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            if dist.get_world_size() != args.gpus:
                sys.exit(f"bench.py: RCCL world size {dist.get_world_size()} != --gpus {args.gpus}")
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        F.gpu_init()
        wl = W.WORKLOADS[args.workload](dev, shard)
        stream = torch.cuda.current_stream(dev)
        sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731

    for _ in range(args.warmup):
        wl.step(stream)
    sync()
    if use_pg:
        dist.barrier()
    sync()

    # HIP events on the launch stream bracket the whole timed region (an event
    # pair per step would add its own overhead to every step: a timing event is
    # a barrier packet with a cache release on ROCm, ~10 us per pair measured
    # on a 0.2 ms varlen step); kernel_ms is the region's GPU time / K
    timed = not dry and not getattr(wl, "host_timed", False)
    if timed:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if timed:
        ev0.record(stream)
    for i in range(args.steps):
        wl.step(stream)
    if timed:
        ev1.record(stream)
    sync()
    if use_pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps if timed else elapsed / args.steps * 1e3

    ok = True
    if not args.no_verify:
        ok = wl.verify()

    stats = torch.tensor([elapsed, float(wl.bytes_per_step), 0.0 if ok else 1.0, kernel_ms, float(shard)],
                         dtype=torch.float64, device=dev)
    per_rank = [stats]
    if use_pg:  # RCCL all_gather over xGMI (gloo on the dry run): max time, byte count, parity, shards
        per_rank = [torch.empty_like(stats) for _ in range(world)]
        dist.all_gather(per_rank, stats)
    per_rank = [[float(x) for x in t.cpu()] for t in per_rank]
    elapsed = max(r[0] for r in per_rank)
    total_bytes = sum(r[1] for r in per_rank) * args.steps
    ok = all(r[2] == 0.0 for r in per_rank)

    if rank == 0:
        value = total_bytes / elapsed / GIB
        host_timed = getattr(wl, "host_timed", False)
        achieved = wl.algorithmic_bytes_per_step / (kernel_ms * 1e-3) / 1e9
        peak = wl.pcie_peak_gbs if host_timed else HBM_PEAK_GBS
        rec = {
            "metric": getattr(wl, "metric", None) or METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": wl.data_desc,
            "config": dict(wl.config, parallelism=f"{world} GPU(s), independent shards per rank; RCCL only "
                                                  "for max-time / byte-count reduction"),
            "pct_of_hbm_read_peak": round(100.0 * value * GIB / 1e9 / HBM_PEAK_GBS, 2),
            "parity_ok": bool(ok),
            "world_size": dist.get_world_size() if use_pg else 1,
            "collective": (dist.get_backend() if use_pg else None),
            "per_rank": [{"rank": i, "shard": int(r[4]), "bytes_per_step": int(r[1]), "elapsed_s": round(r[0], 6),
                          "avg_launch_ms": round(r[3], 4), "parity_ok": r[2] == 0.0} for i, r in enumerate(per_rank)],
            "roofline": {
                "bound": "pcie" if host_timed else "hbm",
                "kernel": wl.kernel_name,
                "achieved": round(achieved, 1),
                "peak": peak,
                "unit": "GB/s",
                "frac": round(achieved / peak, 4),
                "avg_launch_ms": round(kernel_ms, 4),
                "algorithmic_bytes_per_launch": wl.algorithmic_bytes_per_step,
                "traffic": W.pmc_traffic(args.workload),
                "traffic_commit": W.pmc_commit(args.workload),
            },
        }
        if dry:
            rec["data"] = "DRY RUN on CPU (harness test, not a measurement)"
        elif args.cpu_seconds > 0 and world == 1:  # reported at N=1 only
            rec["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds)
            mt = cpu_baseline_threads(wl, min(args.cpu_seconds, 3.0))
            if mt:
                rec["cpu_baseline_threads"] = mt  # context: the same reference path on 16 host cores
        print(json.dumps(rec), flush=True)
    if use_pg:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
