"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/<mode>/*.csv) into
profiles/pmc_<workload>.json, applying the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of the
bytes of a wide coalesced streaming read (x2); WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Counter units are KiB."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(mode, kernel_substrs):
    """Per counter: its total over the step's kernels (every kernel whose name
    holds one of kernel_substrs) per step.  A step may run a kernel only
    sometimes (the varlen engine picks its route per batch, from the previous
    batch's statistics), so each pass is cut into steps by its most-launched
    kernel, the first step (the route not yet adapted) is dropped, and the
    totals of the remaining dispatches are divided by their step count."""
    sums = collections.defaultdict(float)
    dur = 0.0
    npass = 0
    launches = 0
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc", mode, "*_counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if any(k in r["Kernel_Name"] for k in kernel_substrs)]
        trace = [t for t in csv.DictReader(open(f.replace("counter_collection", "kernel_trace")))
                 if any(k in t["Kernel_Name"] for k in kernel_substrs)]
        if not rows:
            continue
        per_kernel = collections.defaultdict(set)
        for r in rows:
            per_kernel[r["Kernel_Name"]].add(int(r["Dispatch_Id"]))
        marker = max(per_kernel.values(), key=len)
        ids = sorted(marker)
        cut = ids[1] if len(ids) > 1 else ids[0]
        steps = len(ids) - 1 if len(ids) > 1 else 1
        counters = collections.defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) >= cut:
                counters[r["Counter_Name"]] += float(r["Counter_Value"])
        for c, v in counters.items():
            sums[c] += v / steps
        dur += sum((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9 for t in trace
                   if int(t["Dispatch_Id"]) >= cut) / steps
        npass += 1
        launches = max(launches, steps)
    return dict(sums), dur / max(npass, 1), launches


def main(mode="pages4k", workload="pages4k", kernel=("k_pages4k",), algorithmic=(1 << 20) * 4100, units=1 << 20):
    if callable(algorithmic):
        algorithmic, units = algorithmic()
    mean, dur, launches = load(mode, kernel)
    fetch = mean["FETCH_SIZE"] * 1024 * 2
    write = mean["WRITE_SIZE"] * 1024
    commit_file = os.path.join(ROOT, "gpurun_out", "pmc", "commit.txt")
    out = {
        "workload": workload,
        "commit": open(commit_file).read().strip() if os.path.exists(commit_file) else None,
        "kernel": " + ".join(kernel),
        "source": f"rocprofv3 --pmc <counters> --kernel-trace, separate passes, {launches} launches per pass",
        "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 reports half of wide streaming reads) + WRITE_SIZE(KiB)*1024",
        "hbm_bytes_per_launch": round(fetch + write),
        "fetch_bytes_per_launch": round(fetch),
        "write_bytes_per_launch": round(write),
        "algorithmic_bytes_per_launch": algorithmic,
        "traffic_over_algorithmic": round((fetch + write) / algorithmic, 4),
        "mean_profiled_launch_ms": round(dur * 1e3, 4),
        "effective_clock_ghz": round(mean["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9, 3) if "GRBM_GUI_ACTIVE" in mean else None,
        "per_unit": {k: round(v / units, 3) for k, v in mean.items()
                     if k.startswith("SQ_INSTS") or k in ("SQ_LDS_BANK_CONFLICT",)},
        "per_launch": {k: v for k, v in mean.items()},
    }
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "traffic_over_algorithmic", "effective_clock_ghz",
                                          "per_unit")}))


def _varlen(fn, per_buffer=20):
    """Algorithmic bytes of a bench_workloads varlen batch: data + 20 B per
    buffer (CRC: offset, length, 4-byte checksum; XXH3: 24 B, an 8-byte digest)."""
    def f():
        sys.path.insert(0, ROOT)
        import bench_workloads as W
        lens = getattr(W, fn)()
        return int(lens.sum()) + per_buffer * lens.size, lens.size
    return f


VARLEN_KERNELS = ("k_v7count", "k_xcount", "k_v7prep", "k_scan", "k_varlen7", "k_bigblocks", "k_xstream", "k_xgrab",
                  "k_xz", "k_xfin")
XXH3_VARLEN_KERNELS = ("k_xplan", "k_xscan", "k_xassign", "k_xlong", "k_xxh3_vrows")
PRESETS = {
    "pages4k": ("pages4k", "pages4k", ("k_pages4k",), (1 << 20) * 4100, 1 << 20),
    "pages8k": ("pages8k", "pages8k", ("k_pages4k",), (1 << 19) * 8196, 1 << 19),
    "xxh3": ("xxh3", "xxh3-pages4k", ("k_xxh3_rows",), (1 << 20) * (4088 + 8), 1 << 20),
    "zipf": ("zipf", "zipf", VARLEN_KERNELS, _varlen("zipf_lengths"), None),
    "chunks": ("chunks", "chunks", VARLEN_KERNELS, _varlen("chunk_lengths"), None),
    "xchunks": ("xchunks", "xxh3-chunks", XXH3_VARLEN_KERNELS, _varlen("chunk_lengths", 24), None),
    "xzipf": ("xzipf", "xxh3-zipf", XXH3_VARLEN_KERNELS, _varlen("zipf_lengths", 24), None),
    "scattered": ("scattered", "zipf-scattered", VARLEN_KERNELS, _varlen("zipf_lengths"), None),
}

if __name__ == "__main__":
    main(*PRESETS[sys.argv[1] if len(sys.argv) > 1 else "pages4k"])
