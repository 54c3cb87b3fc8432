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


def load(mode, kernel_substr):
    agg = collections.defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc", mode, "*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel_substr in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for t in csv.DictReader(open(f.replace("counter_collection", "kernel_trace"))):
            if kernel_substr in t["Kernel_Name"]:
                durs.append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9)
    return agg, durs


def main(mode="pages4k", workload="pages4k", kernel="k_pages4k", algorithmic=(1 << 20) * 4100, units=1 << 20):
    agg, durs = load(mode, kernel)
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    fetch = mean["FETCH_SIZE"] * 1024 * 2
    write = mean["WRITE_SIZE"] * 1024
    dur = sum(durs) / len(durs)
    out = {
        "workload": workload,
        "kernel": kernel,
        "source": f"rocprofv3 --pmc <counters> --kernel-trace, separate passes, {len(durs)} launches",
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


PRESETS = {
    "pages4k": ("pages4k", "pages4k", "k_pages4k", (1 << 20) * 4100, 1 << 20),
    "xxh3": ("xxh3", "xxh3-pages4k", "k_xxh3_rows", (1 << 20) * (4088 + 8), 1 << 20),
}

if __name__ == "__main__":
    main(*PRESETS[sys.argv[1] if len(sys.argv) > 1 else "pages4k"])
