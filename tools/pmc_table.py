"""Tabulate gpurun_out/pmcsq/<mode>/*_counter_collection.csv per kernel (development)."""
import collections, csv, glob, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UNITS = {"pages4k": 1 << 20, "v4096": 1 << 18, "v1024": 1 << 20, "zipf": 406147, "chunks": 5773}  # buffers
for mode in sys.argv[1:] or ["pages4k", "v4096", "v1024", "zipf"]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", "pmcsq", mode, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for t in csv.DictReader(open(f.replace("counter_collection", "kernel_trace"))):
            dur[t["Kernel_Name"][:40]].append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-6)
    for k, c in agg.items():
        if "splitmix" in k:
            continue
        ms = sum(dur[k]) / len(dur[k])
        m = {n: sum(v) / len(v) for n, v in c.items()}
        u = UNITS[mode]
        print(f"{mode:8s} {k:40s} {ms:.4f} ms  clk {m.get('GRBM_GUI_ACTIVE', 0) / 8 / ms / 1e6:.2f} GHz")
        print("   per unit: " + "  ".join(f"{n[3:]}={v / u:.1f}" for n, v in sorted(m.items()) if n.startswith("SQ_INSTS")))
        print("   cycles  : " + "  ".join(f"{n[3:]}={v:.3g}" for n, v in sorted(m.items()) if not n.startswith("SQ_INSTS") and n != "GRBM_GUI_ACTIVE"))
