"""Count instructions by class inside each loop of one kernel's ISA (development).
   python tools/isa_loops.py file.s kernel_symbol_prefix"""
import re, sys, collections
src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(sym) and ":" in l)
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
cur = ("entry", 0)
stats = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):", l)
    if m:
        a = re.search(r"Loop: Header=(\S+) Depth=(\d+)", l)
        b = re.search(r"=>This Loop Header: Depth=(\d+)", l)
        if a:
            cur = (a.group(1), int(a.group(2)))
        elif b:
            cur = (m.group(1).lstrip("."), int(b.group(1)))
        else:
            cur = ("outside", 0)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    cls = ("scratch" if op.startswith("scratch") else "vmem" if op.startswith(("global_", "buffer_")) else
           "lds" if op.startswith("ds_") else "smem" if op.startswith("s_load") or op.startswith("s_buffer") else
           "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "other")
    stats[cur][cls] += 1
for k, v in sorted(stats.items(), key=lambda kv: -kv[0][1]):
    print(k, dict(v))
