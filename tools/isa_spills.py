"""Where a kernel's spills sit (development): scratch accesses and SGPR
spills (v_writelane / v_readlane to spill lanes) by enclosing loop.
  python tools/isa_spills.py <file.hip> <kernel substring> [extra hipcc flags]"""
import re
import subprocess
import sys

src, kname = sys.argv[1], sys.argv[2]
flags = sys.argv[3:]
asm = "/tmp/isa_spills.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-o",
                asm, src] + flags, check=True, stderr=subprocess.DEVNULL)
s = open(asm).read().split("\n")
starts = {m.group(1): i for i, l in enumerate(s) for m in [re.match(r"^(_Z\w+):", l)] if m}
for k, a in starts.items():
    if kname not in k:
        continue
    b = a + 1
    while not s[b].startswith(".Lfunc_end"):
        b += 1
    body = s[a:b]
    labpos = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labpos and labpos[m.group(1)] < i:
            loops.append((labpos[m.group(1)], i))
    print(k, "lines", len(body))
    for i, l in enumerate(body):
        if "scratch_" in l or ("v_writelane" in l or "v_readlane" in l) and "spill" in l.lower():
            inl = [(x, y) for x, y in loops if x <= i <= y]
            big = max([y - x for x, y in inl] or [0])
            print("  %6d %-50s loops=%d largest=%d" % (i, l.strip()[:50], len(inl), big))
