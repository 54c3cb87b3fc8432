"""Page-kernel A/B probe (development): times batch_fixed on 1 Mi x 4 KiB pages
for each library given on the command line, interleaved, and checks each
variant's checksums against the reference digest."""
import ctypes, json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    import torch
    import foundationdb_amd as F
    dev = torch.device("cuda:0")
    F.gpu_init()
    n = 1 << 20
    length = int(os.environ.get("PLEN", "4096"))
    count = int(os.environ.get("PCOUNT", n * 4096 // length))
    big = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    F.fill_splitmix64(big, 0x5EED)
    out = torch.empty(count, dtype=torch.uint32, device=dev)
    fn = lambda: F.batch_fixed(big, length, length, count, out=out)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    res = []
    for rep in range(3):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(30):
            fn()
        b.record(); torch.cuda.synchronize()
        res.append(a.elapsed_time(b) / 30)
    h = out.cpu().numpy()
    print(json.dumps({"ms": min(res), "all": res, "xor": int(h.view("u4").astype("u8").sum() & 0xffffffffffffffff)}))
    sys.exit(0)
libs = sys.argv[1:]
for rnd in range(2):
    for L in libs:
        env = dict(os.environ, FDBCRC_LIB=os.path.join(ROOT, "foundationdb_amd", "lib", f"libfdb_crc32c{L}.so"))
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=120)
        if r.returncode:
            print(L, "FAILED", r.stderr[-500:]); sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        gb = int(os.environ.get("PCOUNT", 1 << 20)) * 4096 / d["ms"] / 1e6
        print(f"{L or 'base':12s} {d['ms']:.4f} ms  {gb:7.1f} GB/s  {gb * 1e9 / 2**30 / 1e3:7.1f} GiB/s  sum={d['xor']:#x}  {['%.4f' % x for x in d['all']]}", flush=True)
