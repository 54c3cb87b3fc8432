"""The host scalar drop-in crc32c_append (contrib/crc32/crc32c.cpp:346-356):
both implementations -- SSE4.2 (3 streams x 1 KiB, then 3 x 256 B) and the
sliced-table fallback the reference takes without the crc32 instruction
(append_table, :124-172, dispatch :344-356) -- against the reference's own
outputs, every alignment and the tier boundaries; and the same checks through
a C++ program that includes the REFERENCE's header and links the library."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_HDR = "/root/reference/contrib/crc32/include"

CHECK = r"""
import sys, json, numpy as np
sys.path.insert(0, %r)
import foundationdb_amd as F
from oracle import oracle as O
g = json.load(open(%r))
L = F.lib()
L.crc32c_host_impl.restype = __import__("ctypes").c_char_p
impl = L.crc32c_host_impl().decode()
bad = 0
for k in g["kat"]:
    bad += F.crc32c_append(k["seed"], bytes.fromhex(k["hex"])) != k["crc"]
e = g["edge"]
data = O.splitmix64(e["nbytes"] // 8, e["state"]).view(np.uint8)
for si, s in enumerate(e["seeds"]):
    for off in range(e["offsets"]):
        for n in range(e["max_len"] + 1):
            bad += F.crc32c_append(s, data[off:off + n]) != e["crc"][si][off][n]
t = g["threshold"]
td = O.splitmix64((t["nbytes"] + 7) // 8, t["state"]).view(np.uint8)
for off, n, s, want in t["cases"]:
    bad += F.crc32c_append(s, td[off:off + n]) != want
rng = np.random.default_rng(5)
for _ in range(400):  # both interleave tiers and their remainders, any alignment
    n = int(rng.integers(0, 12000)); off = int(rng.integers(0, 64)); s = int(rng.integers(0, 2**32))
    bad += F.crc32c_append(s, td[off:off + n]) != O.crc32c(s, td[off:off + n])
print(json.dumps({"impl": impl, "bad": int(bad)}))
"""


def run_check(env):
    code = CHECK % (ROOT, os.path.join(ROOT, "tests", "golden", "crc32c_golden.json"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_sse42_path_matches_reference():
    res = run_check({"FDB_CRC32C_FORCE_SOFTWARE": "0"})
    assert res["bad"] == 0
    assert res["impl"] in ("sse4.2", "sliced")


def test_forced_software_fallback_matches_reference():
    res = run_check({"FDB_CRC32C_FORCE_SOFTWARE": "1"})
    assert res == {"impl": "sliced", "bad": 0}


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_HDR, "crc32", "crc32c.h")),
                    reason="reference tree absent (the consumer compiles against its header)")
def test_compiled_consumer_of_reference_header(tmp_path, golden):
    """A C++ translation unit written against the REFERENCE's header
    (contrib/crc32/include/crc32/crc32c.h:36-39), linked against
    libfdb_crc32c.so instead of contrib/crc32: the link-time drop-in claim."""
    exe = tmp_path / "consumer"
    lib_dir = os.path.dirname(os.environ.get("FDBCRC_LIB") or os.path.join(ROOT, "foundationdb_amd", "lib", "x"))
    lib_name = os.path.basename(os.environ.get("FDBCRC_LIB", "libfdb_crc32c.so"))[3:-3]
    cmd = ["g++", "-O1", "-std=c++17", "-I", REF_HDR, os.path.join(ROOT, "tests", "consumer", "ref_header_consumer.cpp"),
           "-L", lib_dir, f"-l{lib_name}", f"-Wl,-rpath,{lib_dir}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    lines = [f"{k['seed']} {len(bytes.fromhex(k['hex']))} {k['hex'] or '-'} {k['crc']}" for k in golden["kat"]]
    c = golden["chained"]
    lines.append(f"chain {c['state']} {c['nbytes']} {c['read']} {c['crc']}")
    r = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert r.stdout.strip() == f"ok {len(golden['kat']) + 1}"
