"""The C-ABI library: it loads, exports every symbol include/*.h declares, and
its host-side functions (the reference's scalar crc32c_append plus the GF(2)
combine helpers) reproduce the reference's outputs.  No device calls here."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import foundationdb_amd as F
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(pattern=os.path.join(ROOT, "include", "*.h")):
    names = set()
    for h in glob.glob(pattern):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s+\*?([a-z_][a-z0-9_]*)\s*\(", text, re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert {"crc32c_append", "crc32c_gpu_batch_fixed", "crc32c_gpu_batch_varlen", "crc32c_combine"} <= names
    assert {"crc32c_gpu_release_stream", "crc32c_pipeline_submit_varlen", "crc32c_pipeline_poll",
            "fdb_sqlite_verify_pages_host", "fdb_diskqueue_check_pages_host_submit"} <= names
    lib = ctypes.CDLL(F.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_test_utilities_are_not_in_the_product_library():
    """The splitmix64 generator and LDS poisoning live in their own
    libfdb_crc32c_testutil.so; the product library exports none of them."""
    names = declared_functions(os.path.join(ROOT, "foundationdb_amd", "testutil", "*.h"))
    assert names == {"crc32c_testutil_fill_splitmix64", "crc32c_testutil_poison_lds"}
    prod, tu = ctypes.CDLL(F.LIB_PATH), ctypes.CDLL(F.crc32c.TESTUTIL_LIB_PATH)
    assert all(hasattr(tu, n) and not hasattr(prod, n) for n in names)


def test_reference_signature():
    # same symbol name and C signature as contrib/crc32/include/crc32/crc32c.h:36-39
    hdr = open(os.path.join(ROOT, "include", "fdb_crc32c.h")).read()
    assert "uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length);" in hdr


def test_version_string():
    assert F.lib().crc32c_gpu_version().decode().startswith("fdb_crc32c")


def sm_bytes(nbytes, state):
    return O.splitmix64((nbytes + 7) // 8, state).view(np.uint8)[:nbytes].copy()


def test_host_append_golden(golden):
    for k in golden["kat"]:
        assert F.crc32c_append(k["seed"], bytes.fromhex(k["hex"])) == k["crc"], k["name"]
    e = golden["edge"]
    data = sm_bytes(e["nbytes"], e["state"])
    for si, s in enumerate(e["seeds"]):
        for off in range(e["offsets"]):
            for n in range(e["max_len"] + 1):
                assert F.crc32c_append(s, data[off:off + n]) == e["crc"][si][off][n]
    t = golden["threshold"]
    tdata = sm_bytes(t["nbytes"], t["state"])
    for off, n, s, want in t["cases"]:
        assert F.crc32c_append(s, tdata[off:off + n]) == want


def test_host_append_is_chainable(golden):
    c = golden["chained"]
    data = sm_bytes(c["nbytes"] + 64, c["state"])[:c["nbytes"]]
    crc = 0
    for i in range(0, c["nbytes"], c["read"]):
        crc = F.crc32c_append(crc, data[i:i + c["read"]])
    assert crc == c["crc"]


def test_combine_shift_zeros():
    rng = np.random.default_rng(3)
    for _ in range(300):
        a = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert F.crc32c_combine(F.crc32c_append(s, a), F.crc32c_append(0, b), len(b)) == O.crc32c(s, a + b)
        z = int(rng.integers(0, 100000))
        assert F.crc32c_append_zeros(s, z) == O.crc32c(s, bytes(z))
        r = int(rng.integers(0, 2**32))
        assert F.crc32c_shift(r, z) == O.shift(r, z)
    assert F.crc32c_append_zeros(0xDEADBEEF, 0) == 0xDEADBEEF
    assert F.crc32c_combine(0x1234, 0x5678, 0) == 0x1234 ^ 0x5678


def test_device_entry_points_reject_bad_arguments():
    # argument validation happens before any device work: null output with count>0
    L = F.lib()
    assert L.crc32c_gpu_batch_fixed(None, 4096, 4096, 5, 0, None, None, None) == -1
    assert L.crc32c_gpu_batch_varlen(None, None, None, 5, 0, None, None, None) == -1
    assert b"null" in L.crc32c_gpu_last_error()
    # count == 0 is a no-op success
    assert L.crc32c_gpu_batch_fixed(None, 0, 0, 0, 0, None, None, None) == 0


def test_python_batch_requires_device_tensor():
    import torch
    with pytest.raises(F.CRC32CError):
        F.batch_fixed(torch.zeros(4096, dtype=torch.uint8), 4096, 4096, 1)
