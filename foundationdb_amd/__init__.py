"""MI355X-native batched CRC-32C for FoundationDB's crc32c_append() call sites.

The product is the C-ABI shared library ``foundationdb_amd/lib/libfdb_crc32c.so``
(header ``include/fdb_crc32c.h``).  This package is the Python host mirror of
that boundary: ``crc32c_append`` with the reference's signature semantics and
batched device entry points over torch-allocated HBM buffers.
"""
from .crc32c import (  # noqa: F401
    CRC32CError,
    Pipeline,
    PipelineJob,
    LIB_PATH,
    batch_chained,
    batch_fixed,
    batch_varlen,
    crc32c_append,
    crc32c_append_zeros,
    crc32c_combine,
    crc32c_shift,
    fill_splitmix64,
    poison_lds,
    release_stream,
    stream_bytes,
    stream_status,
    workspace_status,
    testutil_lib,
    gpu_init,
    host_impl,
    lib,
    varlen_workspace_bytes,
)

__version__ = "0.1.0"
