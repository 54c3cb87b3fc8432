/* fdb_crc32c_testutil.h -- synthetic data generation and LDS poisoning for
 * tests and bench.py, exported by libfdb_crc32c_testutil.so.  Not part of the
 * product library or its boundary (include/). */
#ifndef FDB_CRC32C_TESTUTIL_H
#define FDB_CRC32C_TESTUTIL_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* d_dst[k] = splitmix64 word k of the stream seeded with `state`
 * (BASELINE.md generator: z = state + (k+1)*0x9E3779B97F4A7C15, then the
 * standard splitmix64 finaliser).  Asynchronous on `stream` (hipStream_t). */
int crc32c_testutil_fill_splitmix64(void* d_dst, uint64_t nwords, uint64_t state, void* stream);
/* Launches `blocks` workgroups that fill their whole 160 KiB LDS with a
 * pattern, so that the next kernels on those CUs start with garbage in LDS
 * (tests: no kernel may depend on LDS contents it did not write). */
int crc32c_testutil_poison_lds(uint32_t pattern, int blocks, void* stream);
#ifdef __cplusplus
}
#endif
#endif
