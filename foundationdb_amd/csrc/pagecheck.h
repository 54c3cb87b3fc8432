// Batched page-format verifiers (pagecheck.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace fdbpc {

uint64_t workspace_bytes(uint64_t count);
// ctr: the stream's eight counter words (fdbcrc::stream_aux + kAuxPageCtr),
// zero on entry and left zero
int sqlite_verify(const uint8_t* pages, uint64_t page_size, uint64_t count, uint32_t first_pgno, uint8_t* status,
                  uint64_t* d_bad, const fdbcrc::DevTables* tabs, int num_cus, void* ws, unsigned long long* ctr,
                  hipStream_t s);
int diskqueue_check(const uint8_t* pages, uint64_t count, uint8_t* ok, uint64_t* d_bad,
                    const fdbcrc::DevTables* tabs, int num_cus, void* ws, unsigned long long* ctr, hipStream_t s);
int sqlite_seal(uint8_t* pages, uint64_t ps, uint64_t count, uint32_t first_pgno, int num_cus, void* ws,
                hipStream_t s);
int diskqueue_seal(uint8_t* pages, uint64_t count, const fdbcrc::DevTables* tabs, int num_cus, void* ws,
                   unsigned long long* ctr, hipStream_t s);

}  // namespace fdbpc
