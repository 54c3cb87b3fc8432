// Batched Redwood page checks (redwood.hip): ArenaPage's postReadHeader /
// postReadPayload and preWrite (fdbserver/kvstore/IPager.h:480-560).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdbrw {

// Status per page (include/fdb_redwood.h): the first check that failed, in the
// reference's order, or 0.
constexpr uint8_t kOk = 0, kVersion = 1, kHeaderChecksum = 2, kWrongPageId = 3, kEncoding = 4, kDecoding = 5;

// Workspace: per page the payload job for the XXH3 engine (offset, length,
// seed = page ID), its digest, the stored digest, the head kernel's status;
// then the engine's planner workspace.
struct Ws {
	uint64_t *off, *len, *seed, *hash, *expect;
	uint8_t* st;
};

uint64_t workspace_bytes(uint64_t count, uint64_t page_size, int num_cus);
int verify(const uint8_t* pages, uint64_t ps, uint64_t count, const uint32_t* ids, uint32_t first_id,
           uint8_t* status, uint64_t* d_bad, int num_cus, void* ws, uint64_t ws_bytes, hipStream_t s);
int seal(uint8_t* pages, uint64_t ps, uint64_t count, const uint32_t* ids, uint32_t first_id, uint8_t* status,
         int num_cus, void* ws, uint64_t ws_bytes, hipStream_t s);

}  // namespace fdbrw
