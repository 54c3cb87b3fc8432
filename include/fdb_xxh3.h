/*
 * Batched XXH3-64 on MI355X (gfx950) -- C ABI of libfdb_crc32c.so.
 *
 * Replaces, for device-resident batches, the per-buffer calls
 *   XXH64_hash_t XXH3_64bits(const void* data, size_t len);
 *   XXH64_hash_t XXH3_64bits_withSeed(const void* data, size_t len, XXH64_hash_t seed);
 * declared at flow/include/flow/xxhash.h:456,465 (xxHash v0.8.0, default
 * secret) and called per page/packet at
 *   fdbserver/kvstore/KeyValueStoreSQLite.cpp:112,138   (SQLite page checksum, 4088 B)
 *   fdbserver/kvstore/DiskQueue.cpp:1086-1088           (DiskQueue V2 page, 4088 B at +8)
 *   fdbserver/kvstore/IPager.h:300,308,325,330          (Redwood headers / payloads, seeded)
 *   fdbrpc/FlowTransport.cpp:1346,2043                  (packet checksums)
 * Results are bit-identical to those functions for every input, length
 * (0 .. 2^64-1) and seed; `seed` 0 is XXH3_64bits.
 *
 * Conventions (shared with include/fdb_crc32c.h): device pointers, caller
 * owns every buffer, calls are asynchronous on `stream` (a hipStream_t, NULL
 * = default stream), return 0 or a negative FDB_CRC32C_E* status; the
 * message of the last failure on this thread is crc32c_gpu_last_error().
 */
#ifndef FDB_XXH3_H
#define FDB_XXH3_H

#include <stdint.h>

#include "fdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Buffer i is bytes [d_base + i*stride, +length); d_out[i] = XXH3_64bits_withSeed(
 * buffer i, length, d_seeds ? d_seeds[i] : seed). */
int xxh3_gpu_batch_fixed(const void* d_base, uint64_t stride, uint64_t length, uint64_t count, uint64_t seed,
                         const uint64_t* d_seeds, uint64_t* d_out, void* stream);

/* Buffer i is bytes [d_base + d_offsets[i], +d_lengths[i]) (any alignment,
 * any order, overlaps allowed).  Work is balanced over the GPU by bytes,
 * whole buffers per wavefront. */
int xxh3_gpu_batch_varlen(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                          uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* stream);

/* Same with a caller-owned device workspace (16-byte aligned, size from
 * xxh3_gpu_varlen_workspace_bytes): no allocation, capture-safe.
 * Buffers longer than 16 KiB take the SPLIT route -- the stripe sums of every
 * 1 KiB block computed in parallel over the whole GPU, then one short
 * sequential pass of scrambles per buffer (xxhash.h:3641-3718) -- when the
 * workspace has room for them: xxh3_gpu_varlen_workspace_bytes_for(count,
 * total_bytes) bytes (total_bytes >= the sum of the lengths) always do;
 * with less room they run one buffer per 16-lane row (same digests).
 * The convenience form sizes the library's workspace from the stream's last
 * batch. */
uint64_t xxh3_gpu_varlen_workspace_bytes(uint64_t count);
uint64_t xxh3_gpu_varlen_workspace_bytes_for(uint64_t count, uint64_t total_bytes);
int xxh3_gpu_batch_varlen_ws(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                             uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* d_workspace,
                             uint64_t workspace_bytes, void* stream);

/* Chains: d_out[c] = XXH3_64bits_withSeed(concatenation of segments
 * [d_chain_starts[c], d_chain_starts[c+1]), d_seeds ? d_seeds[c] : seed) --
 * a packet spread over a PacketBuffer chain, which FlowTransport hashes with
 * XXH3_64bits_reset / _update per buffer / _digest
 * (fdbrpc/FlowTransport.cpp:2025-2068).  Segment j is the d_seg_lengths[j]
 * bytes at d_base + d_seg_offsets[j]; d_chain_starts holds nchains + 1
 * non-decreasing values <= nsegs.  The segments are gathered on the device
 * into a staging area of `total_bytes` (the caller's bound on the sum of the
 * segment lengths: a smaller bound leaves the digests undefined, but no read or
 * write leaves the workspace -- the per-chain ranges are clamped to the
 * staging area and the chain starts to [0, nsegs]), then hashed per chain. */
int xxh3_gpu_batch_chained(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                           uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint64_t total_bytes,
                           uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* stream);
uint64_t xxh3_gpu_chained_workspace_bytes(uint64_t nsegs, uint64_t nchains, uint64_t total_bytes);
int xxh3_gpu_batch_chained_ws(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                              uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint64_t total_bytes,
                              uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* d_workspace,
                              uint64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FDB_XXH3_H */
