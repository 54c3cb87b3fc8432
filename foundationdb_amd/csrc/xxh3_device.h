// Device-side interface of the batched XXH3-64 kernels (xxh3_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdbxxh {

struct XxhParams {
	const uint8_t* base;
	const uint64_t* offsets;     // nullptr: fixed mode, buffer i at base + i*stride
	const uint64_t* lengths;     // varlen lengths
	uint64_t stride, length, count, seed;
	const uint64_t* seeds;       // per-buffer seeds or nullptr
	uint64_t* out;
	const uint64_t* wave_first;  // varlen: first buffer of every wave [nwave + 1] (planner output)
	const uint32_t* idx;         // fixed list mode: buffer i = base + idx[i]*stride, count = *d_count
	const uint64_t* d_count;     // ... varlen: may be null, else the batch is min(count, *d_count) buffers
	uint64_t ws_bytes;           // varlen: workspace size (room past the planner's arrays: the split route)
	uint64_t* hneed;             // varlen: host-mapped word for the blocks the long buffers needed (may be null)
	const uint8_t* lflag;        // (set by launch_xxh3) per buffer: the split route took it (not the row kernel's)
	uint32_t* err;               // stream's host-mapped status word (may be null): kErrXxhStall if a long-route wait ran out
	uint32_t ngen;               // (set by the launcher) k_xxh3_rows: workgroups per CU, the dispatch generations
};
// Status word values shared with the CRC engine's refusal flag (crc32c_gpu_stream_status).
constexpr uint32_t kErrRefused = 1, kErrXxhStall = 2;

constexpr unsigned kWavesPerBlock = 4;

// Long-buffer route (xxh3_split.hip): buffers longer than kXSplitMin, each
// computed by one CU's waves at once (k_xlong), largest first.  Planner
// output in the workspace:
constexpr uint64_t kXSplitMin = 16384;
// varlen buffers of 241 B .. kXQuadMax go to lane quads, longer ones to the rows
#ifndef FDBXXH_QUAD_MAX
#define FDBXXH_QUAD_MAX 1024
#endif
constexpr uint64_t kXQuadMax = FDBXXH_QUAD_MAX;
struct XEnt {       // one long buffer
	uint64_t p;     // its address
	uint64_t len, seed, idx;
};
// sh[] words: [0] long buffers routed, [1] k_xlong's dequeue counter, [2] set
// if a k_xlong wait ran out (never in a correct launch), [8 + c] the planner's
// cursor of size class c (c = 0: the largest).
constexpr uint32_t kXShWords = 32, kXClasses = 16;
struct XLong {
	uint64_t* sh;
	const XEnt* ents;     // [sh[0]], largest size class first
	uint64_t* out;
	uint64_t seed;        // uniform seed (per-buffer seeds travel in the entries)
	uint32_t* err;        // XxhParams::err
};
// Workspace per long block of room (the stream's need is counted in 1 KiB
// blocks; a long buffer has more than 16): one entry per 16 blocks.
constexpr uint64_t kXSplitBytesPerBlock = sizeof(XEnt) / 16;
int launch_xxh3_long(const XLong& S, int num_cus, bool seeds, hipStream_t stream);
// Resident 256-thread blocks per CU of the main kernel (occupancy query, cached).
int xxh3_blocks_per_cu();
inline uint64_t xxh3_nwave(int num_cus) { return (uint64_t)num_cus * xxh3_blocks_per_cu() * kWavesPerBlock; }
uint64_t xxh3_workspace_bytes(uint64_t count, uint64_t nwave);
// ... with room for the split route's `long_blocks` stripe-sum blocks (a
// bound: total bytes / 1024 + total bytes / 16384 + 2 covers any batch).
uint64_t xxh3_workspace_bytes_for(uint64_t count, uint64_t nwave, uint64_t long_blocks);
inline uint64_t xxh3_long_blocks_bound(uint64_t total_bytes) { return total_bytes / 1024 + total_bytes / 16384 + 2; }
int launch_xxh3(const XxhParams& P, int num_cus, void* ws, hipStream_t stream);
// Fixed-length (> 240 B, 16-byte aligned base and stride) pages over a device
// list: buffer j = base + idx[j]*stride, j < *d_count; P.count bounds the grid.
int launch_xxh3_pages_list(const XxhParams& P, int num_cus, hipStream_t stream);
// Chains of segments hashed in place (xxh3_segrows.hip): one 16-lane row per
// chain whose flag[c] is 2 (k_chain_ranges: two to kSegRowsMax segments,
// 241 B to kSegRowsMaxLen bytes), the chain's segments read where they lie.
constexpr uint32_t kSegRowsMax = 16;
constexpr uint64_t kSegRowsMaxLen = 1ull << 20;
struct SegRowsP {
	const uint8_t* base;
	const uint64_t* seg_off;
	const uint64_t* seg_len;
	const uint64_t* starts;
	const uint8_t* flag;
	uint64_t nchains, seed;
	const uint64_t* seeds;
	uint64_t* out;
};
int launch_xxh3_segrows(const SegRowsP& P, int num_cus, hipStream_t stream);
// Short chains staged in LDS (k_xxh3_lchain): a chain of 2..kLChainSegs
// segments and at most kLChainMax bytes, one wave each, listed by
// k_chain_ranges as {chain, first segment | segments << 56} in one list per
// XCD (a workgroup appends to its own XCD's).
#ifndef FDBXXH_LCMAX
#define FDBXXH_LCMAX 16384
#endif
constexpr uint32_t kLChainMax = FDBXXH_LCMAX, kLChainSegs = 8;
struct LChainP {
	const uint8_t* base;
	const uint64_t* seg_off;
	const uint64_t* seg_len;
	const uint64_t* list;    // [8][lcap][2]: per XCD, counts[16 x] entries
	const uint64_t* counts;  // [8 x 16]
	uint64_t lcap;
	uint64_t seed;
	const uint64_t* seeds;
	uint64_t* out;
};
int launch_xxh3_lchain(const LChainP& P, int num_cus, hipStream_t stream);
// Chains of segments (xxh3_chain.hip): gather into a staging area, then varlen.
uint64_t xxh3_chain_workspace_bytes(uint64_t nsegs, uint64_t nchains, uint64_t total_bytes, uint64_t nwave);
int launch_xxh3_chained(const uint8_t* base, const uint64_t* seg_off, const uint64_t* seg_len, uint64_t nsegs,
                        const uint64_t* starts, uint64_t nchains, uint64_t total_bytes, uint64_t seed,
                        const uint64_t* seeds, uint64_t* out, int num_cus, void* ws, hipStream_t stream);

}  // namespace fdbxxh
