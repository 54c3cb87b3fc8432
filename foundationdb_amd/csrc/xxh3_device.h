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
	const uint64_t* d_count;
	uint64_t ws_bytes;           // varlen: workspace size (room past the planner's arrays: the split route)
	uint64_t* hneed;             // varlen: host-mapped word for the blocks the long buffers needed (may be null)
	const uint8_t* lflag;        // (set by launch_xxh3) per buffer: the split route took it (not the row kernel's)
};

constexpr unsigned kWavesPerBlock = 4;

// Split route for long buffers (xxh3_split.hip): buffers longer than
// kXSplitMin whose 1 KiB blocks' stripe sums are computed in parallel
// (phase A, PIECES of up to kXPieceBlocks blocks) and chained per buffer
// (phase B).  Planner output in the workspace:
constexpr uint64_t kXSplitMin = 16384;
constexpr uint32_t kXPieceBlocks = 64;
constexpr uint64_t kXBig = 256;  // phase B starts the chains of this many blocks or more first
struct XEnt {       // one long buffer
	uint64_t F;     // its first block in the flat stripe-sum array D
	uint64_t len, seed, idx;
};
struct XPiece {     // kXPieceBlocks consecutive blocks of one long buffer (fewer at its end)
	uint64_t p;     // the buffer's address
	uint64_t len, d, seed;  // d: flat index of block b0 in D
	uint32_t b0, nb;
	uint64_t pad;
};
struct XSplit {
	const uint64_t* sh;   // planner totals: [0] long buffers, [1] blocks, [2] pieces, [3] blocks per phase-A wave, [4] big entries
	const uint64_t* astart;  // [nwa]: phase-A wave w's first piece << 6 | its first block in that piece (~0: none)
	uint64_t nwa;            // phase-A waves the planner divided D among
	const uint64_t* big;     // [sh[4]]: the entries of kXBig blocks or more (any order)
	const XEnt* ents;
	const XPiece* pcs;
	uint64_t* D;          // 8 x u64 per block
	uint64_t* out;
	uint64_t seed;        // uniform seed (per-buffer seeds travel in the entries)
};
// Per block of capacity: D (64 B) + entries and pieces (<= 8 B): 72 B (plus a
// flag byte per buffer).
constexpr uint64_t kXSplitBytesPerBlock = 72;
int launch_xxh3_split(const XSplit& S, int num_cus, bool seeds, hipStream_t stream);
// Waves of the phase-A launch (the planner's share of D per wave).
uint64_t xxh3_split_waves(int num_cus);
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
// Chains of segments (xxh3_chain.hip): gather into a staging area, then varlen.
uint64_t xxh3_chain_workspace_bytes(uint64_t nsegs, uint64_t nchains, uint64_t total_bytes, uint64_t nwave);
int launch_xxh3_chained(const uint8_t* base, const uint64_t* seg_off, const uint64_t* seg_len, uint64_t nsegs,
                        const uint64_t* starts, uint64_t nchains, uint64_t total_bytes, uint64_t seed,
                        const uint64_t* seeds, uint64_t* out, int num_cus, void* ws, hipStream_t stream);

}  // namespace fdbxxh
