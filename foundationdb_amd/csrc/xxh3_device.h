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
};

constexpr unsigned kWavesPerBlock = 4;
// Resident 256-thread blocks per CU of the main kernel (occupancy query, cached).
int xxh3_blocks_per_cu();
inline uint64_t xxh3_nwave(int num_cus) { return (uint64_t)num_cus * xxh3_blocks_per_cu() * kWavesPerBlock; }
uint64_t xxh3_workspace_bytes(uint64_t count, uint64_t nwave);
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
