// Grouped chains: one CRC-32C per CHAIN of non-contiguous segments.
//
// The reference builds such checksums by calling crc32c_append segment after
// segment with the running CRC as the next seed:
//   MutationRef::populateChecksum / validateChecksum
//     crc = type; crc = append(crc, param1); crc = append(crc, param2)
//     (fdbclient/include/fdbclient/CommitTransaction.h:302-304, 330-332)
//   FileTransfer's whole-file CRC over 8 KiB reads (fdbrpc/FileTransfer.cpp:29-37)
//   a packet spread over a PacketBuffer chain (fdbrpc/FlowTransport.cpp:2025-2068)
// Here every segment of the batch is checksummed independently by the
// variable-length engine and the chains are folded on the device with the
// GF(2) identity of crc32c_math.h.  For a chain of segments M_1..M_k with
// S_j bytes after segment j and T bytes in all:
//   raw(~seed, M_1..M_k) = ~seed * x^(8T)  xor  sum_j raw(0, M_j) * x^(8 S_j)
// and crc32c_append(0xffffffff, M) = ~raw(0, M), so the engine runs with
// seed 0xffffffff and k_chain_fold applies the shifts.
//
// k_chain_fold: one wavefront per chain.  The chain's segments are taken 64
// at a time from its end; a lane's suffix byte count is a wave suffix scan
// plus the bytes of the chunks already folded; the shift by S_j bytes is a
// product of x^(8*2^m) factors (nibble tables pow2[m], L2-resident); the
// 64 terms XOR-reduce across the wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_common.h"
#include "crc32c_device.h"

namespace fdbcrc {

__device__ __forceinline__ uint32_t mul_global(const uint32_t (*__restrict__ t)[16], uint32_t s) {
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= t[n][(s >> (4 * n)) & 15u];
	return r;
}

// r * x^(8n), lane-divergent n
__device__ __forceinline__ uint32_t shift_bytes(const DevTables* __restrict__ tabs, uint32_t r, uint64_t n) {
	for (int m = 0; m < 64 && __any((n >> m) != 0); ++m)
		if ((n >> m) & 1) r = mul_global(tabs->pow2[m], r);
	return r;
}

__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d) {
	const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, d, 64);
	const uint32_t hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), d, 64);
	return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void k_chain_fold(const uint64_t* __restrict__ starts, uint64_t nchains,
                                                    const uint64_t* __restrict__ lengths,
                                                    const uint32_t* __restrict__ segcrc, uint32_t seed,
                                                    const uint32_t* __restrict__ seeds, uint32_t* __restrict__ out,
                                                    const DevTables* __restrict__ tabs) {
	const int lane = threadIdx.x & 63;
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
	for (uint64_t c = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; c < nchains; c += nwaves) {
		const uint64_t a = rdfirst64(starts[c]), e = rdfirst64(starts[c + 1]);
		uint32_t acc = 0;
		uint64_t carry = 0;  // bytes of the chunks already folded (they follow this chunk)
		for (uint64_t hi = e; hi > a;) {
			const uint64_t lo = hi - a > 64 ? hi - 64 : a;
			const uint64_t j = lo + lane;
			const bool valid = j < hi;
			const uint64_t len = valid ? lengths[j] : 0;
			const uint32_t r = valid ? ~segcrc[j] : 0u;  // raw(0, M_j)
			uint64_t incl = len;  // bytes of this lane's segment and every later one in the chunk
#pragma unroll
			for (int d = 1; d < 64; d <<= 1) {
				const uint64_t t = shfl_down64(incl, d);
				if (lane + d < 64) incl += t;
			}
			acc ^= wave_xor(shift_bytes(tabs, r, incl - len + carry));
			carry += rdlane64(incl, 0);
			hi = lo;
		}
		const uint32_t s = seeds ? seeds[c] : seed;
		acc ^= shift_bytes(tabs, ~s, carry);
		if (lane == 0) out[c] = ~acc;
	}
}

int launch_chain_fold(const uint64_t* starts, uint64_t nchains, const uint64_t* lengths, const uint32_t* segcrc,
                      uint32_t seed, const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus,
                      hipStream_t stream) {
	if (nchains == 0) return 0;
	uint64_t blocks = (nchains + 3) / 4;
	const uint64_t cap = (uint64_t)num_cus * 16;
	if (blocks > cap) blocks = cap;
	k_chain_fold<<<(unsigned)blocks, 256, 0, stream>>>(starts, nchains, lengths, segcrc, seed, seeds, out, tabs);
	return 0;
}

}  // namespace fdbcrc
