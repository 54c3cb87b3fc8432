// Synthetic-input generator for tests and bench.py (not on the checksum path).
// Fills device memory with the splitmix64 stream of BASELINE.md: word k is
// mix(state + (k+1)*0x9E3779B97F4A7C15), little-endian -- the same stream as
// oracle_splitmix64_fill, so 4 GiB page batches need no host-to-device copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fdb_crc32c_testutil.h"

namespace fdbcrc {

__global__ void k_splitmix64(uint64_t* __restrict__ dst, uint64_t nwords, uint64_t state) {
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += stride) {
		uint64_t z = state + (k + 1) * 0x9E3779B97F4A7C15ull;
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		dst[k] = z ^ (z >> 31);
	}
}

}  // namespace fdbcrc

extern "C" int crc32c_testutil_fill_splitmix64(void* d_dst, uint64_t nwords, uint64_t state, void* stream) {
	if (nwords == 0) return 0;
	if (!d_dst) return -1;
	uint64_t blocks = (nwords + 255) / 256;
	if (blocks > 8192) blocks = 8192;
	fdbcrc::k_splitmix64<<<(unsigned)blocks, 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
	    static_cast<uint64_t*>(d_dst), nwords, state);
	return hipGetLastError() == hipSuccess ? 0 : -3;
}
