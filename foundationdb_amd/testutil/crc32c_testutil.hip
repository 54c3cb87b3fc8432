// Test and bench utilities, built into their own libfdb_crc32c_testutil.so (never
// linked into the product library).  Synthetic-input generator:
// Fills device memory with the splitmix64 stream of BASELINE.md: word k is
// mix(state + (k+1)*0x9E3779B97F4A7C15), little-endian -- the same stream as
// oracle_splitmix64_fill, so 4 GiB page batches need no host-to-device copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fdb_crc32c_testutil.h"

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

// Fills all of a workgroup's LDS with a pattern, one workgroup per CU and
// more: the next kernels on those CUs start with garbage in LDS, as they may
// on a GPU that ran other work (tests: no kernel may read LDS it did not write).
__global__ __launch_bounds__(1024) void k_poison_lds(uint32_t pattern) {
	__shared__ uint32_t lds[160 * 1024 / 4];
	for (uint32_t k = threadIdx.x; k < 160 * 1024 / 4; k += blockDim.x) lds[k] = pattern ^ (k * 0x9E3779B9u);
	__syncthreads();
	if (lds[(threadIdx.x * 37) % (160 * 1024 / 4)] == 0x12345678u && pattern == 0u) lds[0] = 1u;  // keep the stores
}

}  // namespace fdbcrc

extern "C" int crc32c_testutil_poison_lds(uint32_t pattern, int blocks, void* stream) {
	fdbcrc::k_poison_lds<<<(unsigned)(blocks > 0 ? blocks : 1), 1024, 0, reinterpret_cast<hipStream_t>(stream)>>>(pattern);
	return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int crc32c_testutil_fill_splitmix64(void* d_dst, uint64_t nwords, uint64_t state, void* stream) {
	if (nwords == 0) return 0;
	if (!d_dst) return -1;
	uint64_t blocks = (nwords + 255) / 256;
	if (blocks > 8192) blocks = 8192;
	fdbcrc::k_splitmix64<<<(unsigned)blocks, 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
	    static_cast<uint64_t*>(d_dst), nwords, state);
	return hipGetLastError() == hipSuccess ? 0 : -3;
}
