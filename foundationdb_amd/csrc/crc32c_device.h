// Shared between the HIP kernels and the host engine: the compact operator
// tables that each workgroup expands into its bank-replicated LDS image.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace fdbcrc {

struct DevTables {
	uint32_t slice[2][256];     // [0] byte + one zero byte (T1), [1] single byte (T0)
	uint32_t horner[8][16];     // nibble tables of x^(8*1008): row-to-row lane shift
	uint32_t lane[64][8][16];   // nibble tables of x^(128*(63-l)): lane l to end of row
};

// Build the tables on the host (crc32c_tables.cpp).
void build_dev_tables(DevTables* t);

int launch_pages(int rows, const uint8_t* base, uint64_t stride, uint64_t count, uint32_t seed,
                 const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream);
int launch_general(const uint8_t* base, uint64_t stride, uint64_t length, const uint64_t* offsets,
                   const uint64_t* lengths, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                   const DevTables* tabs, int num_cus, hipStream_t stream);

}  // namespace fdbcrc
