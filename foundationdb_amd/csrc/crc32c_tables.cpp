// Host-side generation of the GPU operator tables (uploaded once per device).
#include <string.h>

#include "crc32c_device.h"
#include "crc32c_math.h"

namespace fdbcrc {

void build_dev_tables(DevTables* t) {
	memset(t, 0, sizeof(*t));
	for (uint32_t b = 0; b < 256; ++b) {
		const uint32_t t0 = byte_step(b);
		t->slice[1][b] = t0;                                  // T0: one byte
		t->slice[0][b] = (t0 >> 8) ^ byte_step(t0 & 0xffu);   // T1: byte then one zero byte
	}
	// Row-to-row shift: a lane's next chunk sits 1024 bytes after its previous
	// one; feeding 16 bytes already multiplies by x^128, so pre-multiply by
	// x^(8*1008).
	mul_tables_nibble(xpow8(1008), t->horner);
	// Lane l's chunk is followed by 16*(63-l) bytes of the same row.
	for (int l = 0; l < 64; ++l) mul_tables_nibble(xpow8(16u * (63 - l)), t->lane[l]);
}

}  // namespace fdbcrc
