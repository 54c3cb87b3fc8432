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
	// 4-byte slicing: slice4[3] = T0 (one byte), slice4[k] = slice4[k+1] followed by one zero byte.
	for (uint32_t b = 0; b < 256; ++b) t->slice4[3][b] = byte_step(b);
	for (int k = 2; k >= 0; --k)
		for (uint32_t b = 0; b < 256; ++b)
			t->slice4[k][b] = (t->slice4[k + 1][b] >> 8) ^ byte_step(t->slice4[k + 1][b] & 0xffu);
	// Block-to-block shift: consecutive 4 KiB blocks of one buffer.
	mul_tables_nibble(xpow8(4096), t->block);
	// Lane l holds bytes [64l, 64l+64) of a block: 64*(63-l) bytes follow it.
	for (int l = 0; l < 64; ++l) mul_tables_nibble(xpow8(64u * (63 - l)), t->lane[l]);
	// Variable shifts for pieces of split buffers and trailing-zero removal.
	for (int z = 0; z < 16; ++z) mul_tables_nibble(xpow8_inv(z), t->inv_z[z]);
	for (int q = 0; q < 4; ++q)
		for (int z = 0; z < 16; ++z) mul_tables_nibble(xpow8_inv(z + 1024u * (3 - q)), t->corr[q][z]);
	mul_tables_nibble(xpow8(1024u * kV7TabSlots), t->table_shift);
	for (int d = 0; d < 64; ++d)
		for (int z = 0; z < 16; ++z) {
			const int64_t e = 1024 * (int64_t)(d - 3) - z;
			mul_tables_nibble(e >= 0 ? xpow8((uint64_t)e) : xpow8_inv((uint64_t)-e), t->slotw[d][z]);
			mul_tables_nibble(xpow8(1024u * (d + 1) - z), t->carryw[d][z]);
		}
	for (int c = 0; c < 256; ++c) mul_tables_nibble(xpow8(16u * (255 - c)), t->chunkpow[c]);
	for (int i = 0; i < 4; ++i)
		for (int j = 0; j < 256; ++j) mul_tables_nibble(xpow8((4096ull * j) << (8 * i)), t->bpow[i][j]);
	for (int j = 0; j <= 64; ++j) mul_tables_nibble(xpow8_inv(64u * j), t->xinv64[j]);
	for (int c = 0; c < 64; ++c) {
		mul_tables_nibble(xpow8(64u * c), t->pow64[c]);
		mul_tables_nibble(xpow8(c), t->pow1[c]);
	}
	mul_tables_byte(xpow8(256), t->stride4);
	for (int l = 0; l < 64; ++l) mul_tables_nibble(xpow8_inv(4u * l), t->lane_s[l]);
	for (int m = 0; m < 64; ++m) {
		// x^(8*2^m) by repeated squaring of x^8
		uint32_t c = kOne >> 8;
		for (int k = 0; k < m; ++k) c = gf2_mul(c, c);
		mul_tables_nibble(c, t->pow2[m]);
	}
}

}  // namespace fdbcrc
