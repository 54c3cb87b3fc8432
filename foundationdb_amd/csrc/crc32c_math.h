// GF(2) arithmetic for CRC-32C (Castagnoli, reflected polynomial 0x82f63b78).
//
// Everything in the engine is built from one identity: a raw CRC register is
// a polynomial modulo P, so appending n zero bytes multiplies it by x^(8n)
// mod P and
//     raw(A || B) = raw(A) * x^(8|B|)  xor  raw(B).
// The reference uses the same identity with two fixed distances (LONG_SHIFT
// 8192 / SHORT_SHIFT 256) to merge its three interleaved SSE4.2 streams
// (contrib/crc32/crc32c.cpp:175-178, 268-269, 286-287).  Here the distances
// are whatever the GPU lane geometry needs, and every operator table is
// generated from the polynomial at start-up -- nothing is copied from
// crc32c-generated-constants.cpp.
//
// Reflected convention: bit 31 of a register word is the coefficient of x^0,
// bit 0 the coefficient of x^31.
#pragma once
#include <stdint.h>

namespace fdbcrc {

constexpr uint32_t kPoly = 0x82f63b78u;   // contrib/crc32/crc32c-generated-constants.cpp:23
constexpr uint32_t kOne = 0x80000000u;    // the polynomial 1

// a * b mod P in the reflected domain.
inline uint32_t gf2_mul(uint32_t a, uint32_t b) {
	uint32_t r = 0;
	for (int i = 0; i < 32; ++i) {
		if (a & 0x80000000u) r ^= b;
		a <<= 1;
		b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
	}
	return r;
}

// x^(8n) mod P
inline uint32_t xpow8(uint64_t nbytes) {
	uint32_t result = kOne;
	uint32_t pw = kOne >> 8;  // x^8
	while (nbytes) {
		if (nbytes & 1) result = gf2_mul(result, pw);
		pw = gf2_mul(pw, pw);
		nbytes >>= 1;
	}
	return result;
}

// x^(-8n) mod P.  x is invertible because P has a constant term:
// x * x^-1 == 1 gives x^-1 = ((kPoly ^ kOne) << 1) | 1 in the reflected domain.
inline uint32_t xpow8_inv(uint64_t nbytes) {
	const uint32_t xinv = ((kPoly ^ kOne) << 1) | 1u;
	uint32_t pw = kOne;
	for (int i = 0; i < 8; ++i) pw = gf2_mul(pw, xinv);  // x^-8
	uint32_t result = kOne;
	while (nbytes) {
		if (nbytes & 1) result = gf2_mul(result, pw);
		pw = gf2_mul(pw, pw);
		nbytes >>= 1;
	}
	return result;
}

// The one-byte register table: raw register after feeding byte b into a zero
// register (append_trivial's 8 bit-steps, contrib/crc32/crc32c.cpp:85-92).
inline uint32_t byte_step(uint32_t b) {
	uint32_t r = b;
	for (int k = 0; k < 8; ++k) r = (r & 1u) ? (r >> 1) ^ kPoly : (r >> 1);
	return r;
}

// Multiplication by a fixed constant c as byte-indexed tables:
// reg*c = T[0][reg&255] ^ T[1][(reg>>8)&255] ^ T[2][(reg>>16)&255] ^ T[3][reg>>24]
inline void mul_tables_byte(uint32_t c, uint32_t out[4][256]) {
	for (int k = 0; k < 4; ++k)
		for (uint32_t v = 0; v < 256; ++v) out[k][v] = gf2_mul(v << (8 * k), c);
}

// The same operator as nibble-indexed tables: 8 lookups of 16 entries.
inline void mul_tables_nibble(uint32_t c, uint32_t out[8][16]) {
	for (int k = 0; k < 8; ++k)
		for (uint32_t v = 0; v < 16; ++v) out[k][v] = gf2_mul(v << (4 * k), c);
}

}  // namespace fdbcrc
