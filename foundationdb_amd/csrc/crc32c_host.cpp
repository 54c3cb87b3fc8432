// Host-side scalar CRC-32C: the link-compatible crc32c_append symbol plus the
// GF(2) shift/combine helpers the batched API needs to merge partial results.
//
// crc32c_append has the semantics of contrib/crc32/crc32c.cpp:346-356 (seed
// pre-inversion :197, post-inversion :310, any alignment, length 0 returns the
// seed).  It exists so a FoundationDB build can link this library in place of
// contrib/crc32 for its single-buffer call sites; the batched GPU entry points
// never route through it.
//
// Implementation: SSE4.2 crc32q (8 bytes per instruction; the reference's
// Linux build takes its 4-byte crc32l branch, since _M_X64 is an MSVC macro,
// crc32c.cpp:207-299) over three independent streams -- kBlock bytes each while
// 3*kBlock remain, then kShort bytes each while 3*kShort remain (the
// reference's two tiers, crc32c.cpp:212-244, at other distances) -- merged with
// byte-indexed tables of x^(8*kBlock) / x^(8*kShort) (own generator,
// crc32c_math.h); a sliced-table fallback when the CPU lacks SSE4.2 or
// FDB_CRC32C_FORCE_SOFTWARE is set in the environment (crc32c_host_impl()
// names the implementation in use).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

#include "crc32c_math.h"

namespace fdbcrc {
namespace {

constexpr size_t kBlock = 1024;  // bytes per stream per interleaved round
constexpr size_t kShort = 256;   // the same for 768 B .. 3 KiB remainders

struct HostTables {
	uint32_t slice[8][256];     // slice[k][b]: byte b followed by k zero bytes
	uint32_t merge[4][256];     // x^(8*kBlock) as byte tables
	uint32_t merge_s[4][256];   // x^(8*kShort)
	HostTables() {
		for (uint32_t b = 0; b < 256; ++b) slice[0][b] = byte_step(b);
		for (int k = 1; k < 8; ++k)
			for (uint32_t b = 0; b < 256; ++b) slice[k][b] = (slice[k - 1][b] >> 8) ^ slice[0][slice[k - 1][b] & 0xffu];
		mul_tables_byte(xpow8(kBlock), merge);
		mul_tables_byte(xpow8(kShort), merge_s);
	}
};

// Built when the library is loaded (as the reference's static hw_available,
// crc32c.cpp:344): no initialisation guard on the per-call path.
const HostTables g_tables;


inline uint32_t apply_merge(const uint32_t (&m)[4][256], uint32_t r) {
	return m[0][r & 0xff] ^ m[1][(r >> 8) & 0xff] ^ m[2][(r >> 16) & 0xff] ^ m[3][r >> 24];
}

inline uint64_t load64(const uint8_t* p) {
	uint64_t v;
	memcpy(&v, p, 8);
	return v;
}

uint32_t raw_sliced(const HostTables& t, uint32_t s, const uint8_t* p, size_t n) {
	for (; n >= 8; n -= 8, p += 8) {
		const uint64_t v = load64(p) ^ s;
		s = t.slice[7][v & 0xff] ^ t.slice[6][(v >> 8) & 0xff] ^ t.slice[5][(v >> 16) & 0xff] ^
		    t.slice[4][(v >> 24) & 0xff] ^ t.slice[3][(v >> 32) & 0xff] ^ t.slice[2][(v >> 40) & 0xff] ^
		    t.slice[1][(v >> 48) & 0xff] ^ t.slice[0][v >> 56];
	}
	for (; n; --n) s = (s >> 8) ^ t.slice[0][(s ^ *p++) & 0xff];
	return s;
}

#if defined(__x86_64__)
// Short buffers (< 64 B: keys, small values, packet headers): no alignment
// prologue (x86 loads need none), 8-byte steps, then 4/2/1-byte steps.
__attribute__((target("sse4.2"))) inline uint32_t raw_sse42_short(uint32_t s, const uint8_t* p, size_t n) {
	uint64_t s0 = s;
	for (; n >= 8; n -= 8, p += 8) s0 = _mm_crc32_u64(s0, load64(p));
	uint32_t r = (uint32_t)s0;
	if (n & 4) {
		uint32_t v;
		memcpy(&v, p, 4);
		r = _mm_crc32_u32(r, v);
		p += 4;
	}
	if (n & 2) {
		uint16_t v;
		memcpy(&v, p, 2);
		r = _mm_crc32_u16(r, v);
		p += 2;
	}
	if (n & 1) r = _mm_crc32_u8(r, *p);
	return r;
}

__attribute__((target("sse4.2"))) uint32_t raw_sse42(const HostTables& t, uint32_t s, const uint8_t* p, size_t n) {
	if (n < 64) return raw_sse42_short(s, p, n);
	while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
		s = _mm_crc32_u8(s, *p++);
		--n;
	}
	uint64_t s0 = s;
	while (n >= 3 * kBlock) {
		uint64_t s1 = 0, s2 = 0;
		const uint8_t* q = p;
		for (const uint8_t* end = p + kBlock; q < end; q += 8) {
			s0 = _mm_crc32_u64(s0, load64(q));
			s1 = _mm_crc32_u64(s1, load64(q + kBlock));
			s2 = _mm_crc32_u64(s2, load64(q + 2 * kBlock));
		}
		s0 = apply_merge(t.merge, apply_merge(t.merge, (uint32_t)s0) ^ (uint32_t)s1) ^ (uint32_t)s2;
		p += 3 * kBlock;
		n -= 3 * kBlock;
	}
	while (n >= 3 * kShort) {
		uint64_t s1 = 0, s2 = 0;
		const uint8_t* q = p;
		for (const uint8_t* end = p + kShort; q < end; q += 8) {
			s0 = _mm_crc32_u64(s0, load64(q));
			s1 = _mm_crc32_u64(s1, load64(q + kShort));
			s2 = _mm_crc32_u64(s2, load64(q + 2 * kShort));
		}
		s0 = apply_merge(t.merge_s, apply_merge(t.merge_s, (uint32_t)s0) ^ (uint32_t)s1) ^ (uint32_t)s2;
		p += 3 * kShort;
		n -= 3 * kShort;
	}
	return raw_sse42_short((uint32_t)s0, p, n);
}
#endif

}  // namespace
}  // namespace fdbcrc

// Dispatch once, at load time (GNU ifunc): crc32c_append binds straight to the
// SSE4.2 or the sliced implementation, with no per-call test -- the reference
// tests its static hw_available on every call (crc32c.cpp:344-356).
namespace fdbcrc {
namespace {
int g_impl = 0;  // 1: sse4.2, 2: sliced (set by the resolver, before any constructor runs)

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t append_sse42(uint32_t crc, const uint8_t* input, size_t length) {
	if (length < 64) return ~raw_sse42_short(~crc, input, length);
	return ~raw_sse42(g_tables, ~crc, input, length);
}
#endif

uint32_t append_sliced(uint32_t crc, const uint8_t* input, size_t length) {
	return ~raw_sliced(g_tables, ~crc, input, length);
}

}  // namespace
}  // namespace fdbcrc

extern "C" {

typedef uint32_t (*crc32c_fn)(uint32_t, const uint8_t*, size_t);

// Runs while the dynamic linker processes relocations, before any constructor
// (sanitizer runtimes included): kept uninstrumented.
__attribute__((no_sanitize("address", "undefined"))) static crc32c_fn resolve_crc32c_append(void) {
	bool sse = false;
#if defined(__x86_64__)
	__builtin_cpu_init();
	sse = __builtin_cpu_supports("sse4.2");
#endif
	const char* force = getenv("FDB_CRC32C_FORCE_SOFTWARE");
	if (force && *force && *force != '0') sse = false;
	fdbcrc::g_impl = sse ? 1 : 2;
#if defined(__x86_64__)
	if (sse) return fdbcrc::append_sse42;
#endif
	return fdbcrc::append_sliced;
}

uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length) __attribute__((ifunc("resolve_crc32c_append")));

const char* crc32c_host_impl(void) { return fdbcrc::g_impl == 1 ? "sse4.2" : "sliced"; }

uint32_t crc32c_shift(uint32_t reg, uint64_t nbytes) { return fdbcrc::gf2_mul(reg, fdbcrc::xpow8(nbytes)); }

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return crc_b ^ crc32c_shift(crc_a, len_b); }

uint32_t crc32c_append_zeros(uint32_t crc, uint64_t nzeros) { return ~crc32c_shift(~crc, nzeros); }

}  // extern "C"
