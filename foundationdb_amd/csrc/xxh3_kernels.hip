// Batched XXH3-64 (xxHash v0.8.0 XXH3_64bits / XXH3_64bits_withSeed) on
// MI355X (gfx950).  Bit-identical to flow/include/flow/xxhash.h:3800-3837 for
// every (bytes, length, seed).  Callers: SQLite page checksums
// (fdbserver/kvstore/KeyValueStoreSQLite.cpp:112,138), DiskQueue V2 pages
// (fdbserver/kvstore/DiskQueue.cpp:1086-1088), Redwood page encodings
// (fdbserver/kvstore/IPager.h:300-361), FlowTransport packets
// (fdbrpc/FlowTransport.cpp:1346,2043).
//
// Long inputs (> 240 B), xxhash.h:3641-3718: one wave per buffer.  A 1 KiB
// block is 16 stripes x 64 B; lane m loads the 16 B at 16m (one coalesced
// 1 KiB load per block), i.e. stripe s = m/4, accumulator pair k = m%4, and
// computes that stripe's contributions to accumulators 2k and 2k+1
// (accumulate_512 swaps adjacent lanes, so the pair is closed).  The 16
// lanes of a pair sum their contributions (DPP row rotates + permlane swaps),
// lanes 0..3 then hold acc[2k], acc[2k+1] and apply the element-wise
// scramble after every full block.  The final partial block has at most 15
// stripes, so lanes 60..63 take the last stripe (at len-64, secret+121).
// Short inputs (<= 240 B), xxhash.h:2734-2951: one lane per buffer.
// No lookup tables: no LDS, occupancy bounded by VGPRs only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xxh3_device.h"

namespace fdbxxh {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;

// The default secret as 24 little-endian words (xxhash.h:2500-2511).
__constant__ uint64_t kSec[24] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
    0xcb00c391bb52283cull, 0xa32e531b8b65d088ull, 0x4ef90da297486471ull, 0xd8acdea946ef1938ull,
    0x3f349ce33f76faa8ull, 0x1d4f0bc7c7bbdcf9ull, 0x3159b4cd4be0518aull, 0x647378d9c97e9fc8ull,
    0xc3ebd33483acc5eaull, 0xeb6313faffa081c5ull, 0x49daf0b751dd0d17ull, 0x9e68d429265516d3ull,
    0xfca1477d58be162bull, 0xce31d07ad1b8f88full, 0x280416958f3acb45ull, 0x7e404bbbcafbd7afull,
};

// Word j of the secret for `seed` (custom secret, xxhash.h:3550-3566; the
// seed-0 secret is the default one).
__device__ __forceinline__ uint64_t sec_word(int j, uint64_t seed) {
	const uint64_t w = kSec[j];
	return (j & 1) ? w - seed : w + seed;
}
// Secret bytes [8j + r, 8j + r + 8), 0 < r < 8.
__device__ __forceinline__ uint64_t sec_at(int j, int r, uint64_t seed) {
	return (sec_word(j, seed) >> (8 * r)) | (sec_word(j + 1, seed) << (64 - 8 * r));
}
// Default-secret bytes at any offset (short paths never use a custom secret).
__device__ __forceinline__ uint64_t ksec(int off) {
	const int j = off >> 3, r = off & 7;
	return r ? (kSec[j] >> (8 * r)) | (kSec[j + 1] << (64 - 8 * r)) : kSec[j];
}
__device__ __forceinline__ uint32_t ksec32(int off) { return (uint32_t)ksec(off); }

__device__ __forceinline__ uint64_t mulfold(uint64_t a, uint64_t b) { return a * b ^ __umul64hi(a, b); }
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xxh64_aval(uint64_t h) {
	h ^= h >> 33;
	h *= P64_2;
	h ^= h >> 29;
	h *= P64_3;
	return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t xxh3_aval(uint64_t h) {
	h ^= h >> 37;
	h *= 0x165667919E3779F9ull;
	return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {
	h ^= rotl64(h, 49) ^ rotl64(h, 24);
	h *= 0x9FB21C651E98DF25ull;
	h ^= (h >> 35) + len;
	h *= 0x9FB21C651E98DF25ull;
	return h ^ (h >> 28);
}

typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef __attribute__((address_space(1))) const u64x2 g_u64x2;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

// Little-endian 8-byte read at any address: aligned 8-byte words only (a word
// holding a wanted byte never crosses a page, so nothing past the buffer's
// last 8-byte word is touched).
__device__ __forceinline__ uint64_t ldu64(uint64_t p) {
	const uint64_t a = p & ~uint64_t(7);
	const int sh = (int)(p & 7);
	const uint64_t lo = *((g_u64*)a);
	if (!sh) return lo;
	const uint64_t hi = *((g_u64*)(a + 8));
	return (lo >> (8 * sh)) | (hi << (64 - 8 * sh));
}
__device__ __forceinline__ uint32_t ldu32(uint64_t p) {
	// bytes p..p+3 lie in at most two aligned words; read only what is needed
	const uint64_t a = p & ~uint64_t(3);
	const int sh = (int)(p & 3);
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	const uint32_t lo = *((g_u32*)a);
	if (!sh) return lo;
	const uint32_t hi = *((g_u32*)(a + 4));
	return (lo >> (8 * sh)) | (hi << (32 - 8 * sh));
}
__device__ __forceinline__ uint32_t ldu8(uint64_t p) { return *((g_u8*)p); }

// ---------------------------------------------------------------------------
// Short inputs, one lane per buffer (xxhash.h:2734-2951, default secret).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix16(uint64_t p, int soff, uint64_t seed) {
	return mulfold(ldu64(p) ^ (ksec(soff) + seed), ldu64(p + 8) ^ (ksec(soff + 8) - seed));
}

__device__ uint64_t xxh3_short(uint64_t p, uint64_t len, uint64_t seed) {
	if (len <= 16) {
		if (len > 8) {
			const uint64_t f1 = (ksec(24) ^ ksec(32)) + seed, f2 = (ksec(40) ^ ksec(48)) - seed;
			const uint64_t lo = ldu64(p) ^ f1, hi = ldu64(p + len - 8) ^ f2;
			return xxh3_aval(len + __builtin_bswap64(lo) + hi + mulfold(lo, hi));
		}
		if (len >= 4) {
			const uint64_t s2 = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
			const uint32_t i1 = ldu32(p), i2 = ldu32(p + len - 4);
			const uint64_t flip = (ksec(8) ^ ksec(16)) - s2;
			return rrmxmx(((uint64_t)i2 + ((uint64_t)i1 << 32)) ^ flip, len);
		}
		if (len) {
			const uint32_t c1 = ldu8(p), c2 = ldu8(p + (len >> 1)), c3 = ldu8(p + len - 1);
			const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
			return xxh64_aval((uint64_t)comb ^ ((uint64_t)(ksec32(0) ^ ksec32(4)) + seed));
		}
		return xxh64_aval(seed ^ (ksec(56) ^ ksec(64)));
	}
	uint64_t acc = len * P64_1;
	if (len <= 128) {
		const int pairs = (int)((len - 1) >> 5);  // 0..3 extra pairs beyond the first
		for (int i = pairs; i >= 1; --i) {
			acc += mix16(p + 16 * i, 32 * i, seed);
			acc += mix16(p + len - 16 * (i + 1), 32 * i + 16, seed);
		}
		acc += mix16(p, 0, seed);
		acc += mix16(p + len - 16, 16, seed);
		return xxh3_aval(acc);
	}
	const int rounds = (int)len / 16;
	for (int i = 0; i < 8; ++i) acc += mix16(p + 16 * i, 16 * i, seed);
	acc = xxh3_aval(acc);
	for (int i = 8; i < rounds; ++i) acc += mix16(p + 16 * i, 16 * (i - 8) + 3, seed);
	acc += mix16(p + len - 16, 136 - 17, seed);
	return xxh3_aval(acc);
}

// ---------------------------------------------------------------------------
// Long inputs, one wave per buffer.
// ---------------------------------------------------------------------------
// Sum over the 16 lanes m' == m (mod 4) (the stripes of one pair): DPP row
// rotates by 4 and 8, then the permlane16/32 swaps add the four rows.
template <int CTRL>
__device__ __forceinline__ void add_dpp(uint32_t& lo, uint32_t& hi) {
	const uint32_t l2 = __builtin_amdgcn_update_dpp(0u, lo, CTRL, 0xF, 0xF, false);
	const uint32_t h2 = __builtin_amdgcn_update_dpp(0u, hi, CTRL, 0xF, 0xF, false);
	const uint64_t s = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2);
	lo = (uint32_t)s;
	hi = (uint32_t)(s >> 32);
}

__device__ __forceinline__ uint64_t pair_sum(uint64_t v) {
	uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
	add_dpp<0x124>(lo, hi);  // row_ror:4
	add_dpp<0x128>(lo, hi);  // row_ror:8
	{
		const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
		const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
		const uint64_t s = (((uint64_t)b[0] << 32) | a[0]) + (((uint64_t)b[1] << 32) | a[1]);
		lo = (uint32_t)s;
		hi = (uint32_t)(s >> 32);
	}
	{
		const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
		const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
		const uint64_t s = (((uint64_t)b[0] << 32) | a[0]) + (((uint64_t)b[1] << 32) | a[1]);
		lo = (uint32_t)s;
		hi = (uint32_t)(s >> 32);
	}
	return ((uint64_t)hi << 32) | lo;
}

// Per-lane secret words of one seed.
struct Keys {
	uint64_t k0, k1;   // normal stripe: secret + 8s + 16k, +8
	uint64_t l0, l1;   // last stripe (lanes 60..63): secret + 121 + 16k, +8
	uint64_t c0, c1;   // scramble (lanes 0..3): secret + 128 + 16k, +8
	uint64_t g0, g1;   // merge (lanes 0..3): secret + 11 + 16k, +8
};
__device__ __forceinline__ Keys make_keys(int lane, uint64_t seed) {
	const int s = lane >> 2, k = lane & 3;
	Keys K;
	K.k0 = sec_word(s + 2 * k, seed);
	K.k1 = sec_word(s + 2 * k + 1, seed);
	K.l0 = sec_at(15 + 2 * k, 1, seed);
	K.l1 = sec_at(16 + 2 * k, 1, seed);
	K.c0 = sec_word(16 + 2 * k, seed);
	K.c1 = sec_word(17 + 2 * k, seed);
	K.g0 = sec_at(1 + 2 * k, 3, seed);
	K.g1 = sec_at(2 + 2 * k, 3, seed);
	return K;
}

struct Acc {
	uint64_t a0, a1;  // lanes 0..3: acc[2k], acc[2k+1]
};
__device__ __forceinline__ Acc acc_init(int lane) {
	const int k = lane & 3;
	Acc A;
	A.a0 = k == 0 ? P32_3 : (k == 1 ? P64_2 : (k == 2 ? P64_4 : P64_5));
	A.a1 = k == 0 ? P64_1 : (k == 1 ? P64_3 : (k == 2 ? P32_2 : P32_1));
	return A;
}

// One block's contributions: v0/v1 = the lane's two data words, key words
// per lane (normal or last-stripe), `on` = lane takes part.
__device__ __forceinline__ void block_step(Acc& A, uint64_t v0, uint64_t v1, uint64_t key0, uint64_t key1, bool on) {
	const uint64_t x0 = v0 ^ key0, x1 = v1 ^ key1;
	uint64_t d0 = v1 + (uint64_t)(uint32_t)x0 * (x0 >> 32);
	uint64_t d1 = v0 + (uint64_t)(uint32_t)x1 * (x1 >> 32);
	d0 = on ? d0 : 0;
	d1 = on ? d1 : 0;
	A.a0 += pair_sum(d0);
	A.a1 += pair_sum(d1);
}
__device__ __forceinline__ void scramble(Acc& A, const Keys& K) {
	A.a0 = ((A.a0 ^ (A.a0 >> 47)) ^ K.c0) * P32_1;
	A.a1 = ((A.a1 ^ (A.a1 >> 47)) ^ K.c1) * P32_1;
}
// mergeAccs (xxhash.h:3678-3700), result valid in every lane
__device__ __forceinline__ uint64_t merge(const Acc& A, const Keys& K, uint64_t len, int lane) {
	uint64_t r = (lane < 4) ? mulfold(A.a0 ^ K.g0, A.a1 ^ K.g1) : 0;
	uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
	add_dpp<0xB1>(lo, hi);  // quad_perm [1,0,3,2]
	add_dpp<0x4E>(lo, hi);  // quad_perm [2,3,0,1]: lane 0 = sum of lanes 0..3
	const uint64_t tot = ((uint64_t)__builtin_amdgcn_readlane(hi, 0) << 32) | (uint32_t)__builtin_amdgcn_readlane(lo, 0);
	return xxh3_aval(len * P64_1 + tot);
}

// A unit: up to 4 consecutive blocks of one buffer, loaded together.
struct Unit {
	uint64_t p, len, seed, buf;
	uint64_t b0;   // first block index
	int n;         // blocks in the unit (0: none)
	bool first, fin;
};
struct Data {
	uint64_t v[4][2];
};

template <bool ALIGNED>
__device__ __forceinline__ void load_unit(Data& D, const Unit& u, int lane) {
	const uint64_t nfull = (u.len - 1) >> 10;
	const uint64_t ns = ((u.len - 1) - (nfull << 10)) >> 6;
#pragma unroll
	for (int j = 0; j < 4; ++j) {
		D.v[j][0] = D.v[j][1] = 0;
		if (j < u.n) {
			const uint64_t blk = u.b0 + j;
			const bool fin = blk == nfull;
			uint64_t q = u.p + (blk << 10) + 16 * lane;
			bool on = true;
			bool aligned = ALIGNED;
			if (fin) {
				if (lane >= 60) {
					q = u.p + u.len - 64 + 16 * (lane - 60);
					aligned = false;
				} else {
					on = (uint64_t)lane < 4 * ns;
				}
			}
			if (on) {
				if (aligned) {
					const u64x2 w = __builtin_nontemporal_load((g_u64x2*)q);
					D.v[j][0] = w[0];
					D.v[j][1] = w[1];
				} else {
					D.v[j][0] = ldu64(q);
					D.v[j][1] = ldu64(q + 8);
				}
			}
		}
	}
}

__device__ __forceinline__ void compute_unit(Acc& A, const Keys& K, const Data& D, const Unit& u, int lane,
                                             uint64_t* __restrict__ out) {
	const uint64_t nfull = (u.len - 1) >> 10;
	const uint64_t ns = ((u.len - 1) - (nfull << 10)) >> 6;
	if (u.first) A = acc_init(lane);
#pragma unroll
	for (int j = 0; j < 4; ++j) {
		if (j < u.n) {
			const uint64_t blk = u.b0 + j;
			if (blk < nfull) {
				block_step(A, D.v[j][0], D.v[j][1], K.k0, K.k1, true);
				scramble(A, K);
			} else {
				const bool last = lane >= 60;
				block_step(A, D.v[j][0], D.v[j][1], last ? K.l0 : K.k0, last ? K.l1 : K.k1,
				           last || (uint64_t)lane < 4 * ns);
			}
		}
	}
	if (u.fin) {
		const uint64_t h = merge(A, K, u.len, lane);
		if (lane == 0) out[u.buf] = h;
	}
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_xxh3(XxhParams P) {
	const int lane = threadIdx.x & 63;
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t nwave = (uint64_t)gridDim.x * wpb;
	const uint64_t w = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const bool fixed = P.offsets == nullptr;
	// this wave's buffers [begin, end)
	uint64_t begin, end;
	if (fixed) {
		const uint64_t per = (P.count + nwave - 1) / nwave;
		begin = w * per;
		end = begin + per < P.count ? begin + per : P.count;
	} else {
		begin = P.wave_first[w];
		end = P.wave_first[w + 1];
		end = end < P.count ? end : P.count;
	}
	if (begin >= end) return;
	const uint64_t base = reinterpret_cast<uint64_t>(P.base);
	auto off_of = [&](uint64_t i) -> uint64_t { return fixed ? i * P.stride : P.offsets[i]; };
	auto len_of = [&](uint64_t i) -> uint64_t { return fixed ? P.length : P.lengths[i]; };
	auto seed_of = [&](uint64_t i) -> uint64_t { return P.seeds ? P.seeds[i] : P.seed; };

	// ---- short buffers: one lane each, 64 per pass
	for (uint64_t b0 = begin; b0 < end; b0 += 64) {
		const uint64_t i = b0 + lane;
		if (i < end) {
			const uint64_t len = len_of(i);
			if (len <= 240) P.out[i] = xxh3_short(base + off_of(i), len, seed_of(i));
		}
	}

	// ---- long buffers: one wave each, units of up to 4 blocks, next unit in flight
	uint64_t gi = begin;       // next buffer to start
	uint64_t gblk = 0, gtot = 0;  // next block of the current buffer, its block count
	Unit g{};                  // current buffer (uniform)
	auto next_unit = [&](Unit& u) {
		u.n = 0;
		if (gblk == gtot) {  // find the next long buffer
			for (;;) {
				if (gi >= end) return;
				if (len_of(gi) > 240) break;
				++gi;
			}
			g.len = len_of(gi);
			g.p = base + off_of(gi);
			g.seed = seed_of(gi);
			g.buf = gi;
			++gi;
			gblk = 0;
			gtot = ((g.len - 1) >> 10) + 1;
		}
		u = g;
		u.b0 = gblk;
		u.n = gtot - gblk < 4 ? (int)(gtot - gblk) : 4;
		u.first = gblk == 0;
		gblk += u.n;
		u.fin = gblk == gtot;
	};
	Unit cur, nxt;
	Data dc, dn;
	Acc A{0, 0};
	Keys K{};
	uint64_t kseed = ~uint64_t(0);
	bool have_keys = false;
	next_unit(cur);
	if (cur.n) load_unit<ALIGNED>(dc, cur, lane);
	while (cur.n) {
		next_unit(nxt);
		if (nxt.n) load_unit<ALIGNED>(dn, nxt, lane);
		__builtin_amdgcn_sched_barrier(0);
		if (!have_keys || cur.seed != kseed) {
			K = make_keys(lane, cur.seed);
			kseed = cur.seed;
			have_keys = true;
		}
		compute_unit(A, K, dc, cur, lane, P.out);
		__builtin_amdgcn_sched_barrier(0);
		cur = nxt;
		dc = dn;
	}
}

// ---------------------------------------------------------------------------
// Fixed-length long buffers (> 240 B): four buffers per wave in lockstep, one
// per 16-lane row.  Lane (g, k) = (l/4, l%4) of row r takes stripes
// g, g+4, g+8, g+12 of every block for accumulator pair k: four contributions
// add up in registers, then two DPP row rotates close the 4-lane sum (no
// cross-row traffic).  A load instruction covers 256 contiguous bytes per
// row.  The block stream of the wave's buffer groups runs two blocks per
// unit, the next unit's loads in flight.
// ---------------------------------------------------------------------------
struct RowKeys {
	uint64_t k0[4], k1[4];  // stripe g + 4i: secret + 8(g + 4i) + 16k, +8
	uint64_t l0, l1;        // last stripe: secret + 121 + 16k, +8
	uint64_t c0, c1;        // scramble: secret + 128 + 16k, +8
	uint64_t g0, g1;        // merge: secret + 11 + 16k, +8
};
__device__ __forceinline__ RowKeys row_keys(int lane, uint64_t seed) {
	const int l = lane & 15, k = l & 3, g = l >> 2;
	RowKeys K;
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		K.k0[i] = sec_word(g + 4 * i + 2 * k, seed);
		K.k1[i] = sec_word(g + 4 * i + 2 * k + 1, seed);
	}
	K.l0 = sec_at(15 + 2 * k, 1, seed);
	K.l1 = sec_at(16 + 2 * k, 1, seed);
	K.c0 = sec_word(16 + 2 * k, seed);
	K.c1 = sec_word(17 + 2 * k, seed);
	K.g0 = sec_at(1 + 2 * k, 3, seed);
	K.g1 = sec_at(2 + 2 * k, 3, seed);
	return K;
}

struct RowData {
	uint64_t v[4][2];
};

// A16: base and stride 16-byte aligned (dwordx4 loads), else 8-byte aligned
// (two dwordx2 loads per 16 B).
#ifndef FDBXXH_G3W0
#define FDBXXH_G3W0 42
#define FDBXXH_G3W1 37
#endif
constexpr uint64_t kRowsG3W0 = FDBXXH_G3W0, kRowsG3W1 = FDBXXH_G3W1;  // k_xxh3_rows, three generations (32nds)
#ifndef FDBXXH_ROWS_XE
#define FDBXXH_ROWS_XE 33
#define FDBXXH_ROWS_XO 31
#endif
constexpr uint64_t kRowsXE = FDBXXH_ROWS_XE, kRowsXO = FDBXXH_ROWS_XO;  // k_xxh3_rows, even / odd XCDs (32nds)
#ifdef FDBXXH_TIMES
// development: per-wave timestamps of the row kernels (start, rows done, end; s_memrealtime, 100 MHz)
__device__ uint64_t g_vt[16384][4];
#endif
template <bool SEEDS, bool LIST = false, bool A16 = true>
__global__ __launch_bounds__(256) void k_xxh3_rows(XxhParams P) {
	if (LIST) P.count = *P.d_count;
	const int lane = threadIdx.x & 63;
	const int r = lane >> 4, l = lane & 15, k = l & 3, g = l >> 2;
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t nwave = (uint64_t)gridDim.x * wpb;
	const uint64_t w = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef FDBXXH_TIMES
	const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
	// Static page ranges weighted by dispatch generation: with ngen workgroups
	// per CU, the waves of the first-dispatched ones win the SIMDs' issue
	// arbitration (per-wave timestamps, 1 Mi 4 KiB pages, three generations:
	// 573 / 613 / 669 us median for equal ranges), so their ranges are longer
	// -- 42 : 37 : 32 (633 / 619 / 614 us; 37 : 35 : 32 left 584 / 612 / 642;
	// two generations: 42 : 32) -- and the generations end together.
	// Within a generation, workgroup b runs on XCD b % 8 and the odd XCDs
	// stream ~6 % slower (as in k_pages4k, crc32c_device.h: xcd_range): an even
	// workgroup's waves take kRowsXE / kRowsXO of an odd one's.  Same box,
	// bench protocol: xxh3-pages4k 674 -> 668 us, SQLite's list 499 -> 495 us;
	// the 8-byte-aligned form (DiskQueue's 4092 B at +4) ran 557 -> 570 us with
	// them, so it keeps equal weights.
	const uint64_t kXE = A16 ? kRowsXE : 32, kXO = A16 ? kRowsXO : 32;
	uint64_t begin, end;
	if (P.ngen == 2 || P.ngen == 3) {
		const uint64_t wpg = nwave / P.ngen;
		const uint64_t gsel = w / wpg;
		const uint64_t W0 = P.ngen == 3 ? kRowsG3W0 : 42, W1 = P.ngen == 3 ? kRowsG3W1 : 32, W2 = 32;
		const uint64_t sumW = P.ngen == 3 ? W0 + W1 + W2 : W0 + W1;
		const uint64_t bpg = wpg / wpb, ne = (bpg + 1) / 2, no = bpg / 2;  // workgroups per generation, even / odd
		const uint64_t den = sumW * wpb * (ne * kXE + no * kXO);
		const uint64_t unit = (P.count * 1024 + den - 1) / den;  // pages per wave at weight 32 x 32
		auto per_of = [&](uint64_t Wg, uint64_t Wx) { return ((unit * Wg * Wx + 1023) / 1024 + 3) & ~uint64_t(3); };
		auto gen_pages = [&](uint64_t Wg) { return wpb * (ne * per_of(Wg, kXE) + no * per_of(Wg, kXO)); };
		const uint64_t Wg = gsel == 0 ? W0 : (gsel == 1 ? W1 : W2);
		const uint64_t start = gsel == 0 ? 0 : (gsel == 1 ? gen_pages(W0) : gen_pages(W0) + gen_pages(W1));
		const uint64_t wi = w - gsel * wpg, bi = wi / wpb;
		const uint64_t pe = per_of(Wg, kXE), po = per_of(Wg, kXO);
		begin = start + wpb * (((bi + 1) / 2) * pe + (bi / 2) * po) + (wi % wpb) * ((bi & 1) ? po : pe);
		const uint64_t pg = (bi & 1) ? po : pe;
		end = begin + pg < P.count ? begin + pg : P.count;
	} else {
		uint64_t per = (P.count + nwave - 1) / nwave;
		per = (per + 3) & ~uint64_t(3);
		begin = w * per;
		end = begin + per < P.count ? begin + per : P.count;
	}
	if (begin >= end) return;
	const uint64_t len = P.length;
	const uint64_t nfull = (len - 1) >> 10;
	const uint64_t ns = ((len - 1) - (nfull << 10)) >> 6;
	const uint64_t nblk = nfull + 1;
	const uint64_t ngroups = (end - begin + 3) >> 2;
	const uint64_t E = ngroups * nblk;
	const uint64_t base = reinterpret_cast<uint64_t>(P.base);
	auto page_of = [&](uint64_t q) -> uint64_t {  // this lane's row's buffer in group q (clamped)
		const uint64_t i = begin + 4 * q + r;
		return i < end ? i : end - 1;
	};
	// LIST: the four page numbers of a group as scalar loads (lgkmcnt, off the
	// vmcnt queue of the data prefetch), selected by row
	auto addr_of = [&](uint64_t q) -> uint64_t {
		if (!LIST) return base + page_of(q) * P.stride;
		const uint64_t i0 = begin + 4 * q;
		const uint64_t c = end - 1;
		const uint32_t p0 = P.idx[i0 < end ? i0 : c], p1 = P.idx[i0 + 1 < end ? i0 + 1 : c];
		const uint32_t p2 = P.idx[i0 + 2 < end ? i0 + 2 : c], p3 = P.idx[i0 + 3 < end ? i0 + 3 : c];
		const uint32_t pr = r == 0 ? p0 : (r == 1 ? p1 : (r == 2 ? p2 : p3));
		return base + (uint64_t)pr * P.stride;
	};
	// stream positions (group, block) of the next load and the next compute
	uint64_t lq = 0, lb = 0, cq = 0, cb = 0;
	auto load = [&](RowData& D) {
#pragma unroll
		for (int i = 0; i < 4; ++i) D.v[i][0] = D.v[i][1] = 0;
		if (lq >= ngroups) return;
		const uint64_t q = lq, b = lb;
		if (++lb == nblk) {
			lb = 0;
			++lq;
		}
		const uint64_t p = addr_of(q);
		const bool fin = b == nfull;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint64_t s = g + 4 * i;
			if (fin && s == 15) {  // last stripe, any alignment
				const uint64_t a = p + len - 64 + 16 * k;
				D.v[i][0] = ldu64(a);
				D.v[i][1] = ldu64(a + 8);
			} else if (!fin || s < ns) {
				const uint64_t a = p + (b << 10) + 64 * s + 16 * k;
				if (A16) {
					const u64x2 x = __builtin_nontemporal_load((g_u64x2*)a);
					D.v[i][0] = x[0];
					D.v[i][1] = x[1];
				} else {
#ifndef FDBXXH_ROWS_X2
					// one unaligned dwordx4 (gfx950: full rate at a 4- or 8-byte
					// aligned address, tools/membench3.hip), not two dwordx2
					typedef uint64_t u64x2r __attribute__((ext_vector_type(2), aligned(4)));
					typedef __attribute__((address_space(1))) const u64x2r g_u64x2r;
					const u64x2r x = __builtin_nontemporal_load((g_u64x2r*)a);
					D.v[i][0] = x[0];
					D.v[i][1] = x[1];
#else
					D.v[i][0] = __builtin_nontemporal_load((g_u64*)a);
					D.v[i][1] = __builtin_nontemporal_load((g_u64*)(a + 8));
#endif
				}
			}
		}
	};
	RowKeys K = row_keys(lane, P.seed);
	uint64_t a0 = 0, a1 = 0;
	auto compute = [&](const RowData& D) {
		if (cq >= ngroups) return;
		const uint64_t q = cq, b = cb;
		if (++cb == nblk) {
			cb = 0;
			++cq;
		}
		const bool fin = b == nfull;
		if (b == 0) {
			if (SEEDS) K = row_keys(lane, P.seeds[page_of(q)]);
			a0 = k == 0 ? P32_3 : (k == 1 ? P64_2 : (k == 2 ? P64_4 : P64_5));
			a1 = k == 0 ? P64_1 : (k == 1 ? P64_3 : (k == 2 ? P32_2 : P32_1));
		}
		uint64_t d0 = 0, d1 = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint64_t s = g + 4 * i;
			const bool last = fin && s == 15;
			const bool on = !fin || s < ns || last;
			const uint64_t x0 = D.v[i][0] ^ (last ? K.l0 : K.k0[i]);
			const uint64_t x1 = D.v[i][1] ^ (last ? K.l1 : K.k1[i]);
			const uint64_t c0 = D.v[i][1] + (uint64_t)(uint32_t)x0 * (x0 >> 32);
			const uint64_t c1 = D.v[i][0] + (uint64_t)(uint32_t)x1 * (x1 >> 32);
			d0 += on ? c0 : 0;
			d1 += on ? c1 : 0;
		}
		// sum over g (lanes l, l+4, l+8, l+12 of the row)
		uint32_t lo0 = (uint32_t)d0, hi0 = (uint32_t)(d0 >> 32), lo1 = (uint32_t)d1, hi1 = (uint32_t)(d1 >> 32);
		add_dpp<0x124>(lo0, hi0);
		add_dpp<0x124>(lo1, hi1);
		add_dpp<0x128>(lo0, hi0);
		add_dpp<0x128>(lo1, hi1);
		a0 += ((uint64_t)hi0 << 32) | lo0;
		a1 += ((uint64_t)hi1 << 32) | lo1;
		if (!fin) {
			a0 = ((a0 ^ (a0 >> 47)) ^ K.c0) * P32_1;
			a1 = ((a1 ^ (a1 >> 47)) ^ K.c1) * P32_1;
		} else {
			// merge: lanes 0..3 of the row (g = 0) hold the 8 accumulators
			const uint64_t m = mulfold(a0 ^ K.g0, a1 ^ K.g1);
			uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
			add_dpp<0xB1>(lo, hi);
			add_dpp<0x4E>(lo, hi);
			const uint64_t h = xxh3_aval(len * P64_1 + (((uint64_t)hi << 32) | lo));
			const uint64_t i = begin + 4 * q + r;
			if (l == 0 && i < end) P.out[i] = h;
		}
	};
	RowData c0, c1, n0, n1;
	load(c0);
	load(c1);
	for (uint64_t e = 0; e < E; e += 2) {
		load(n0);
		load(n1);
		__builtin_amdgcn_sched_barrier(0);
		compute(c0);
		compute(c1);
		__builtin_amdgcn_sched_barrier(0);
		c0 = n0;
		c1 = n1;
	}
#ifdef FDBXXH_TIMES
	if (lane == 0 && w < 16384) {
		g_vt[w][0] = rt0;
		g_vt[w][1] = rt0;
		g_vt[w][2] = __builtin_amdgcn_s_memrealtime();
		g_vt[w][3] = end - begin;
	}
#endif
}

// ---------------------------------------------------------------------------
// Variable-length batches (packets, chained staging ranges): the row layout of
// k_xxh3_rows, each 16-lane row walking its own sequence of buffers.  The
// planner gives the wave whole buffers balanced by bytes; short ones (<= 240 B)
// go last, one lane each.  The long ones are handed to the rows dynamically:
// whenever a row has loaded its buffer's last block, it takes the next long
// buffer of a 64-buffer POOL (lengths/offsets in lanes, a uniform bitmask of
// the unclaimed long buffers; picks are v_readlane), so the four rows stay busy
// until the wave's range is exhausted whatever the lengths.  Every data load is
// unconditional: a row without work reads the planner's workspace (1 KiB,
// discarded), and lanes whose stripe is unused in a final block read the last
// 64 bytes (the last-stripe lanes' line).  Offsets are arbitrary: the
// `dwordx4` loads are unaligned (gfx950 runs with unaligned global access
// enabled).  A pool refill waits for the loads in flight: once per 64 buffers.
// ---------------------------------------------------------------------------
typedef uint64_t u64x2u __attribute__((ext_vector_type(2), aligned(1)));
typedef __attribute__((address_space(1))) const u64x2u g_u64x2u;
typedef __attribute__((address_space(1))) const uint32_t g_u32a;

// xxh3_short (17-240 B, xxhash.h:2847-2951) for one lane's buffer in two
// halves, so that a pass issues every data load it has (these and the lane
// quads') before it waits for any: the 17-240 B forms read up to sixteen
// 16-byte chunks (unaligned loads, all inside the buffer; unused chunks
// re-read its first 16 bytes) and add the used ones' mix16 terms (the sums are
// order-free).  Chunks no lane of the wave uses are not loaded.  `on` lanes
// only: the others pass a readable dummy.
struct ShortLd {
	u64x2u x[16];
};
__device__ __forceinline__ void short_load(ShortLd& S, uint64_t p, uint64_t len, bool on) {
	const bool big = len > 128;
	const int pairs = (int)((len - 1) >> 5);  // 17-128 B: 0..3 extra pairs
	const int rounds = (int)len >> 4;         // 129-240 B: 8..15 chunks
	const bool anybig = __ballot(on && big) != 0;
	const bool need1 = __ballot(on && !big && pairs >= 1) != 0, need2 = __ballot(on && !big && pairs >= 2) != 0,
	           need3 = __ballot(on && !big && pairs >= 3) != 0;
#pragma unroll
	for (int k = 0; k < 16; ++k) {
		const int q = k & 3;
		const bool used = anybig || (k < 8 && (q == 0 || (q == 1 && need1) || (q == 2 && need2) || (q == 3 && need3)));
		if (!used) {
			S.x[k] = u64x2u{0, 0};
			continue;
		}
		uint64_t a;
		if (k < 8) {  // big: chunk k; else front chunk k (< 4) or back chunk k - 4
			const uint64_t m = k < 4 ? p + 16 * k : p + len - 16 * (k - 3);
			a = big ? p + 16 * k : ((k & 3) <= pairs ? m : p);
		} else if (k < 15) {
			a = big && k < rounds ? p + 16 * k : p;
		} else {
			a = big ? p + len - 16 : p;
		}
		S.x[k] = __builtin_nontemporal_load((g_u64x2u*)a);
	}
}
__device__ __forceinline__ uint64_t short_fin(const ShortLd& S, uint64_t len, uint64_t seed) {
	const bool big = len > 128;
	const int pairs = (int)((len - 1) >> 5);
	const int rounds = (int)len >> 4;
	auto mix = [&](int k, int soff) __attribute__((always_inline)) {
		return mulfold(S.x[k][0] ^ (ksec(soff) + seed), S.x[k][1] ^ (ksec(soff + 8) - seed));
	};
	uint64_t acc = len * P64_1;
	if (!big) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint64_t t = mix(i, 32 * i) + mix(4 + i, 32 * i + 16);
			acc += i <= pairs ? t : 0;
		}
		return xxh3_aval(acc);
	}
#pragma unroll
	for (int i = 0; i < 8; ++i) acc += mix(i, 16 * i);
	acc = xxh3_aval(acc);
#pragma unroll
	for (int i = 8; i < 15; ++i) acc += i < rounds ? mix(i, 16 * (i - 8) + 3) : 0;
	acc += mix(15, 136 - 17);
	return xxh3_aval(acc);
}

// The same from a key table in LDS (uniform seed): key pair q = (secret at
// soff_q + 8 bytes) + seed, (secret at soff_q + 8, + 8) - seed, for the 16
// secret offsets the 17-240 B forms use -- 16j (j < 8), 16j + 3 (j < 7) and
// 119 -- so that slot q is chunk q on the 129-240 B path and chunks i, 4 + i
// take slots 2i, 2i + 1 on the 17-128 B one.  (As constants + seed the 32
// keys sat in SGPRs across the row loop and spilled.)
__device__ __forceinline__ void short_keys(uint64_t* keys, int t, uint64_t seed) {
	if (t < 32) {
		const int q = t >> 1, soff = q < 8 ? 16 * q : (q < 15 ? 16 * (q - 8) + 3 : 119);
		keys[t] = (t & 1) ? ksec(soff + 8) - seed : ksec(soff) + seed;
	}
}
// SEEDED: the table holds the seed-0 keys and each lane adds its own seed.
template <bool SEEDED>
__device__ __forceinline__ uint64_t short_fin_k(const ShortLd& S, uint64_t len, const uint64_t* keys, uint64_t seed) {
	typedef uint64_t u64x2k __attribute__((ext_vector_type(2)));
	const u64x2k* kp = reinterpret_cast<const u64x2k*>(keys);
	const bool big = len > 128;
	const int pairs = (int)((len - 1) >> 5);
	const int rounds = (int)len >> 4;
	auto mix = [&](int k, int q) __attribute__((always_inline)) {
		const u64x2k kk = kp[q];
		return mulfold(S.x[k][0] ^ (SEEDED ? kk[0] + seed : kk[0]), S.x[k][1] ^ (SEEDED ? kk[1] - seed : kk[1]));
	};
	uint64_t acc = len * P64_1;
	if (!big) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint64_t t = mix(i, 2 * i) + mix(4 + i, 2 * i + 1);
			acc += i <= pairs ? t : 0;
		}
		return xxh3_aval(acc);
	}
#pragma unroll
	for (int i = 0; i < 8; ++i) acc += mix(i, i);
	acc = xxh3_aval(acc);
#pragma unroll
	for (int i = 8; i < 15; ++i) acc += i < rounds ? mix(i, i) : 0;
	acc += mix(15, 15);
	return xxh3_aval(acc);
}

// XXH3 of 241 B - 1 KiB (one partial block, xxhash.h:3641-3718: no scramble)
// on a lane quad: lane k keeps accumulator pair k over the (len-1)/64 stripes
// and the last one, the four merge terms add over the quad.  Every data load
// is issued up front; stripes no lane of the wave has are not loaded.
// Secret word j (+-seed by parity, xxhash.h:3550-3566) from an LDS copy of
// the default secret, at a lane-dependent index (constants would sit in
// SGPRs across the whole kernel and spill).
__device__ __forceinline__ uint64_t lword(const uint64_t* ks, int j, uint64_t seed) {
	return (j & 1) ? ks[j] - seed : ks[j] + seed;
}
template <int S>
__device__ __forceinline__ void quad_stripe(uint64_t& a0, uint64_t& a1, const u64x2u& v, bool on, int k,
                                            const uint64_t* ks, uint64_t seed) {
	const uint64_t x0 = v[0] ^ lword(ks, S + 2 * k, seed), x1 = v[1] ^ lword(ks, S + 2 * k + 1, seed);
	a0 += on ? v[1] + (uint64_t)(uint32_t)x0 * (x0 >> 32) : 0;
	a1 += on ? v[0] + (uint64_t)(uint32_t)x1 * (x1 >> 32) : 0;
}
// secret bytes [8j + r, 8j + r + 8), 0 < r < 8
__device__ __forceinline__ uint64_t lat(const uint64_t* ks, int j, int r, uint64_t seed) {
	return (lword(ks, j, seed) >> (8 * r)) | (lword(ks, j + 1, seed) << (64 - 8 * r));
}
struct QuadLd {
	u64x2u v[15], vl;
};
__device__ __forceinline__ void quad_load(QuadLd& Q, uint64_t p, uint64_t len, int k) {
	const int ns = (int)((len - 1) >> 6);  // 3..15 full stripes
#pragma unroll
	for (int st = 0; st < 15; ++st) {
		if (st < 3 || __ballot(st < ns) != 0)
			Q.v[st] = __builtin_nontemporal_load((g_u64x2u*)(p + 64 * st + 16 * k));
		else
			Q.v[st] = u64x2u{0, 0};
	}
	Q.vl = __builtin_nontemporal_load((g_u64x2u*)(p + len - 64 + 16 * k));
}
__device__ __forceinline__ uint64_t quad_fin(const QuadLd& Q, uint64_t len, uint64_t seed, int k, const uint64_t* ks) {
	const int ns = (int)((len - 1) >> 6);
	uint64_t a0 = k == 0 ? P32_3 : (k == 1 ? P64_2 : (k == 2 ? P64_4 : P64_5));
	uint64_t a1 = k == 0 ? P64_1 : (k == 1 ? P64_3 : (k == 2 ? P32_2 : P32_1));
	quad_stripe<0>(a0, a1, Q.v[0], true, k, ks, seed);
	quad_stripe<1>(a0, a1, Q.v[1], true, k, ks, seed);
	quad_stripe<2>(a0, a1, Q.v[2], true, k, ks, seed);
	quad_stripe<3>(a0, a1, Q.v[3], 3 < ns, k, ks, seed);
	quad_stripe<4>(a0, a1, Q.v[4], 4 < ns, k, ks, seed);
	quad_stripe<5>(a0, a1, Q.v[5], 5 < ns, k, ks, seed);
	quad_stripe<6>(a0, a1, Q.v[6], 6 < ns, k, ks, seed);
	quad_stripe<7>(a0, a1, Q.v[7], 7 < ns, k, ks, seed);
	quad_stripe<8>(a0, a1, Q.v[8], 8 < ns, k, ks, seed);
	quad_stripe<9>(a0, a1, Q.v[9], 9 < ns, k, ks, seed);
	quad_stripe<10>(a0, a1, Q.v[10], 10 < ns, k, ks, seed);
	quad_stripe<11>(a0, a1, Q.v[11], 11 < ns, k, ks, seed);
	quad_stripe<12>(a0, a1, Q.v[12], 12 < ns, k, ks, seed);
	quad_stripe<13>(a0, a1, Q.v[13], 13 < ns, k, ks, seed);
	quad_stripe<14>(a0, a1, Q.v[14], 14 < ns, k, ks, seed);
	{  // the last stripe: secret + 121
		const uint64_t x0 = Q.vl[0] ^ lat(ks, 15 + 2 * k, 1, seed), x1 = Q.vl[1] ^ lat(ks, 16 + 2 * k, 1, seed);
		a0 += Q.vl[1] + (uint64_t)(uint32_t)x0 * (x0 >> 32);
		a1 += Q.vl[0] + (uint64_t)(uint32_t)x1 * (x1 >> 32);
	}
	const uint64_t m = mulfold(a0 ^ lat(ks, 1 + 2 * k, 3, seed), a1 ^ lat(ks, 2 + 2 * k, 3, seed));  // merge: secret + 11
	uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
	add_dpp<0xB1>(lo, hi);
	add_dpp<0x4E>(lo, hi);
	return xxh3_aval(len * P64_1 + (((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int j) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j);
	return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t rdfirst64v(uint64_t v) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}

// lanes below this one with their bit set in m
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t permute64(int addr, uint64_t v) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t bpermute64(int addr, uint64_t v) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}

struct VStep {
	uint64_t v[4][2];
	uint64_t len, buf, seed;  // this row's buffer
	uint32_t blk;             // block loaded
	uint32_t ra;              // FDBXXH_ALN: the row's byte shift (0: loaded at the bytes' own address)
	uint32_t nx;              // ... lane 15: the dword after the block
	bool act;                 // row has a buffer
	bool any;                 // some row has one (uniform)
};
#ifndef FDBXXH_ALN
#define FDBXXH_ALN 1
#endif

constexpr int kTailPasses = 4;                    // buffers listed at once: 64 each
constexpr uint32_t kTailCap = 64 * kTailPasses;  // list entries per wave
template <bool SEEDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_xxh3_vrows(XxhParams P) {
	if (P.d_count) P.count = min(P.count, (uint64_t)*P.d_count);  // device-sized batch (the planner's too)
	const int lane = threadIdx.x & 63;
	const int r = lane >> 4, l = lane & 15, k = l & 3, g = l >> 2;
	__shared__ uint64_t ksl[24];  // the default secret (the quad path's keys)
	__shared__ __attribute__((aligned(16))) uint64_t skey[32];  // the short path's keys (short_keys)
	// per wave: the tail's short (from the front) and quad (from the back) lists
	__shared__ uint64_t tlen[4][kTailCap], toff[4][kTailCap];
	__shared__ uint32_t tidx[4][kTailCap];
	__shared__ uint64_t tsd[SEEDS ? 4 : 1][SEEDS ? kTailCap : 1];
	if (threadIdx.x < 24) ksl[threadIdx.x] = SEEDS ? kSec[threadIdx.x] : sec_word((int)threadIdx.x, P.seed);
	short_keys(skey, (int)threadIdx.x, SEEDS ? 0 : P.seed);
	__syncthreads();
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t w = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef FDBXXH_TIMES
	const uint64_t vt0 = __builtin_amdgcn_s_memrealtime();
#endif
	const uint64_t begin = rdfirst64v(P.wave_first[w]);
	uint64_t end = rdfirst64v(P.wave_first[w + 1]);
	end = end < P.count ? end : P.count;
	if (begin >= end) return;
	const uint64_t base = reinterpret_cast<uint64_t>(P.base);
	const uint64_t* __restrict__ lengths = P.lengths;
	const uint64_t* __restrict__ offsets = P.offsets;
	const uint64_t* __restrict__ seeds = P.seeds;
	uint64_t* __restrict__ out = P.out;
	const uint64_t seed0 = P.seed;
	// long buffers on the split route (xxh3_split.hip) are not this kernel's
	const uint8_t* __restrict__ lflag = P.lflag;


	// ---- long buffers: rows
	const uint64_t dummy = reinterpret_cast<uint64_t>(P.wave_first);
	// Two pool banks.  B holds the next 64 buffers as loaded; its loads are
	// issued a pool ahead and read only when A runs dry, so the wait finds
	// them long complete.  A holds the row buffers of a taken pool COMPACTED
	// (ds_permute) into lanes 0 .. na-1, handed out in order from the cursor
	// ac: the rows that need a buffer pull theirs with ds_bpermute, all rows
	// at once (a serial pick per row cost ~40 instructions a buffer, the
	// bound for buffers of a block or two).
	uint64_t bb = 0, pnext = begin;
	uint64_t alen = 0, aoff = 0, aseed = 0, blen = 0, boff = 0, bseed = 0;
	uint32_t aj = 0, bfl = 0, na = 0, ac = 0;
	bool bpend = false;  // B loaded, not yet taken (uniform)
	auto issue_b = [&]() __attribute__((always_inline)) {
		bb = rdfirst64v(pnext);  // keep the pool cursor in SGPRs
		pnext = bb + 64;
		const uint64_t i = bb + lane;
		const bool in = i < end;
		blen = in ? lengths[i] : 0;
		boff = in ? offsets[i] : 0;
		if (SEEDS) bseed = in ? seeds[i] : 0;
		bfl = (lflag && in) ? lflag[i] : 0;
		bpend = true;
	};
	// A <- B, compacted (A exhausted); false when the wave's range has no row buffer left
	auto take_b = [&]() __attribute__((always_inline)) -> bool {
		for (;;) {
			if (!bpend) {
				if (pnext >= end) return false;
				issue_b();
			}
			bpend = false;
			const bool on = blen > kXQuadMax && !(blen > kXSplitMin && bfl);
			const uint64_t m = __ballot(on);
			const uint32_t n = (uint32_t)__builtin_popcountll(m);
			if (n == 0) continue;
			const uint32_t below = mbcnt64(m);
			const int d = (int)(((on ? below : n + (uint32_t)lane - below) & 63u) << 2);
			alen = permute64(d, blen);
			aoff = permute64(d, boff);
			if (SEEDS) aseed = permute64(d, bseed);
			aj = (uint32_t)__builtin_amdgcn_ds_permute(d, (int)(uint32_t)(bb - begin + (uint64_t)lane));
			na = n;
			ac = 0;
			return true;
		}
	};
	auto refill = [&]() __attribute__((always_inline)) {
		if (ac == na && bpend) take_b();
		if (!bpend && pnext < end) issue_b();
	};
	// load cursor of this lane's row (row-uniform)
	uint64_t lp = dummy, llen = 1024, lbuf = 0, lseed = seed0;
	uint32_t lblk = 0, lnblk = 0;
	bool lact = false;

	auto grab = [&]() __attribute__((always_inline)) {
		const uint64_t need = __ballot(l == 0 && lblk == lnblk);
		if (need != 0) {
			const bool mine = lblk == lnblk;
			// this row's rank among the rows that need one
			const uint32_t rk = mbcnt64(need) - (mine && l != 0 ? 1u : 0u);
			const uint32_t nn = (uint32_t)__builtin_popcountll(need);
			uint32_t got = 0;
			while (got < nn) {
				if (ac == na && !take_b()) break;
				const uint32_t t = min(nn - got, na - ac);
				const bool pick = mine && rk - got < t;  // unsigned: rk in [got, got + t)
				const int src = (int)((ac + rk - got) & 63u) << 2;
				const uint64_t len = bpermute64(src, alen), off = bpermute64(src, aoff);
				const uint64_t sd = SEEDS ? bpermute64(src, aseed) : seed0;
				const uint32_t j = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)aj);
				if (pick) {
					llen = len;
					lp = base + off;
					lblk = 0;
					lnblk = (uint32_t)((len - 1) >> 10) + 1;
					lbuf = begin + j;
					lseed = sd;
					lact = true;
				}
				ac += t;
				got += t;
			}
		}
		if (lblk == lnblk) {  // no buffer for this row: read the dummy KiB
			lact = false;
			lp = dummy;
			llen = 1024;
			lblk = 0;
			lnblk = 1;
		}
	};
	auto load = [&](VStep& S) __attribute__((always_inline)) {
		grab();
		const uint64_t nfull = (llen - 1) >> 10;
		const uint32_t ns = (uint32_t)(((llen - 1) - (nfull << 10)) >> 6);
		const bool fin = lblk == nfull;
		// FDBXXH_ALN: a full block of a byte-unaligned buffer loads from the
		// dword-aligned address below its bytes (a byte-unaligned dwordx4 streams
		// ~23 % slower, a dword-aligned one at full rate: tools/membench3.hip),
		// and compute() shifts the bytes back (v_alignbyte; the dword after each
		// lane's chunk from the next lane, DPP; after the block's last chunk, lane
		// 15's own extra load, issued only by the rows that shift).  A dword
		// holding a buffer byte never crosses a page, so nothing outside a mapped
		// page is read.
		const uint32_t ra = FDBXXH_ALN && !fin ? (uint32_t)lp & 3u : 0u;
		const uint64_t lpa = lp - ra;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool tail = fin && (s == 15 || s >= ns);
			const uint64_t a = tail ? lp + llen - 64 + 16 * k : lpa + ((uint64_t)lblk << 10) + 64 * s + 16 * k;
			const u64x2u x = __builtin_nontemporal_load((g_u64x2u*)a);
			S.v[i][0] = x[0];
			S.v[i][1] = x[1];
		}
		if (FDBXXH_ALN && l == 15 && ra != 0) S.nx = __builtin_nontemporal_load((g_u32a*)(lpa + ((uint64_t)(lblk + 1) << 10)));
		S.ra = ra;
		S.len = llen;
		S.buf = lbuf;
		S.seed = lseed;
		S.blk = lblk;
		S.act = lact;
		S.any = __ballot(lact) != 0;
		++lblk;
	};

	// Results collect in lanes (rx = hash, rj = buffer - begin, rn used; the
	// finishing rows' values move in with ds_permute) and leave 64 at a time:
	// a store in the loop holds up every later wait on the loads issued
	// behind it (in-order vmcnt).
	uint64_t rx = 0;
	uint32_t rj = 0, rn = 0;
	auto flush = [&]() __attribute__((always_inline)) {
		if ((uint32_t)lane < rn) out[begin + rj] = rx;
		rn = 0;
	};
	RowKeys K = row_keys(lane, seed0);
	uint64_t a0 = 0, a1 = 0;
	auto compute = [&](VStep& S) __attribute__((always_inline)) {
		const uint64_t nfull = (S.len - 1) >> 10;
		const uint32_t ns = (uint32_t)(((S.len - 1) - (nfull << 10)) >> 6);
		const bool fin = S.blk == nfull;
		if (FDBXXH_ALN && __ballot(S.ra != 0) != 0) {  // some row loaded dword-aligned: shift its bytes back
			uint32_t nxt[4];
#pragma unroll
			for (int i = 0; i < 4; ++i)  // lane l <- dword 0 of lane l + 1 (mod 16) of load i
				nxt[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)S.v[i][0], 0x12F, 0xF, 0xF, false);
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const uint32_t w0 = (uint32_t)S.v[i][0], w1 = (uint32_t)(S.v[i][0] >> 32);
				const uint32_t w2 = (uint32_t)S.v[i][1], w3 = (uint32_t)(S.v[i][1] >> 32);
				const uint32_t w4 = l == 15 ? (i < 3 ? nxt[i + 1] : S.nx) : nxt[i];
				const uint32_t sh = S.ra;
				S.v[i][0] = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
				S.v[i][1] = ((uint64_t)__builtin_amdgcn_alignbyte(w4, w3, sh) << 32) | __builtin_amdgcn_alignbyte(w3, w2, sh);
			}
		}
		if (SEEDS && __ballot(S.blk == 0 && S.act) != 0) K = row_keys(lane, S.seed);
		if (S.blk == 0) {
			a0 = k == 0 ? P32_3 : (k == 1 ? P64_2 : (k == 2 ? P64_4 : P64_5));
			a1 = k == 0 ? P64_1 : (k == 1 ? P64_3 : (k == 2 ? P32_2 : P32_1));
		}
		uint64_t d0 = 0, d1 = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool last = fin && s == 15;
			const bool on = !fin || s < ns || last;
			const uint64_t x0 = S.v[i][0] ^ (last ? K.l0 : K.k0[i]);
			const uint64_t x1 = S.v[i][1] ^ (last ? K.l1 : K.k1[i]);
			const uint64_t c0 = S.v[i][1] + (uint64_t)(uint32_t)x0 * (x0 >> 32);
			const uint64_t c1 = S.v[i][0] + (uint64_t)(uint32_t)x1 * (x1 >> 32);
			d0 += on ? c0 : 0;
			d1 += on ? c1 : 0;
		}
		uint32_t lo0 = (uint32_t)d0, hi0 = (uint32_t)(d0 >> 32), lo1 = (uint32_t)d1, hi1 = (uint32_t)(d1 >> 32);
		add_dpp<0x124>(lo0, hi0);
		add_dpp<0x124>(lo1, hi1);
		add_dpp<0x128>(lo0, hi0);
		add_dpp<0x128>(lo1, hi1);
		a0 += ((uint64_t)hi0 << 32) | lo0;
		a1 += ((uint64_t)hi1 << 32) | lo1;
		uint64_t done = __ballot(l == 0 && fin && S.act);
		uint64_t h = 0;
		if (done != 0) {  // some row's buffer ends at this block: the merge (uniform branch, most steps skip it)
			const uint64_t m = mulfold(a0 ^ K.g0, a1 ^ K.g1);
			uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
			add_dpp<0xB1>(lo, hi);
			add_dpp<0x4E>(lo, hi);
			h = xxh3_aval(S.len * P64_1 + (((uint64_t)hi << 32) | lo));
		}
		if (!fin) {
			a0 = ((a0 ^ (a0 >> 47)) ^ K.c0) * P32_1;
			a1 = ((a1 ^ (a1 >> 47)) ^ K.c1) * P32_1;
		}
		if (done != 0) {
			const uint32_t n = (uint32_t)__builtin_popcountll(done);
			if (rn + n > 64) flush();
			const bool on = l == 0 && fin && S.act;
			const uint32_t below = mbcnt64(done);
			const int d = (int)(((on ? rn + below : rn + n + (uint32_t)lane - below) & 63u) << 2);
			const uint64_t rh = permute64(d, h);
			const uint32_t rr = (uint32_t)__builtin_amdgcn_ds_permute(d, (int)(uint32_t)(S.buf - begin));
			const bool in = (uint32_t)lane - rn < n;
			rx = in ? rh : rx;
			rj = in ? rr : rj;
			rn += n;
		}
	};

	// ---- sparse ranges: a wave whose range is one pool holding at most two
	// row buffers (the chunks batch: its 4-16 KiB chunks beside the long
	// route, about one per wave) spreads each buffer's blocks over its four
	// rows -- block b on row b % 4 -- and chains the rows' stripe sums in
	// block order (the decomposition of xxh3_split.hip): a 16 KiB buffer is
	// four steps, not sixteen.
	auto split_one = [&](uint64_t len, uint64_t off, uint64_t sd, uint64_t idx) __attribute__((always_inline)) {
		const uint64_t p = base + off;
		const uint32_t nb = (uint32_t)((len - 1) >> 10) + 1, nfull = nb - 1;
		const uint32_t ns = (uint32_t)(((len - 1) - ((uint64_t)nfull << 10)) >> 6);
		const uint32_t nsteps = (nb + 3) / 4;
		if (SEEDS) K = row_keys(lane, sd);
		auto ld = [&](uint64_t (&v)[4][2], uint32_t t) __attribute__((always_inline)) {
			uint32_t b = 4 * t + (uint32_t)r;
			b = b < nb ? b : nfull;  // (a row past the end re-reads the final block: discarded)
			const bool fin = b == nfull;
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const uint32_t st = g + 4 * i;
				const bool tail = fin && (st == 15 || st >= ns);
				const uint64_t a = tail ? p + len - 64 + 16 * k : p + ((uint64_t)b << 10) + 64 * st + 16 * k;
				const u64x2u x = __builtin_nontemporal_load((g_u64x2u*)a);
				v[i][0] = x[0];
				v[i][1] = x[1];
			}
		};
		uint64_t s0 = k == 0 ? P32_3 : (k == 1 ? P64_2 : (k == 2 ? P64_4 : P64_5));
		uint64_t s1 = k == 0 ? P64_1 : (k == 1 ? P64_3 : (k == 2 ? P32_2 : P32_1));
		uint64_t va[4][2], vb[4][2];
		ld(va, 0);
		for (uint32_t t = 0; t < nsteps; ++t) {
			if (t + 1 < nsteps) ld(vb, t + 1);
			uint32_t b = 4 * t + (uint32_t)r;
			const bool fin = b == nfull;
			uint64_t d0 = 0, d1 = 0;
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const uint32_t st = g + 4 * i;
				const bool last = fin && st == 15;
				const bool on = !fin || st < ns || last;
				const uint64_t x0 = va[i][0] ^ (last ? K.l0 : K.k0[i]);
				const uint64_t x1 = va[i][1] ^ (last ? K.l1 : K.k1[i]);
				d0 += on ? va[i][1] + (uint64_t)(uint32_t)x0 * (x0 >> 32) : 0;
				d1 += on ? va[i][0] + (uint64_t)(uint32_t)x1 * (x1 >> 32) : 0;
			}
			uint32_t lo0 = (uint32_t)d0, hi0 = (uint32_t)(d0 >> 32), lo1 = (uint32_t)d1, hi1 = (uint32_t)(d1 >> 32);
			add_dpp<0x124>(lo0, hi0);
			add_dpp<0x124>(lo1, hi1);
			add_dpp<0x128>(lo0, hi0);
			add_dpp<0x128>(lo1, hi1);
			d0 = ((uint64_t)hi0 << 32) | lo0;
			d1 = ((uint64_t)hi1 << 32) | lo1;
			// the four rows' sums in block order, in every lane of pair k
#pragma unroll
			for (int rr = 0; rr < 4; ++rr) {
				const uint32_t bb = 4 * t + rr;
				if (bb >= nb) break;  // (uniform)
				const int a = (16 * rr + k) << 2;
				s0 += bpermute64(a, d0);
				s1 += bpermute64(a, d1);
				if (bb < nfull) {
					s0 = ((s0 ^ (s0 >> 47)) ^ K.c0) * P32_1;
					s1 = ((s1 ^ (s1 >> 47)) ^ K.c1) * P32_1;
				}
			}
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				va[i][0] = vb[i][0];
				va[i][1] = vb[i][1];
			}
		}
		const uint64_t m = mulfold(s0 ^ K.g0, s1 ^ K.g1);
		uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
		add_dpp<0xB1>(lo, hi);
		add_dpp<0x4E>(lo, hi);
		const uint64_t h = xxh3_aval(len * P64_1 + (((uint64_t)hi << 32) | lo));
		if (lane == 0) out[idx] = h;
	};
	if (end - begin <= 64) {
		issue_b();
		if (take_b() && na <= 2) {
			for (uint32_t j = 0; j < na; ++j) {
				const int a = (int)(j << 2);
				split_one(bpermute64(a, alen), bpermute64(a, aoff), SEEDS ? bpermute64(a, aseed) : seed0,
				          begin + (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)aj));
			}
			ac = na;
		}
		if (SEEDS) K = row_keys(lane, seed0);
	}

	// Two steps per half-iteration, the other half's two steps in flight; the
	// halves alternate register sets (no copies of data in flight).
	// s0/s1 start as idle steps (nothing loaded), so no data load precedes the
	// loop and every load lands in the loop's own registers.
	VStep s0, s1, t0, t1;
#pragma unroll
	for (int i = 0; i < 4; ++i) s0.v[i][0] = s0.v[i][1] = s1.v[i][0] = s1.v[i][1] = 0;
	s0.len = s1.len = 1024;
	s0.buf = s1.buf = 0;
	s0.seed = s1.seed = seed0;
	s0.blk = s1.blk = 0;
	s0.ra = s1.ra = 0;
	s0.nx = s1.nx = 0;
	s0.act = s1.act = false;
	s0.any = s1.any = false;
	for (;;) {
		if (!s0.any && !s1.any && ac == na && !bpend && pnext >= end) break;
		refill();
		load(t0);
		load(t1);
		__builtin_amdgcn_sched_barrier(0);
		compute(s0);
		compute(s1);
		__builtin_amdgcn_sched_barrier(0);
		if (!t0.any && !t1.any && ac == na && !bpend && pnext >= end) break;
		refill();
		load(s0);
		load(s1);
		__builtin_amdgcn_sched_barrier(0);
		compute(t0);
		compute(t1);
		__builtin_amdgcn_sched_barrier(0);
	}
	flush();
	// ---- short buffers (<= 240 B, one lane each) and 241 B - 1 KiB ones (lane
	// quads, xxh3_quad): after the long ones, so that every wave starts
	// streaming at once (their dependent length -> data loads kept HBM idle at
	// the start of the launch: zipf 0.272 -> 0.253 ms, unaligned zipf 0.352 ->
	// 0.303 ms).  This part is a chain of memory round trips per wave (zipf: 30
	// us of the row kernel), so it is made dense: the lengths and offsets of
	// up to 512 buffers load at once, the short and quad ones are listed in the
	// wave's LDS (compacted), and then every pass is full -- 64 short buffers,
	// or 16 quads, one round trip each.  A pass's results are stored after the
	// next pass's loads are issued (a store holds up every later wait on loads
	// issued behind it: in-order vmcnt).
#ifdef FDBXXH_NOTAIL
	if (P.count != 12345) return;  // timing experiment: no short/quad phase (wrong results)
#endif
#ifdef FDBXXH_TIMES
	const uint64_t vt1 = __builtin_amdgcn_s_memrealtime();
#endif
	const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint64_t* const tl_len = tlen[wv];
	uint64_t* const tl_off = toff[wv];
	uint32_t* const tl_idx = tidx[wv];
	uint64_t* const tl_sd = SEEDS ? tsd[wv] : nullptr;
	uint64_t pend_h = 0, pend_i = 0;
	bool pend = false;
	auto flushp = [&]() __attribute__((always_inline)) {  // after the next pass's loads
		if (pend) out[pend_i] = pend_h;
		pend = false;
	};
	auto put = [&](bool on, uint64_t h, uint64_t idx) __attribute__((always_inline)) {
		pend_h = h;
		pend_i = idx;
		pend = on;
	};
	for (uint64_t c0 = begin; c0 < end; c0 += 64 * kTailPasses) {
		uint64_t L[kTailPasses], O[kTailPasses], D[kTailPasses];
#pragma unroll
		for (int q = 0; q < kTailPasses; ++q) {
			const uint64_t i = c0 + 64 * q + lane;
			const bool in = i < end;
			const uint64_t ic = in ? i : begin;  // (every load unconditional)
			L[q] = lengths[ic];
			O[q] = offsets[ic];
			D[q] = SEEDS ? seeds[ic] : seed0;
			if (!in) L[q] = ~0ull;  // (no class)
		}
		uint32_t ns = 0, nq = 0;
#pragma unroll
		for (int q = 0; q < kTailPasses; ++q) {
			const uint64_t i = c0 + 64 * q + lane;
			const uint64_t len = L[q];
			const bool tiny = len <= 16, sh = len > 16 && len <= 240, qd = len > 240 && len <= kXQuadMax;
			if (__ballot(tiny) != 0 && tiny) out[i] = xxh3_short(base + O[q], len, D[q]);  // (rare)
			const uint64_t ms = __ballot(sh), mq = __ballot(qd);
			if (sh) {
				const uint32_t e = ns + mbcnt64(ms);
				tl_len[e] = len;
				tl_off[e] = O[q];
				tl_idx[e] = (uint32_t)(i - begin);
				if (SEEDS) tl_sd[e] = D[q];
			}
			if (qd) {
				const uint32_t e = kTailCap - 1 - (nq + mbcnt64(mq));
				tl_len[e] = len;
				tl_off[e] = O[q];
				tl_idx[e] = (uint32_t)(i - begin);
				if (SEEDS) tl_sd[e] = D[q];
			}
			ns += (uint32_t)__builtin_popcountll(ms);
			nq += (uint32_t)__builtin_popcountll(mq);
		}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		for (uint32_t s0 = 0; s0 < ns; s0 += 64) {  // full passes of short buffers
			const uint32_t e = s0 + lane;
			const bool on = e < ns;
			const uint32_t ec = on ? e : s0;
			const uint64_t len = tl_len[ec], off = tl_off[ec], sd = SEEDS ? tl_sd[ec] : seed0;
			const uint64_t idx = begin + tl_idx[ec];
			ShortLd SL;
			short_load(SL, base + off, len, on);
			flushp();
			put(on, short_fin_k<SEEDS>(SL, len, skey, sd), idx);
		}
		for (uint32_t t0 = 0; t0 < nq; t0 += 16) {  // full passes of sixteen quads
			const uint32_t e = t0 + ((uint32_t)lane >> 2);
			const bool act = e < nq;
			const uint32_t ec = kTailCap - 1 - (act ? e : t0);
			const uint64_t len = act ? tl_len[ec] : 256, off = act ? base + tl_off[ec] : dummy;
			const uint64_t sd = SEEDS ? tl_sd[ec] : 0;
			const uint64_t idx = begin + tl_idx[ec];
			QuadLd QL;
			quad_load(QL, off, len, lane & 3);
			flushp();
			put(act && (lane & 3) == 0, quad_fin(QL, len, sd, lane & 3, ksl), idx);  // (unseeded: ksl holds the seed's secret)
		}
		__builtin_amdgcn_wave_barrier();  // (the list is rewritten by the next chunk)
	}
	if (pend) out[pend_i] = pend_h;
#ifdef FDBXXH_TIMES
	const uint64_t vt2 = __builtin_amdgcn_s_memrealtime();
	if (lane == 0 && w < 16384) {
		g_vt[w][0] = vt0;
		g_vt[w][1] = vt1;
		g_vt[w][2] = vt2;
		g_vt[w][3] = end - begin;
	}
#endif
}

// ---------------------------------------------------------------------------
// Varlen planning: whole buffers per wave, balanced by bytes.  Wave w takes
// the buffers whose start lies in [w*Q, (w+1)*Q) of the concatenated stream
// (cost = length + 64 on the rows, kXTailCost for a short or quad buffer).  With room for the long-buffer route in the
// workspace, the buffers longer than kXSplitMin take it (xxh3_split.hip) if
// their entries fit the room (else the row kernel takes the whole batch).
// No counters to reset: k_xplan writes per-tile sums, k_xscan scans them (the
// route, the cost prefixes, the size classes' bases), k_xassign gives every
// buffer its place -- the row kernel's waves, the flag byte that takes a long
// buffer off the row kernel (cost 64 there) and the long buffer's entry in
// its size class (largest class first: k_xlong takes them in that order).
// Batches of at most kXFuseTiles tiles skip k_xscan: k_xassign<true> reduces
// the tiles' sums in every workgroup (chunks batch: 224 against 228 us).
// ---------------------------------------------------------------------------
struct XPlanP {
	const uint64_t* lengths;  // nullptr: fixed length
	const uint64_t* offsets;  // nullptr: fixed stride
	const uint64_t* seeds;
	const uint8_t* base;
	uint64_t stride, length, count, seed;
	uint64_t* tiles;          // [ntile + 2]: cost if routed (k_xplan) -> exclusive cost prefixes, total, quantum
	uint64_t* tcns;           // [ntile]: cost if not routed
	uint64_t* tneed;          // [ntile]: long blocks (the stream's need) -> route flag (k_xscan)
	uint64_t* tcls;           // [4][ntile]: long buffers per size class, 16-bit fields (class c: word c / 4)
	uint64_t* sh;             // [kXShWords] (XLong::sh)
	uint8_t* flag;            // per buffer: 1 if the long route took it
	uint64_t* wave_first;
	uint64_t ntile, nwave;
	uint64_t older;           // waves of the first-dispatched workgroups (0: all weighted alike)
	XEnt* ents;
	uint64_t capS;            // entries the room holds (0: no room)
	uint64_t* hneed;          // host-mapped word (may be null): blocks the batch's long buffers need
	const uint64_t* dcount;   // may be null: the batch size is min(count, *dcount) (count bounds the grid)
};
constexpr uint64_t kTileRouted = 1ull << 63;
// The row kernel's waves as placed on the CUs: with two workgroups per CU the
// first-dispatched one's waves are older and win the SIMD's issue arbitration,
// and stream the same bytes ~19 % sooner (zipf, per-wave timestamps: 142 vs
// 169 us median).  Their ranges are longer by about that ratio (kXOlderW /
// 16: 21/16 measured a little faster end to end than 17/16, 19/16 or 23/16),
// so both generations end together.  B(w) = w * qa for the `older` first waves,
// then qb per wave.
#ifndef FDBXXH_OLDER16
#define FDBXXH_OLDER16 21
#endif
constexpr uint64_t kXOlderW = FDBXXH_OLDER16;
struct XQuant {
	uint64_t qa, qb, h;
};
__device__ __forceinline__ XQuant xquant(uint64_t total, uint64_t nwave, uint64_t older) {
	XQuant W;
	if (older == 0 || older >= nwave) {
		W.qa = W.qb = max((total + nwave - 1) / nwave, (uint64_t)1);
		W.h = 0;
		return W;
	}
	const uint64_t den = 16 * (nwave - older) + kXOlderW * older;
	W.qb = max((16 * total + den - 1) / den, (uint64_t)1);
	W.qa = (W.qb * kXOlderW + 15) / 16;
	W.h = older;
	return W;
}
// the last wave w with B(w) <= x
__device__ __forceinline__ uint64_t xquant_wave(const XQuant& W, uint64_t x) {
	const uint64_t ha = W.h * W.qa;
	return x < ha ? x / W.qa : W.h + (x - ha) / W.qb;
}
__device__ __forceinline__ uint64_t xp_len(const XPlanP& Q, uint64_t i) { return Q.lengths ? Q.lengths[i] : Q.length; }
__device__ __forceinline__ uint64_t xp_off(const XPlanP& Q, uint64_t i) { return Q.offsets ? Q.offsets[i] : i * Q.stride; }
__device__ __forceinline__ uint64_t xp_blocks(uint64_t len) { return ((len - 1) >> 10) + 1; }
// A wave's cost of a buffer, in bytes of row streaming: its bytes + 64 on the
// rows, a flat kXTailCost for the short and quad ones (<= kXQuadMax: their
// part is a chain of memory round trips, ~0.24 us of the wave's time each on
// zipf against 0.29 us per row KiB; 1152-1280 measured best of 640-1280 under
// the bench protocol), 64 on the long route.
#ifndef FDBXXH_TAIL_COST
#define FDBXXH_TAIL_COST 1152
#endif
constexpr uint64_t kXTailCost = FDBXXH_TAIL_COST;
__device__ __forceinline__ uint64_t xp_cost(uint64_t len, bool routed) {
	return routed ? 64 : (len <= kXQuadMax ? kXTailCost : len + 64);
}
// a long buffer (its blocks count in the stream's need whether or not there is room)
__device__ __forceinline__ bool xp_long(uint64_t len) { return len > kXSplitMin; }
// Size class of a long buffer: 0 for 2^19 blocks (512 MiB) or more, then one
// per power of two down to 15 for 16-31 blocks.
__device__ __forceinline__ uint32_t xp_class(uint64_t nb) {
	const uint32_t lg = 63 - __builtin_clzll(nb);
	return lg >= 19 ? 0u : 19u - (lg < 4 ? 4u : lg);
}

// Inclusive prefix sum of a 64-bit value over the wave on DPP (row shifts,
// then the row broadcasts of lanes 15 and 31; every lane active).
__device__ __forceinline__ uint64_t dpp_incl64(uint64_t v) {
#define XDPP_STEP(ctrl, rm)                                                                          \
	{                                                                                                \
		const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, ctrl, rm, 0xF, false);         \
		const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), ctrl, rm, 0xF, false); \
		v += ((uint64_t)hi << 32) | lo;                                                              \
	}
	XDPP_STEP(0x111, 0xF)  // row_shr:1
	XDPP_STEP(0x112, 0xF)  // row_shr:2
	XDPP_STEP(0x114, 0xF)  // row_shr:4
	XDPP_STEP(0x118, 0xF)  // row_shr:8
	XDPP_STEP(0x142, 0xA)  // row_bcast:15 -> rows 1, 3
	XDPP_STEP(0x143, 0xC)  // row_bcast:31 -> rows 2, 3
#undef XDPP_STEP
	return v;
}
__device__ __forceinline__ uint64_t rdlane63(uint64_t v) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
	return ((uint64_t)hi << 32) | lo;
}

// Planner tiles: 256 buffers (one per thread) for batches of up to
// 256 x kXFuseTiles buffers, else 256 x kXPerBig (kXPerBig per thread).  A
// zipf batch (406 k buffers) is then 397 tiles, under kXFuseTiles, so
// k_xassign reduces the tile sums itself and k_xscan is not launched: planner
// kernels 7.1 + 6.6 + 7.3 us -> 5.4 + 7.9 us (same box).  Eight per thread
// (199 tiles) measured 5.5 + 8.7 us: a thread's buffers are a serial chain,
// and a fused k_xassign of 199 workgroups holds under one wave per SIMD.
#ifndef FDBXXH_PLAN_PER
#define FDBXXH_PLAN_PER 4
#endif
constexpr uint32_t kXPerBig = FDBXXH_PLAN_PER;
static_assert(256ull * kXPerBig < 65536, "a tile's class counts are 16-bit fields");

// One workgroup per tile: the tile's sums (thread t takes buffers t + 256u).
template <uint32_t kXPer>
__global__ __launch_bounds__(256) void k_xplan(XPlanP Q) {
	constexpr uint64_t kXTile = 256ull * kXPer;
	__shared__ uint64_t part[4][8];
	if (Q.dcount) Q.count = min(Q.count, (uint64_t)*Q.dcount);
	const uint64_t i0 = (uint64_t)blockIdx.x * kXTile + threadIdx.x;
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint64_t len[kXPer];
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) {
		const uint64_t i = i0 + 256u * u;
		len[u] = i < Q.count ? xp_len(Q, i) : 0;
	}
	uint64_t v[8] = {};
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) {
		const bool in = i0 + 256u * u < Q.count;
		const bool lg = in && xp_long(len[u]);
		const uint64_t nb = lg ? xp_blocks(len[u]) : 0;
		const uint32_t cl = lg ? xp_class(nb) : 0;
		v[0] += in ? xp_cost(len[u], lg) : 0;
		v[1] += in ? xp_cost(len[u], false) : 0;
		v[2] += nb;
		const uint64_t bit = lg ? 1ull << (16 * (cl & 3)) : 0;  // (16-bit fields: at most kXTile per tile)
#pragma unroll
		for (uint32_t w = 0; w < 4; ++w) v[4 + w] += (cl >> 2) == w ? bit : 0;
	}
#pragma unroll
	for (int q = 0; q < 8; ++q) v[q] = rdlane63(dpp_incl64(v[q]));
	if (lane == 0)
#pragma unroll
		for (int q = 0; q < 8; ++q) part[wv][q] = v[q];
	__syncthreads();
	if (threadIdx.x < 8 && threadIdx.x != 3) {
		const int q = threadIdx.x;
		const uint64_t s = part[0][q] + part[1][q] + part[2][q] + part[3][q];
		uint64_t* dst = q == 0 ? Q.tiles : q == 1 ? Q.tcns : q == 2 ? Q.tneed : Q.tcls + (uint64_t)(q - 4) * Q.ntile;
		dst[blockIdx.x] = s;
	}
}

// Single workgroup.  The long route takes every long buffer or none: all of
// them if their entries fit the room (the library sizes the room from the
// stream's last need; the _ws form's caller sizes it with
// xxh3_gpu_varlen_workspace_bytes_for), else the row kernel takes the whole
// batch.  In place: the exclusive prefixes of the routed tile costs,
// tiles[ntile] = total cost (k_xassign derives the waves' quanta from it,
// xquant), the route flag in tneed; in sh[] the long buffers routed, the
// dequeue counter (0) and the size classes' cursors (their bases, largest
// class first).
__global__ __launch_bounds__(1024) void k_xscan(XPlanP Q) {
	__shared__ uint64_t red[kXClasses + 1][16];
	__shared__ uint64_t tot_s[kXClasses + 1];
	__shared__ uint64_t carry_s;
	const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
	const uint64_t ntile = Q.ntile;
	uint64_t* tiles = Q.tiles;
	// totals: long blocks and the classes' counts
	uint64_t a[kXClasses + 1] = {};
	for (uint64_t k = t; k < ntile; k += 1024) {
		const uint64_t nb = Q.tneed[k];
		a[kXClasses] += nb;
		if (nb)  // (tiles without long buffers have no class counts)
#pragma unroll
			for (uint32_t w = 0; w < 4; ++w) {
				const uint64_t f = Q.tcls[w * ntile + k];
#pragma unroll
				for (uint32_t u = 0; u < 4; ++u) a[4 * w + u] += (f >> (16 * u)) & 0xFFFFu;
			}
	}
	if (t == 0) carry_s = 0;
	const bool anylong = __syncthreads_or(a[kXClasses] != 0);
	if (anylong) {
#pragma unroll
		for (uint32_t q = 0; q <= kXClasses; ++q) {
			const uint64_t s = rdlane63(dpp_incl64(a[q]));
			if (lane == 0) red[q][wv] = s;
		}
		__syncthreads();
		if (t <= kXClasses) {
			uint64_t s = 0;
			for (uint32_t u = 0; u < 16; ++u) s += red[t][u];
			tot_s[t] = s;
		}
	} else if (t <= kXClasses) {
		tot_s[t] = 0;
	}
	__syncthreads();
	uint64_t nlong = 0;
	for (uint32_t q = 0; q < kXClasses; ++q) nlong += tot_s[q];
	const bool routed = nlong != 0 && Q.capS && nlong <= Q.capS;
	__syncthreads();  // (red is reused below)
	for (uint64_t c0 = 0; c0 < ntile; c0 += 1024) {
		const uint64_t k = c0 + t;
		const bool in = k < ntile;
		const uint64_t x = in ? (routed ? tiles[k] : Q.tcns[k]) : 0;
		const uint64_t inc = dpp_incl64(x);
		if (lane == 63) red[0][wv] = inc;
		__syncthreads();
		uint64_t ex = carry_s + inc - x;
		for (uint32_t u = 0; u < wv; ++u) ex += red[0][u];
		if (in) {
			tiles[k] = ex;
			Q.tneed[k] = routed ? kTileRouted : 0;
		}
		__syncthreads();
		if (t == 1023) carry_s = ex + x;
		__syncthreads();
	}
	if (t == 0) {
		const uint64_t total = carry_s;
		tiles[ntile] = total;
		tiles[ntile + 1] = 0;  // (the quantum: xquant of the total)
		Q.sh[0] = routed ? nlong : 0;
		Q.sh[1] = 0;
		Q.sh[2] = 0;
		uint64_t b = 0;
		for (uint32_t q = 0; q < kXClasses; ++q) {
			Q.sh[8 + q] = b;
			b += tot_s[q];
		}
		if (Q.hneed) *(volatile uint64_t*)Q.hneed = tot_s[kXClasses];  // every long buffer's blocks, routed or not
	}
}

// One workgroup per tile (thread t: buffers t*kXPer .. t*kXPer + kXPer - 1 of
// it, contiguous, so their starts follow from one scan): buffer i (cost c_i, start s_i) is
// the first buffer of every wave w with s_{i-1} < w*Q <= s_i; waves past
// the last buffer get `count`.  A routed long buffer writes its entry in its
// size class (any order within the class).
//
// FUSED (batches of at most kXFuseTiles tiles): no k_xscan -- every workgroup
// reduces all the tiles' sums itself (thread k takes tile k) to the batch's
// route, its tile's start and the quantum, and its classes' bases from the
// counts of the tiles before it (no cursor atomics); workgroup 0 writes sh[].
#ifndef FDBXXH_FUSE_TILES
#define FDBXXH_FUSE_TILES 512
#endif
constexpr uint64_t kXFuseTiles = FDBXXH_FUSE_TILES;
template <bool FUSED, uint32_t kXPer>
__global__ __launch_bounds__(256) void k_xassign(XPlanP Q) {
	constexpr uint64_t kXTile = 256ull * kXPer;
	__shared__ uint64_t wsum[4];
	if (Q.dcount) Q.count = min(Q.count, (uint64_t)*Q.dcount);
	__shared__ uint32_t ccount[kXClasses];
	__shared__ uint64_t cbase[kXClasses];
	const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
	// this thread's kXPer consecutive buffers, their metadata loaded before
	// the tile sums are reduced (no load waits behind the barriers)
	const uint64_t ib = (uint64_t)blockIdx.x * kXTile + (uint64_t)t * kXPer;
	uint64_t len[kXPer], off[kXPer], sdv[kXPer];
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) len[u] = ib + u < Q.count ? xp_len(Q, ib + u) : 0;
	// the buffer before this thread's first (its start gives that buffer's wave range)
	const uint64_t lp = ib != 0 && ib < Q.count ? xp_len(Q, ib - 1) : 0;
	// a long buffer's entry: its offset and seed (with room for the long route)
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) {
		const bool in = Q.capS && ib + u < Q.count;
		off[u] = in && Q.offsets ? Q.offsets[ib + u] : 0;
		sdv[u] = in && Q.seeds ? Q.seeds[ib + u] : Q.seed;
	}
	bool routed;
	uint64_t tile_start;
	XQuant W;
	if (FUSED) {
		// r[0..7]: the classes' counts over all tiles, r[8..15] over the tiles
		// before this one (32-bit fields, two classes a word); r[16], r[17]: the
		// earlier tiles' cost routed / not; r[18], r[19]: all tiles' cost
		// routed / not; r[20]: long blocks
		constexpr int kR = 21;
		__shared__ uint64_t red[kR][4];
		uint64_t r[kR] = {};
		// (thread t takes tiles t, t + 256, ...: two at a time, their loads together)
#pragma unroll 2
		for (uint32_t k = t; k < Q.ntile; k += 256) {
			const uint64_t cr = Q.tiles[k], cu = Q.tcns[k], nb = Q.tneed[k];
			const bool before = k < blockIdx.x;
			r[18] += cr;
			r[19] += cu;
			r[20] += nb;
			if (before) {
				r[16] += cr;
				r[17] += cu;
			}
			if (nb)
#pragma unroll
				for (uint32_t w = 0; w < 4; ++w) {
					const uint64_t f = Q.tcls[w * Q.ntile + k];
					const uint64_t a = (f & 0xFFFFull) | ((f >> 16 & 0xFFFFull) << 32);
					const uint64_t b = (f >> 32 & 0xFFFFull) | ((f >> 48) << 32);
					r[2 * w] += a;
					r[2 * w + 1] += b;
					if (before) {
						r[8 + 2 * w] += a;
						r[8 + 2 * w + 1] += b;
					}
				}
		}
		const bool anylong = __syncthreads_or(r[20] != 0);
#pragma unroll
		for (int k = 0; k < kR; ++k) {
			if (k < 16 && !anylong) continue;
			const uint64_t v = rdlane63(dpp_incl64(r[k]));
			if (lane == 0) red[k][wv] = v;
		}
		__syncthreads();
		uint64_t tot[kR];
#pragma unroll
		for (int k = 0; k < kR; ++k) tot[k] = k < 16 && !anylong ? 0 : red[k][0] + red[k][1] + red[k][2] + red[k][3];
		uint64_t cnt[kXClasses], nlong = 0;
#pragma unroll
		for (uint32_t c = 0; c < kXClasses; ++c) {
			cnt[c] = (tot[c >> 1] >> (32 * (c & 1))) & 0xFFFFFFFFull;
			nlong += cnt[c];
		}
		routed = nlong != 0 && Q.capS && nlong <= Q.capS;
		tile_start = routed ? tot[16] : tot[17];
		const uint64_t total = routed ? tot[18] : tot[19];
		W = xquant(total, Q.nwave, Q.older);
		if (t < kXClasses) {
			uint64_t b = 0;
#pragma unroll
			for (uint32_t c = 0; c < kXClasses; ++c) b += c < t ? cnt[c] : 0;
			uint64_t e = 0;  // (selects, not a register index: that would go to scratch)
#pragma unroll
			for (uint32_t w = 0; w < 8; ++w) e = (t >> 1) == w ? tot[8 + w] : e;
			cbase[t] = b + ((e >> (32 * (t & 1))) & 0xFFFFFFFFull);
		}
		if (blockIdx.x == 0 && t == 0) {
			Q.sh[0] = routed ? nlong : 0;
			Q.sh[1] = 0;
			Q.sh[2] = 0;
			if (Q.hneed) *(volatile uint64_t*)Q.hneed = tot[20];  // every long buffer's blocks, routed or not
		}
	} else {
		routed = (Q.tneed[blockIdx.x] & kTileRouted) != 0;
		W = xquant(Q.tiles[Q.ntile], Q.nwave, Q.older);
		tile_start = Q.tiles[blockIdx.x];
	}
	uint64_t cost[kXPer];
	uint32_t cl[kXPer], rank[kXPer];
	bool lg[kXPer];
	uint64_t tsum = 0;
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) {
		const bool in = ib + u < Q.count;
		lg[u] = in && routed && xp_long(len[u]);
		cost[u] = in ? xp_cost(len[u], lg[u]) : 0;
		cl[u] = lg[u] ? xp_class(xp_blocks(len[u])) : 0;
		tsum += cost[u];
		if (Q.capS && in) Q.flag[ib + u] = lg[u] ? 1 : 0;
	}
	const uint64_t inc = dpp_incl64(tsum);
	if (lane == 63) wsum[wv] = inc;
	if (t < kXClasses) ccount[t] = 0;
	__syncthreads();
	// a long buffer's rank in its class within the tile (LDS), then one global
	// add per class and tile (the classes' cursors are a handful of words: one
	// add per buffer measured 16 us of contention on the chunks batch)
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) rank[u] = lg[u] ? atomicAdd(&ccount[cl[u]], 1u) : 0;
	__syncthreads();
	if (!FUSED && t < kXClasses && ccount[t]) cbase[t] = atomicAdd((unsigned long long*)&Q.sh[8 + t], (unsigned long long)ccount[t]);
	__syncthreads();
	uint64_t ex = inc - tsum;
	for (uint32_t u = 0; u < wv; ++u) ex += wsum[u];
	uint64_t start = tile_start + ex;
	// waves w with s_{i-1} < B(w) <= s_i, i.e. [floor(s_{i-1}/q) + 1, floor(s_i/q)]
	// for a single quantum; buffer 0 takes w = 0.  One division per thread:
	// the starts grow along its buffers, so the next wave's boundary B(wn) is
	// stepped, not divided for (a 64-bit division per buffer, in a chain per
	// thread, cost the 8-buffer tiles ~0.4 us per buffer).
	uint64_t wn = ib == 0 ? 0 : xquant_wave(W, start - xp_cost(lp, routed && xp_long(lp))) + 1;
	const uint64_t ha = W.h * W.qa;
	auto bound = [&](uint64_t w) { return w < W.h ? w * W.qa : ha + (w - W.h) * W.qb; };
	uint64_t bn = bound(wn);
#pragma unroll
	for (uint32_t u = 0; u < kXPer; ++u) {
		const uint64_t i = ib + u;
		if (i < Q.count) {
			while (wn < Q.nwave && bn <= start) {
				Q.wave_first[wn] = i;
				bn = bound(++wn);
			}
			if (lg[u]) {
				const uint64_t pos = cbase[cl[u]] + rank[u];
				const uint64_t o = Q.offsets ? off[u] : i * Q.stride;
				Q.ents[pos] = XEnt{reinterpret_cast<uint64_t>(Q.base) + o, len[u], sdv[u], i};
			}
			start += cost[u];
			if (i + 1 == Q.count)  // waves whose first byte lies past the last buffer's start: none
				for (uint64_t w = wn; w <= Q.nwave; ++w) Q.wave_first[w] = Q.count;
		}
	}
}

// Workspace of the varlen path: the planner arrays, then (given more room)
// the long route's flags and entries.
struct XLayout {
	uint64_t tiles, tcns, tneed, tcls, wave_first, sh, flag, ents, base;
	uint64_t capS;
};
static uint64_t al64(uint64_t x) { return (x + 63) & ~uint64_t(63); }
static XLayout xlayout(uint64_t count, uint64_t nwave, uint64_t ws_bytes) {
	const uint64_t ntile = (count + 255) / 256;  // (the largest tile count: tiles of 256)
	XLayout L{};
	L.tiles = 0;
	L.tcns = al64(8 * (ntile + 2));
	L.tneed = al64(L.tcns + 8 * ntile);
	L.tcls = al64(L.tneed + 8 * ntile);
	L.wave_first = al64(L.tcls + 32 * ntile);
	L.sh = al64(L.wave_first + 8 * (nwave + 1) + 64);
	L.base = L.sh + 8 * kXShWords;
	// room: flags (1 B per buffer), then the entries
	const uint64_t fl = al64(count);
	uint64_t capS = ws_bytes > L.base + fl ? (ws_bytes - L.base - fl) / sizeof(XEnt) : 0;
	L.capS = capS;
	L.flag = L.base;
	L.ents = L.flag + fl;
	return L;
}

uint64_t xxh3_workspace_bytes(uint64_t count, uint64_t nwave) { return xlayout(count, nwave, 0).base; }
uint64_t xxh3_workspace_bytes_for(uint64_t count, uint64_t nwave, uint64_t long_blocks) {
	if (long_blocks == 0) return xxh3_workspace_bytes(count, nwave);
	// (a long buffer has more than 16 blocks)
	return xlayout(count, nwave, 0).base + al64(count) + sizeof(XEnt) * (long_blocks / 16 + 1);
}

int xxh3_blocks_per_cu() {
	static const int n = [] {
		int a = 0, b = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_xxh3<true>, 256, 0) != hipSuccess) a = 4;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_xxh3<false>, 256, 0) != hipSuccess) b = 4;
		int c = 0, d = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, k_xxh3_vrows<false>, 256, 0) != hipSuccess) c = 3;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&d, k_xxh3_vrows<true>, 256, 0) != hipSuccess) d = 3;
		int m = a < b ? a : b;
		m = m < c ? m : c;
		m = m < d ? m : d;
		return m < 1 ? 1 : m;
	}();
	return n;
}

int launch_xxh3(const XxhParams& P0, int num_cus, void* ws, hipStream_t stream) {
	XxhParams P = P0;
	const unsigned wpb = kWavesPerBlock;
	const uint64_t grid = (uint64_t)num_cus * xxh3_blocks_per_cu();
	const uint64_t nwave = grid * wpb;
	const uint64_t mis = (reinterpret_cast<uint64_t>(P.base) | (P.offsets ? 1 : P.stride));
	const bool aligned = (mis & 15) == 0;
	// the planner: varlen batches, and fixed-length long buffers given room for the long route
	const bool fixed_split = !P.offsets && ws && P.length > kXSplitMin;
	if (P.offsets || fixed_split) {
		// tiles of 256 buffers for small batches (more workgroups, short
		// per-thread chains), of 256 x kXPerBig past 256 such tiles (fewer
		// tiles to reduce: zipf's 1587 become 199, and k_xscan drops out)
		const bool big = P.count > 256 * kXFuseTiles;
		const uint64_t tile = big ? 256ull * kXPerBig : 256ull;
		const uint64_t ntile = (P.count + tile - 1) / tile;
		const XLayout L = xlayout(P.count, nwave, P.ws_bytes);
		uint8_t* w8 = static_cast<uint8_t*>(ws);
		XPlanP Q{};
		Q.lengths = P.lengths;
		Q.offsets = P.offsets;
		Q.seeds = P.seeds;
		Q.base = P.base;
		Q.stride = P.stride;
		Q.length = P.length;
		Q.count = P.count;
		Q.seed = P.seed;
		Q.tiles = reinterpret_cast<uint64_t*>(w8 + L.tiles);
		Q.tcns = reinterpret_cast<uint64_t*>(w8 + L.tcns);
		Q.tneed = reinterpret_cast<uint64_t*>(w8 + L.tneed);
		Q.tcls = reinterpret_cast<uint64_t*>(w8 + L.tcls);
		Q.sh = reinterpret_cast<uint64_t*>(w8 + L.sh);
		Q.flag = w8 + L.flag;
		Q.wave_first = reinterpret_cast<uint64_t*>(w8 + L.wave_first);
		Q.ntile = ntile;
		Q.nwave = nwave;
		Q.older = xxh3_blocks_per_cu() == 2 ? nwave / 2 : 0;
		Q.ents = reinterpret_cast<XEnt*>(w8 + L.ents);
		Q.capS = L.capS;
		Q.hneed = P.hneed;
		Q.dcount = P.d_count;
		if (!big) {
			k_xplan<1><<<(unsigned)ntile, 256, 0, stream>>>(Q);
			k_xassign<true, 1><<<(unsigned)ntile, 256, 0, stream>>>(Q);
		} else {
			k_xplan<kXPerBig><<<(unsigned)ntile, 256, 0, stream>>>(Q);
			if (ntile <= kXFuseTiles) {
				k_xassign<true, kXPerBig><<<(unsigned)ntile, 256, 0, stream>>>(Q);
			} else {
				k_xscan<<<1, 1024, 0, stream>>>(Q);
				k_xassign<false, kXPerBig><<<(unsigned)ntile, 256, 0, stream>>>(Q);
			}
		}
		if (L.capS) {
			XLong S{};
			S.sh = Q.sh;
			S.ents = Q.ents;
			S.out = P.out;
			S.seed = P.seed;
			S.err = P.err;
			launch_xxh3_long(S, num_cus, P.seeds != nullptr, stream);
		}
		// fixed-length long buffers whose entries all fit: the long route did them all
		if (fixed_split && L.capS >= P.count) return 0;
		P.wave_first = Q.wave_first;
		P.lflag = L.capS ? Q.flag : nullptr;
		if (P.seeds)
			k_xxh3_vrows<true><<<(unsigned)grid, 256, 0, stream>>>(P);
		else
			k_xxh3_vrows<false><<<(unsigned)grid, 256, 0, stream>>>(P);
		return 0;
	}
	if (!P.offsets && P.length > 240 && (mis & 7) == 0) {
		// fixed-length pages: four per wave in lockstep
		static const int rows_bpc = [] {
			int a = 0;
			if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_xxh3_rows<true>, 256, 0) != hipSuccess) a = 3;
			return a < 1 ? 1 : a;
		}();
		const uint64_t g2 = (uint64_t)num_cus * rows_bpc;
		P.ngen = (uint32_t)rows_bpc;
		if (P.seeds && aligned)
			k_xxh3_rows<true, false, true><<<(unsigned)g2, 256, 0, stream>>>(P);
		else if (P.seeds)
			k_xxh3_rows<true, false, false><<<(unsigned)g2, 256, 0, stream>>>(P);
		else if (aligned)
			k_xxh3_rows<false, false, true><<<(unsigned)g2, 256, 0, stream>>>(P);
		else
			k_xxh3_rows<false, false, false><<<(unsigned)g2, 256, 0, stream>>>(P);
	} else if (aligned)
		k_xxh3<true><<<(unsigned)grid, 256, 0, stream>>>(P);
	else
		k_xxh3<false><<<(unsigned)grid, 256, 0, stream>>>(P);
	return 0;
}

int launch_xxh3_pages_list(const XxhParams& P0, int num_cus, hipStream_t stream) {
	static const int bpc = [] {
		int a = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_xxh3_rows<false, true>, 256, 0) != hipSuccess) a = 3;
		return a < 1 ? 1 : a;
	}();
	const unsigned grid = (unsigned)((uint64_t)num_cus * bpc);
	const bool a16 = ((reinterpret_cast<uint64_t>(P0.base) | P0.stride) & 15) == 0;
	if (((reinterpret_cast<uint64_t>(P0.base) | P0.stride) & 7) != 0 || P0.length <= 240) return -1;
	XxhParams P = P0;
	P.ngen = (uint32_t)bpc;
	if (a16)
		k_xxh3_rows<false, true, true><<<grid, 256, 0, stream>>>(P);
	else
		k_xxh3_rows<false, true, false><<<grid, 256, 0, stream>>>(P);
	return 0;
}

// ---------------------------------------------------------------------------
// Short chains staged in LDS (round 6; xxh3_chain.hip's third route).  A chain
// of 2..kLChainSegs segments and at most kLChainMax bytes -- a packet over two
// or three PacketBuffers, FlowTransport.cpp:2025-2068 -- is hashed by one wave
// from LDS: its segments are read once, coalesced (16-byte loads at each
// segment's own alignment, 16-byte aligned LDS writes; the bytes of the chunks
// a segment boundary cuts one by one), and the one-wave long form (the block
// step of k_xxh3: lane = stripe x accumulator pair) or the short forms run
// over the LDS copy -- no staging area in HBM, so each byte crosses HBM once
// instead of three times (gather read + write, hash read).  Per wave the
// chains go through a three-stage pipeline: chain t+2's list entry (scalar
// loads), chain t+1's segment metadata and data loads in flight while chain t
// is hashed.
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* L, uint32_t o) {
	const uint32_t a = o >> 2;
	return __builtin_amdgcn_alignbyte(L[a + 1], L[a], o & 3u);
}
__device__ __forceinline__ uint64_t lds_u64(const uint32_t* L, uint32_t o) {
	const uint32_t a = o >> 2, w0 = L[a], w1 = L[a + 1], w2 = L[a + 2];
	return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, o & 3u) << 32) | __builtin_amdgcn_alignbyte(w1, w0, o & 3u);
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }
__device__ __forceinline__ uint32_t lds_u8(const uint32_t* L, uint32_t o) { return (L[o >> 2] >> (8 * (o & 3u))) & 255u; }
// The secret from an LDS copy (ks: the default secret's 24 words): kSec in
// constant memory is a global load, and one issued behind a chain's data loads
// waited for all of them (in-order vmcnt) before the hash could start.
__device__ __forceinline__ uint64_t ksec_l(const uint64_t* ks, int off) {
	const int j = off >> 3, r = off & 7;
	return r ? (ks[j] >> (8 * r)) | (ks[j + 1] << (64 - 8 * r)) : ks[j];
}
__device__ __forceinline__ uint64_t sec_word_l(const uint64_t* ks, int j, uint64_t seed) {
	const uint64_t w = ks[j];
	return (j & 1) ? w - seed : w + seed;
}
__device__ __forceinline__ uint64_t sec_at_l(const uint64_t* ks, int j, int r, uint64_t seed) {
	return (sec_word_l(ks, j, seed) >> (8 * r)) | (sec_word_l(ks, j + 1, seed) << (64 - 8 * r));
}
__device__ __forceinline__ Keys make_keys_l(const uint64_t* ks, int lane, uint64_t seed) {  // make_keys
	const int s = lane >> 2, k = lane & 3;
	Keys K;
	K.k0 = sec_word_l(ks, s + 2 * k, seed);
	K.k1 = sec_word_l(ks, s + 2 * k + 1, seed);
	K.l0 = sec_at_l(ks, 15 + 2 * k, 1, seed);
	K.l1 = sec_at_l(ks, 16 + 2 * k, 1, seed);
	K.c0 = sec_word_l(ks, 16 + 2 * k, seed);
	K.c1 = sec_word_l(ks, 17 + 2 * k, seed);
	K.g0 = sec_at_l(ks, 1 + 2 * k, 3, seed);
	K.g1 = sec_at_l(ks, 2 + 2 * k, 3, seed);
	return K;
}
__device__ __forceinline__ uint64_t mix16_lds(const uint64_t* ks, const uint32_t* L, uint32_t o, int soff, uint64_t seed) {
	return mulfold(lds_u64(L, o) ^ (ksec_l(ks, soff) + seed), lds_u64(L, o + 8) ^ (ksec_l(ks, soff + 8) - seed));
}
// xxh3_short over an LDS copy (xxhash.h:2734-2951)
__device__ uint64_t xxh3_short_lds(const uint64_t* ks, const uint32_t* L, uint32_t len, uint64_t seed) {
	if (len <= 16) {
		if (len > 8) {
			const uint64_t f1 = (ksec_l(ks, 24) ^ ksec_l(ks, 32)) + seed, f2 = (ksec_l(ks, 40) ^ ksec_l(ks, 48)) - seed;
			const uint64_t lo = lds_u64(L, 0) ^ f1, hi = lds_u64(L, len - 8) ^ f2;
			return xxh3_aval(len + __builtin_bswap64(lo) + hi + mulfold(lo, hi));
		}
		if (len >= 4) {
			const uint64_t s2 = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
			const uint32_t i1 = lds_u32(L, 0), i2 = lds_u32(L, len - 4);
			const uint64_t flip = (ksec_l(ks, 8) ^ ksec_l(ks, 16)) - s2;
			return rrmxmx(((uint64_t)i2 + ((uint64_t)i1 << 32)) ^ flip, len);
		}
		if (len) {
			const uint32_t c1 = lds_u8(L, 0), c2 = lds_u8(L, len >> 1), c3 = lds_u8(L, len - 1);
			const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
			return xxh64_aval((uint64_t)comb ^ ((uint64_t)((uint32_t)(ksec_l(ks, 0) ^ (ksec_l(ks, 4)))) + seed));
		}
		return xxh64_aval(seed ^ (ksec_l(ks, 56) ^ ksec_l(ks, 64)));
	}
	uint64_t acc = (uint64_t)len * P64_1;
	if (len <= 128) {
		const int pairs = (int)((len - 1) >> 5);
		for (int i = pairs; i >= 1; --i) {
			acc += mix16_lds(ks, L, 16 * i, 32 * i, seed);
			acc += mix16_lds(ks, L, len - 16 * (i + 1), 32 * i + 16, seed);
		}
		acc += mix16_lds(ks, L, 0, 0, seed);
		acc += mix16_lds(ks, L, len - 16, 16, seed);
		return xxh3_aval(acc);
	}
	const int rounds = (int)len / 16;
	for (int i = 0; i < 8; ++i) acc += mix16_lds(ks, L, 16 * i, 16 * i, seed);
	acc = xxh3_aval(acc);
	for (int i = 8; i < rounds; ++i) acc += mix16_lds(ks, L, 16 * i, 16 * (i - 8) + 3, seed);
	acc += mix16_lds(ks, L, len - 16, 136 - 17, seed);
	return xxh3_aval(acc);
}
}  // namespace

constexpr uint32_t kLcSlots = kLChainMax / 1024;  // 16-byte chunks per lane
__global__ __launch_bounds__(256) void k_xxh3_lchain(LChainP P) {
	__shared__ __attribute__((aligned(16))) uint32_t lbuf[4][kLChainMax / 4 + 16];
	__shared__ uint64_t ks[25];
	__shared__ uint32_t tcs[4][kLChainSegs], tend[4][kLChainSegs];  // per wave: the chain's segment table
	__shared__ uint64_t td[4][kLChainSegs];
	if (threadIdx.x < 25) ks[threadIdx.x] = threadIdx.x < 24 ? kSec[threadIdx.x] : 0;
	__syncthreads();
	const int lane = threadIdx.x & 63;
	const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint32_t* const L = lbuf[wv];
	typedef __attribute__((address_space(4))) const uint64_t k_u64;
	k_u64* const lst = (k_u64*)P.list;  // written by k_chain_ranges (an earlier launch): scalar loads
	// this XCD's list (workgroup b runs on XCD b % 8; k_chain_ranges appended
	// to the list of its own), strided over the XCD's waves
	const uint32_t x = blockIdx.x & 7;
	const uint64_t nx = ((k_u64*)P.counts)[16 * x];
	const uint64_t wx = (uint64_t)(blockIdx.x >> 3) * 4 + wv, nwx = (uint64_t)(gridDim.x >> 3) * 4;
	if (wx >= nx) return;
	k_u64* const lx = lst + 2 * P.lcap * x;
	const uint64_t dummy = reinterpret_cast<uint64_t>(P.list);  // 16 readable bytes
	const uint64_t base = reinterpret_cast<uint64_t>(P.base);

	// chain t's list entry: chain index, first segment, segment count
	uint64_t ec1 = 0, es1 = 0;
	uint32_t en1 = 0;
	// List entries and seeds by vector loads (every lane the same address),
	// issued a chain ahead of their use and ahead of the data loads of the
	// chain in flight, so that reading them waits for nothing: a scalar load
	// is waited for at the next LDS wait (lgkmcnt counts both), one read at
	// its use held up the metadata loads behind it every chain.
	typedef uint64_t u64x2e __attribute__((ext_vector_type(2)));
	typedef __attribute__((address_space(1))) const u64x2e g_u64x2e;
	const uint64_t lgx = reinterpret_cast<uint64_t>(P.list + 2 * P.lcap * x);  // (16-byte aligned entries)
	u64x2e eraw = u64x2e{0, 0};
	auto entry_load = [&](uint64_t i) { eraw = *(g_u64x2e*)(lgx + 16 * i); };
	auto entry_take = [&](uint64_t& c, uint64_t& s0, uint32_t& ns) {
		const uint64_t a = rdfirst64v(eraw[0]), b = rdfirst64v(eraw[1]);
		c = a;
		s0 = b & ((1ull << 56) - 1);
		ns = (uint32_t)(b >> 56);
	};
	auto seed_load = [&](uint64_t c) -> uint64_t { return P.seeds ? P.seeds[c] : P.seed; };
	// segment metadata in lanes 0 .. ns-1
	uint64_t moff = 0;
	uint32_t mlen = 0;
	auto meta_issue = [&](uint64_t s0, uint32_t ns) {
		const uint64_t j = s0 + ((uint32_t)lane < ns ? (uint32_t)lane : 0u);
		moff = P.seg_off[j];
		mlen = reinterpret_cast<const uint32_t*>(P.seg_len)[2 * j];  // (the low word: a chain here is under 2^14 bytes; a dead high word's load held up the register's next use)
	};
	// The geometry derived from the metadata: per segment its chain offset, end
	// and source displacement (address - chain offset) as LDS tables of the
	// wave, read by segment index -- a position's segment is a count over the
	// segment starts held in SGPRs (selecting each field over the segments in
	// SGPRs cost ~90 instructions per chunk, a chunk -> segment map in LDS its
	// byte writes).
	uint32_t gns = 0, gL = 0;
	uint32_t gst[kLChainSegs];  // [1 ..]: segment starts (past the chain: ~0)
	auto seg_of = [&](uint32_t pos) {
		uint32_t j = 0;
#pragma unroll
		for (uint32_t k = 1; k < kLChainSegs; ++k) j += gst[k] <= pos ? 1u : 0u;
		return j;
	};
	auto geometry = [&](uint32_t ns) {
		uint32_t len = (uint32_t)lane < ns ? mlen : 0u;  // (a chain of this route is under 2^14 bytes)
		uint32_t inc = len;
#pragma unroll
		for (int d = 1; d < (int)kLChainSegs; d <<= 1) {
			const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((lane - d) << 2, (int)inc);
			inc += lane >= d ? y : 0u;
		}
		const uint32_t cs = inc - len;
		gns = ns;
		gL = rdlane(inc, (int)kLChainSegs - 1);
		if ((uint32_t)lane < kLChainSegs) {
			tcs[wv][lane] = cs;
			tend[wv][lane] = inc;
			td[wv][lane] = moff - cs;
		}
		// the segment starts (but the first) in SGPRs: a position's segment is
		// the count of starts at or below it (a chunk map in LDS cost its byte
		// writes: 70 us of the bench's step)
#pragma unroll
		for (uint32_t j = 1; j < kLChainSegs; ++j) gst[j] = j < ns ? rdlane(cs, (int)j) : 0xFFFFFFFFu;
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	};
	// data loads: 16-byte chunk q = lane + 64 r of the chain (full chunks), and
	// the bytes of the chunks a boundary cuts (items lane, lane + 64: boundary
	// p = item / 16 -- segment p's end --, byte item % 16 of its chunk)
	typedef __attribute__((address_space(1))) const u64x2u g_u64x2u_;
	u64x2u R[kLcSlots];
	uint32_t full = 0;  // bit r: slot r is a full chunk
	uint32_t bv[2], bo[2];
	bool bon[2];
	auto data_issue = [&]() {
		const uint32_t nr = (gL + 1023) >> 10;
		full = 0;
#pragma unroll
		for (uint32_t r = 0; r < kLcSlots; ++r) {
			if (r < nr) {
				const uint32_t q16 = 16u * ((uint32_t)lane + 64u * r);
				const uint32_t j = seg_of(q16);
				const uint64_t d = td[wv][j];
				const uint32_t e = tend[wv][j];
				const bool f = q16 < gL && q16 + 16u <= e;  // (e <= gL)
				full |= f ? 1u << r : 0u;
				R[r] = __builtin_nontemporal_load((g_u64x2u_*)(f ? base + d + q16 : dummy));
			}
		}
#pragma unroll
		for (int v = 0; v < 2; ++v) {
#ifdef FDBXXH_LC_NOBYTES
			bon[v] = false;  // timing experiment: no cut bytes (wrong results)
			continue;
#endif
			const uint32_t it = (uint32_t)lane + 64u * v, p = it >> 4;
			const uint32_t bp = tend[wv][p & (kLChainSegs - 1)];
			const uint32_t e = (bp & ~15u) + (it & 15u);
			const bool on = p < gns && (bp & 15u) != 0 && e < gL;
			const uint32_t j = seg_of(e);  // (e < gL: a segment of the chain)
			const uint64_t a = on ? base + td[wv][j] + e : dummy;
			bon[v] = on;
			bo[v] = e | ((uint32_t)a & 3u) << 16;  // (the byte's place in its dword, extracted at the commit)
			typedef __attribute__((address_space(1))) const uint32_t g_u32_;
			bv[v] = *((g_u32_*)(a & ~3ull));  // (a dword holding a wanted byte never crosses a page)
		}
	};
	auto data_commit = [&]() {
		const uint32_t nr = (gL + 1023) >> 10;
#pragma unroll
		for (uint32_t r = 0; r < kLcSlots; ++r)
#ifdef FDBXXH_LC_NOCOMMIT
			if (r == 99) {  // timing experiment: no stage writes (wrong results)
#else
			if (r < nr && (full >> r & 1u)) {
#endif
				typedef uint64_t u64x2a __attribute__((ext_vector_type(2)));
				*reinterpret_cast<u64x2a*>(L + 4u * ((uint32_t)lane + 64u * r)) = u64x2a{R[r][0], R[r][1]};
			}
#pragma unroll
		for (int v = 0; v < 2; ++v)
			if (bon[v]) reinterpret_cast<uint8_t*>(L)[bo[v] & 0xFFFFu] = (uint8_t)(bv[v] >> (8 * (bo[v] >> 16)));
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	};

	// prologue: the first chain's geometry and data in flight, the second one's
	// entry, seed and metadata, the third one's entry
	uint64_t c0, s00;
	uint32_t n0;
	entry_load(wx);
	entry_take(c0, s00, n0);
	uint64_t sdr0 = seed_load(c0), sdr1 = 0;  // (vector: read a chain later)
	meta_issue(s00, n0);
	geometry(n0);
	uint64_t i1 = wx + nwx;
	if (i1 < nx) {
		entry_load(i1);
		entry_take(ec1, es1, en1);
		sdr1 = seed_load(ec1);
		meta_issue(es1, en1);
		if (i1 + nwx < nx) entry_load(i1 + nwx);
	}
	data_issue();
	for (uint64_t i = wx; i < nx; i += nwx) {
		const uint32_t len = gL;
		const uint64_t c = c0;
		data_commit();  // this chain in LDS (its data were the last loads issued)
		const uint64_t sd = rdfirst64v(sdr0);  // (issued before that data)
		// the next chain: its geometry, then its data in flight while this one is
		// hashed; the one after: its seed and metadata, then the entry after that
		if (i1 < nx) {
			c0 = ec1;
			sdr0 = sdr1;
			geometry(en1);
			i1 += nwx;
			if (i1 < nx) {
				entry_take(ec1, es1, en1);
				sdr1 = seed_load(ec1);
				meta_issue(es1, en1);
				if (i1 + nwx < nx) entry_load(i1 + nwx);
			}
			data_issue();
		}
		uint64_t h;
#ifdef FDBXXH_LC_NOHASH
		if (len != 0x7fffffff) {  // timing experiment: no hash (wrong results)
			h = L[lane];
		} else
#endif
		if (len <= 240) {
			h = xxh3_short_lds(ks, L, len, sd);
		} else {
			const Keys K = make_keys_l(ks, lane, sd);
			Acc A = acc_init(lane);
			const uint32_t nfull = (len - 1) >> 10, ns = ((len - 1) - (nfull << 10)) >> 6;
			for (uint32_t b = 0; b < nfull; ++b) {
				typedef uint64_t u64x2a __attribute__((ext_vector_type(2)));
				const u64x2a v = *reinterpret_cast<const u64x2a*>(L + 256u * b + 4u * (uint32_t)lane);
				block_step(A, v[0], v[1], K.k0, K.k1, true);
				scramble(A, K);
			}
			const bool last = lane >= 60;
			const uint32_t o = last ? len - 64u + 16u * (uint32_t)(lane - 60) : (nfull << 10) + 16u * (uint32_t)lane;
			const uint64_t v0 = lds_u64(L, o), v1 = lds_u64(L, o + 8);
			block_step(A, v0, v1, last ? K.l0 : K.k0, last ? K.l1 : K.k1, last || (uint32_t)lane < 4 * ns);
			h = merge(A, K, len, lane);
		}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();  // (every lane's LDS reads before the next chain's writes)
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		if (lane == 0) P.out[c] = h;
	}
}

int launch_xxh3_lchain(const LChainP& P, int num_cus, hipStream_t stream) {
	k_xxh3_lchain<<<(unsigned)(8 * ((2 * num_cus + 7) / 8)), 256, 0, stream>>>(P);  // (a multiple of 8: the XCD lists)
	return 0;
}

}  // namespace fdbxxh

#ifdef FDBXXH_TIMES
extern "C" int fdbxxh_debug_times(void* host, uint64_t nwave) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbxxh::g_vt), nwave * 32, 0, hipMemcpyDeviceToHost);
}
#endif
