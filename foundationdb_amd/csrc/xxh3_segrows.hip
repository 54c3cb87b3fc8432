// XXH3-64 of a chain of segments IN PLACE: a packet laid over a PacketBuffer
// chain (fdbrpc/FlowTransport.cpp:2025-2068: XXH3_64bits_reset, _update per
// buffer, _digest), hashed where its segments lie instead of gathered into a
// staging area first (xxh3_chain.hip used to copy every multi-segment chain:
// twice its bytes through HBM, 411 of the 0.72 ms bench step).
//
// One 16-lane ROW per chain.  XXH3's long form (xxhash.h:3641-3718, 192-byte
// secret: 1 KiB blocks of 16 stripes, the 8 accumulators scrambled after each
// block, the last stripe at len - 64, then the merge) with the row layout of
// the page kernels (xxh3_kernels.hip k_xxh3_rows): lane (g, k), g = lane / 4,
// k = lane % 4, takes stripe 4q + g of quarter q of every block for the
// accumulator pair k, so one load instruction reads 256 contiguous logical
// bytes per row; the four g lanes of a pair add with two DPP row rotates.
// A 16-byte chunk at logical offset o is loaded from the segment holding it
// (each lane walks the chain's segment table, kept in LDS, forward only); a
// chunk that straddles a segment end is assembled byte by byte (a few per
// chain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xxh3_device.h"

namespace fdbxxh {

namespace {

// The default secret as little-endian u64 words (xxhash.h:2500-2511, algorithm constant).
__constant__ uint64_t kSegSec[24] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
    0xcb00c391bb52283cull, 0xa32e531b8b65d088ull, 0x4ef90da297486471ull, 0xd8acdea946ef1938ull,
    0x3f349ce33f76faa8ull, 0x1d4f0bc7c7bbdcf9ull, 0x3159b4cd4be0518aull, 0x647378d9c97e9fc8ull,
    0xc3ebd33483acc5eaull, 0xeb6313faffa081c5ull, 0x49daf0b751dd0d17ull, 0x9e68d429265516d3ull,
    0xfca1477d58be162bull, 0xce31d07ad1b8f88full, 0x280416958f3acb45ull, 0x7e404bbbcafbd7afull,
};
constexpr uint64_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint64_t sr_mulfold(uint64_t a, uint64_t b) { return a * b ^ __umul64hi(a, b); }
__device__ __forceinline__ uint64_t sr_aval(uint64_t h) {  // xxhash.h:2680-2685
	h ^= h >> 37;
	h *= 0x165667919E3779F9ull;
	return h ^ (h >> 32);
}
// Word j of the secret for `seed` (the custom secret of XXH3_64bits_withSeed,
// xxhash.h:3550-3566: +seed on the low word of each 16-byte pair, -seed on the high).
__device__ __forceinline__ uint64_t sr_word(uint32_t j, uint64_t seed) {
	return (j & 1) ? kSegSec[j] - seed : kSegSec[j] + seed;
}
// Secret bytes [off, off + 8) for `seed`, any offset.
__device__ __forceinline__ uint64_t sr_sec(uint32_t off, uint64_t seed) {
	const uint32_t w = off >> 3, s = (off & 7) * 8;
	const uint64_t a = sr_word(w, seed);
	return s ? (a >> s) | (sr_word(w + 1, seed) << (64 - s)) : a;
}
// Sum over the four lanes of the row with the same k (lanes k, k+4, k+8, k+12).
__device__ __forceinline__ uint64_t sr_rowsum(uint64_t v) {
	uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
	uint32_t l2 = __builtin_amdgcn_update_dpp(0u, lo, 0x124, 0xF, 0xF, false);  // row_ror:4
	uint32_t h2 = __builtin_amdgcn_update_dpp(0u, hi, 0x124, 0xF, 0xF, false);
	uint64_t s = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2);
	lo = (uint32_t)s;
	hi = (uint32_t)(s >> 32);
	l2 = __builtin_amdgcn_update_dpp(0u, lo, 0x128, 0xF, 0xF, false);  // row_ror:8
	h2 = __builtin_amdgcn_update_dpp(0u, hi, 0x128, 0xF, 0xF, false);
	return s + (((uint64_t)h2 << 32) | l2);
}

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4u g_u32x4u;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

}  // namespace

// Per row: its chain's segments in LDS (logical start, address, end).
struct SegEnt {
	uint64_t ls, a, le;
};

template <bool SEEDED>
__global__ __launch_bounds__(256) void k_xxh3_segrows(SegRowsP P) {
	__shared__ SegEnt st[256 / 16][kSegRowsMax];
	const uint32_t lane = threadIdx.x & 63, r = lane & 15, g = r >> 2, k = r & 3;
	const uint32_t row = threadIdx.x >> 4;
	const uint64_t nrow = (uint64_t)gridDim.x * (blockDim.x >> 4);
	SegEnt* const tab = st[row];
	for (uint64_t c0 = (uint64_t)blockIdx.x * (blockDim.x >> 4); c0 < P.nchains; c0 += nrow) {
		const uint64_t c = c0 + row;
		const bool on = c < P.nchains && P.flag[c] == 2;  // (k_chain_ranges: 2 = hashed here)
		uint64_t s0 = 0, ns = 0;
		if (on) {
			s0 = P.starts[c];
			ns = P.starts[c + 1] - s0;
		}
		// the segment table: lane r < ns holds segment s0 + r; logical starts by a row prefix
		uint64_t so = 0, sl = 0;
		if (on && r < ns) {
			so = P.seg_off[s0 + r];
			sl = P.seg_len[s0 + r];
		}
		uint64_t pre = sl;
#pragma unroll
		for (int d = 1; d < 16; d <<= 1) {
			const uint64_t y = __shfl_up(pre, d, 16);
			pre += r >= (uint32_t)d ? y : 0;
		}
		const uint64_t L = __shfl(pre, 15, 16);  // the chain's length (lanes past ns add 0)
		if (on && r < ns) tab[r] = SegEnt{pre - sl, reinterpret_cast<uint64_t>(P.base) + so, pre};
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_s_waitcnt(0xC07F);  // (lgkmcnt(0): the table is written before any lane reads it)
		if (!on) continue;
		const uint64_t sd = SEEDED ? (P.seeds ? P.seeds[c] : P.seed) : 0;
		// this lane's segment cursor (forward only)
		uint32_t sj = 0;
		SegEnt cur = tab[0];
		auto seek = [&](uint64_t o) {
			while (o >= cur.le && sj + 1 < ns) cur = tab[++sj];
		};
		// 16 logical bytes at o as two little-endian words
		auto load16 = [&](uint64_t o, uint64_t& w0, uint64_t& w1) {
			seek(o);
			if (o + 16 <= cur.le) {
				const u32x4u v = *((g_u32x4u*)(cur.a + (o - cur.ls)));
				w0 = ((uint64_t)v[1] << 32) | v[0];
				w1 = ((uint64_t)v[3] << 32) | v[2];
				return;
			}
			// straddles a segment end: byte by byte, on its own cursor
			uint32_t j = sj;
			SegEnt e = cur;
			uint64_t b[2] = {0, 0};
			for (uint32_t t = 0; t < 16; ++t) {
				while (o + t >= e.le && j + 1 < ns) e = tab[++j];
				const uint64_t x = *((g_u8*)(e.a + (o + t - e.ls)));
				b[t >> 3] |= x << (8 * (t & 7));
			}
			w0 = b[0];
			w1 = b[1];
		};
		uint64_t a0 = k == 0 ? P32_3 : k == 1 ? P64_2 : k == 2 ? P64_4 : P64_5;  // acc[2k]
		uint64_t a1 = k == 0 ? P64_1 : k == 1 ? P64_3 : k == 2 ? P32_2 : P32_1;  // acc[2k + 1]
		// keys of the lane's four stripes 4q + g, words 2k, 2k + 1: secret + 8(4q + g) + 16k
		uint64_t kq0[4], kq1[4];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			kq0[q] = sr_word(4 * q + g + 2 * k, sd);
			kq1[q] = sr_word(4 * q + g + 2 * k + 1, sd);
		}
		auto stripe = [&](uint64_t& s0w, uint64_t& s1w, uint64_t v0, uint64_t v1, uint64_t k0, uint64_t k1) {
			const uint64_t x0 = v0 ^ k0, x1 = v1 ^ k1;
			s0w += v1 + (uint64_t)(uint32_t)x0 * (x0 >> 32);
			s1w += v0 + (uint64_t)(uint32_t)x1 * (x1 >> 32);
		};
		const uint64_t nb = (L - 1) >> 10;  // full blocks (L > 240 here)
		for (uint64_t b = 0; b < nb; ++b) {
			uint64_t v[4][2];
#pragma unroll
			for (uint32_t q = 0; q < 4; ++q) load16(1024 * b + 256 * q + 64 * g + 16 * k, v[q][0], v[q][1]);
			uint64_t s0w = 0, s1w = 0;
#pragma unroll
			for (uint32_t q = 0; q < 4; ++q) stripe(s0w, s1w, v[q][0], v[q][1], kq0[q], kq1[q]);
			a0 += sr_rowsum(s0w);
			a1 += sr_rowsum(s1w);
			// scramble (xxhash.h:3490-3503): secret + 128 + 16k
			a0 = (a0 ^ (a0 >> 47) ^ sr_word(16 + 2 * k, sd)) * P32_1;
			a1 = (a1 ^ (a1 >> 47) ^ sr_word(17 + 2 * k, sd)) * P32_1;
		}
		// the last block's whole stripes, then the last stripe at L - 64 (secret + 121)
		const uint64_t nst = ((L - 1) - 1024 * nb) >> 6;
		{
			uint64_t s0w = 0, s1w = 0;
#pragma unroll
			for (uint32_t q = 0; q < 4; ++q) {
				const uint32_t s = 4 * q + g;
				if (s < nst) {
					uint64_t v0, v1;
					load16(1024 * nb + 64 * s + 16 * k, v0, v1);
					stripe(s0w, s1w, v0, v1, kq0[q], kq1[q]);
				}
			}
			if (g == 0) {
				uint64_t v0, v1;
				sj = 0;
				cur = tab[0];
				load16(L - 64 + 16 * k, v0, v1);
				stripe(s0w, s1w, v0, v1, sr_sec(121 + 16 * k, sd), sr_sec(129 + 16 * k, sd));
			}
			a0 += sr_rowsum(s0w);
			a1 += sr_rowsum(s1w);
		}
		// merge (xxhash.h:3678-3700): L * P64_1 + sum over the pairs of mulfold(acc ^ secret + 11 + 16k)
		uint64_t m = sr_mulfold(a0 ^ sr_sec(11 + 16 * k, sd), a1 ^ sr_sec(19 + 16 * k, sd));
		m += __shfl_xor(m, 1, 16);
		m += __shfl_xor(m, 2, 16);
		if (r == 0) P.out[c] = sr_aval(L * P64_1 + m);
	}
}

int launch_xxh3_segrows(const SegRowsP& P, int num_cus, hipStream_t stream) {
	if (P.nchains == 0) return 0;
	const uint64_t rows = (P.nchains + 15) / 16 * 16;
	uint64_t grid = (rows + 15) / 16;  // 16 rows per 256-thread workgroup
	const uint64_t cap = (uint64_t)num_cus * 32;
	if (grid > cap) grid = cap;
	if (P.seeds || P.seed)
		k_xxh3_segrows<true><<<(unsigned)grid, 256, 0, stream>>>(P);
	else
		k_xxh3_segrows<false><<<(unsigned)grid, 256, 0, stream>>>(P);
	return 0;
}

}  // namespace fdbxxh
