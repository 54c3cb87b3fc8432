// Split XXH3-64 route for LONG buffers (gfx950): xxHash v0.8.0
// XXH3_64bits[_withSeed] (flow/include/flow/xxhash.h:3641-3718, 3800-3837)
// of buffers longer than kXSplitMin, bit-identical, with the work of one
// buffer spread over the whole GPU.
//
// A long input accumulates 64-byte stripes into eight 64-bit lanes and
// scrambles them after every 1 KiB block.  The accumulation of one block is a
// SUM (per lane, mod 2^64) of its stripes' contributions -- the block's STRIPE
// SUM D[b] does not depend on the accumulators -- and only the scramble is
// sequential:
//     acc <- scramble(acc + D[b])  for b < nfull = (len - 1) >> 10
//     acc <- acc + D[nfull]        (the last block's stripes + the last stripe)
//     hash = mergeAccs(acc, secret + 11, len * PRIME64_1)
// (tests/xxh3_split_model.py restates this and checks it against the oracle.)
//
//   phase A  k_xsplit_a: every block of every long buffer as one flat stream
//            (D order, PIECES of 64 consecutive blocks of one buffer carry the
//            metadata), an equal share of blocks per wave; the row layout of k_xxh3_rows (a 16-lane row per
//            block: four coalesced 256-byte loads, 32x32->64 products, two DPP
//            row rotates) writes D[b] (64 B per KiB) to the workspace.
//   phase B  k_xsplit_b: one wave per long buffer: 4 KiB of stripe sums per
//            round by LDS-DMA (the next round in flight), eight chain lanes
//            (one accumulator each), one scramble per block, the merge.
// The planner (xxh3_kernels.hip: k_xplan / k_xscan / k_xassign) picks the
// long buffers, lays out the pieces and D in buffer order, divides D among
// phase A's waves, and takes the long buffers off the row kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xxh3_device.h"

namespace fdbxxh {

namespace {

constexpr uint64_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;

// The default secret as 24 little-endian words (xxhash.h:2500-2511).
__constant__ uint64_t kSecS[24] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
    0xcb00c391bb52283cull, 0xa32e531b8b65d088ull, 0x4ef90da297486471ull, 0xd8acdea946ef1938ull,
    0x3f349ce33f76faa8ull, 0x1d4f0bc7c7bbdcf9ull, 0x3159b4cd4be0518aull, 0x647378d9c97e9fc8ull,
    0xc3ebd33483acc5eaull, 0xeb6313faffa081c5ull, 0x49daf0b751dd0d17ull, 0x9e68d429265516d3ull,
    0xfca1477d58be162bull, 0xce31d07ad1b8f88full, 0x280416958f3acb45ull, 0x7e404bbbcafbd7afull,
};

// Word j of the secret for `seed` (xxhash.h:3550-3566: +seed / -seed per word).
__device__ __forceinline__ uint64_t swd(int j, uint64_t seed) {
	const uint64_t w = kSecS[j];
	return (j & 1) ? w - seed : w + seed;
}
// Secret bytes [8j + r, 8j + r + 8), 0 < r < 8.
__device__ __forceinline__ uint64_t sat(int j, int r, uint64_t seed) {
	return (swd(j, seed) >> (8 * r)) | (swd(j + 1, seed) << (64 - 8 * r));
}

template <int CTRL>
__device__ __forceinline__ void add_dpp(uint32_t& lo, uint32_t& hi) {
	const uint32_t l2 = __builtin_amdgcn_update_dpp(0u, lo, CTRL, 0xF, 0xF, false);
	const uint32_t h2 = __builtin_amdgcn_update_dpp(0u, hi, CTRL, 0xF, 0xF, false);
	const uint64_t s = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2);
	lo = (uint32_t)s;
	hi = (uint32_t)(s >> 32);
}

__device__ __forceinline__ uint64_t rdf64(uint64_t v) {
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}

typedef uint64_t u64x2u __attribute__((ext_vector_type(2), aligned(1)));
typedef __attribute__((address_space(1))) const u64x2u g_u64x2u;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u64x2 g_u64x2;
typedef __attribute__((address_space(1))) u64x2 gw_u64x2;
typedef __attribute__((address_space(1))) const uint64_t g_u64;

__device__ __forceinline__ uint64_t gld64(const uint64_t* p) { return *((g_u64*)reinterpret_cast<uintptr_t>(p)); }
// A piece's metadata through the scalar cache (constant address space, a
// wave-uniform address: s_load, counted by lgkmcnt): as a vector load it
// would sit in the data loads' in-order vmcnt queue, and every piece change
// would wait for the blocks in flight.  The planner wrote the pieces in an
// earlier launch; nothing in this one writes them.
typedef __attribute__((address_space(4))) const uint64_t c_u64;
__device__ __forceinline__ XPiece ld_piece(const XPiece* pcs, uint64_t i) {
	static_assert(sizeof(XPiece) == 48, "six words");
	const c_u64* q = (const c_u64*)reinterpret_cast<uintptr_t>(pcs + i);
	XPiece r;
	r.p = q[0];
	r.len = q[1];
	r.d = q[2];
	r.seed = q[3];
	const uint64_t w = q[4];
	r.b0 = (uint32_t)w;
	r.nb = (uint32_t)(w >> 32);
	r.pad = 0;
	return r;
}

}  // namespace

// ---------------------------------------------------------------------------
// Phase A: stripe sums, an equal share of D's blocks per wave (pieces of 64
// blocks per wave measured 13 % of imbalance on the chunks batch: ~6 pieces
// per wave, a third of them partial).
// Lane (r, g, k) = (lane / 16, (lane % 16) / 4, lane % 4): row r takes block
// b + r of a STEP (four consecutive blocks of one piece), stripes g, g+4,
// g+8, g+12 for accumulator pair k.  The row sums close with two DPP row
// rotates, after which every lane of a row holds its pair's sums; a step's
// sums stay in the lanes with g == step % 4 and leave in bursts (kXGroup).
// ---------------------------------------------------------------------------
struct AStep {
	uint64_t v[4][2];
	uint64_t p, len, seed, d;  // the piece's buffer; d: flat index of row 0's block
	uint32_t b, nrows;         // row 0's block in the buffer; rows in use (0: idle step)
};

template <bool SEEDS>
__global__ __launch_bounds__(256) void k_xsplit_a(XSplit S) {
	const uint64_t npc = rdf64(gld64(S.sh + 2));
	if (npc == 0) return;  // no long buffer this batch
	const int lane = threadIdx.x & 63;
	const int r = lane >> 4, l = lane & 15, k = l & 3, g = l >> 2;
	const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	if (w >= S.nwa) return;
	// this wave's share of D: blocks [w*pb, min((w+1)*pb, total)), starting at
	// block `a & 63` of piece `a >> 6` (the planner, k_xassign)
	const uint64_t a = rdf64(gld64(S.astart + w));
	if (a == ~0ull) return;
	const uint64_t tb = rdf64(gld64(S.sh + 1)), pb = rdf64(gld64(S.sh + 3));
	const uint64_t fb1 = (w + 1) * pb < tb ? (w + 1) * pb : tb;
	const XPiece* __restrict__ pcs = S.pcs;
	// load cursor: piece lq (metadata in Lm) at block lpos of it, rem blocks of
	// the share left; the next piece's metadata (scalar loads, lgkmcnt: off the
	// data loads' vmcnt queue)
	uint64_t lq = a >> 6, rem = fb1 - w * pb;
	uint32_t lpos = (uint32_t)(a & 63);
	XPiece Lm = ld_piece(pcs, rdf64(lq));
	XPiece Nm = ld_piece(pcs, rdf64(lq + 1 < npc ? lq + 1 : lq));
	const uint64_t idle_p = Lm.p;  // an idle step reads the share's first block again (discarded)
	auto load = [&](AStep& St) __attribute__((always_inline)) {
		if (rem != 0) {
			St.p = Lm.p;
			St.len = Lm.len;
			St.seed = Lm.seed;
			St.b = Lm.b0 + lpos;
			St.d = Lm.d + lpos;
			uint32_t n = Lm.nb - lpos < 4 ? Lm.nb - lpos : 4;
			n = rem < n ? (uint32_t)rem : n;
			St.nrows = n;
			lpos += n;
			rem -= n;
			if (lpos >= Lm.nb && rem != 0) {
				++lq;
				lpos = 0;
				Lm = Nm;
				Nm = ld_piece(pcs, rdf64(lq + 1 < npc ? lq + 1 : lq));
			}
		} else {
			St.p = idle_p;
			St.len = 1025;
			St.seed = 0;
			St.b = 0;
			St.d = 0;
			St.nrows = 0;
		}
		const uint32_t rr = (uint32_t)r < St.nrows ? (uint32_t)r : 0u;  // rows past the piece: row 0's block
		const uint64_t blk = St.b + rr;
		const uint64_t nfull = (St.len - 1) >> 10;
		const uint32_t ns = (uint32_t)(((St.len - 1) - (nfull << 10)) >> 6);
		const bool fin = blk == nfull;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool tail = fin && (s == 15 || s >= ns);
			const uint64_t a = tail ? St.p + St.len - 64 + 16 * k : St.p + (blk << 10) + 64 * s + 16 * k;
			const u64x2u x = __builtin_nontemporal_load((g_u64x2u*)a);
			St.v[i][0] = x[0];
			St.v[i][1] = x[1];
		}
	};
	// keys of the current seed: stripe g + 4i (secret + 8s + 16k), last stripe (secret + 121 + 16k)
	uint64_t k0[4], k1[4], l0, l1, kseed = S.seed;
	auto keys = [&](uint64_t sd) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			k0[i] = swd(g + 4 * i + 2 * k, sd);
			k1[i] = swd(g + 4 * i + 2 * k + 1, sd);
		}
		l0 = sat(15 + 2 * k, 1, sd);
		l1 = sat(16 + 2 * k, 1, sd);
	};
	keys(kseed);
	// saved sums: lane (r, g, k) keeps the sums of row r, pair k of steps
	// g, g + 4, g + 8, g + 12 of a group of kXGroup steps, which leave together
	// as kXGroup / 4 16-byte stores per lane.  A store holds up the next wait on
	// the data loads issued after it (vmcnt counts stores and loads in issue
	// order) until it has reached memory, which under the read stream takes
	// several us: one store per four steps cost phase A ~25 % (212 -> 162 us
	// without the stores on the chunks batch), so they go out in bursts.
	constexpr uint32_t kXGroup = 16;
	uint64_t e0[kXGroup / 4], e1[kXGroup / 4], ei[kXGroup / 4];
	bool ev[kXGroup / 4];
#pragma unroll
	for (uint32_t j = 0; j < kXGroup / 4; ++j) {
		e0[j] = e1[j] = ei[j] = 0;
		ev[j] = false;
	}
	uint32_t slot = 0;  // steps saved since the last store (uniform)
	uint64_t* __restrict__ D = S.D;
	auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
		for (uint32_t j = 0; j < kXGroup / 4; ++j) {
			if (ev[j]) *((gw_u64x2*)reinterpret_cast<uintptr_t>(D + 8 * ei[j] + 2 * k)) = u64x2{e0[j], e1[j]};
			ev[j] = false;
		}
	};
	auto compute = [&](const AStep& St) __attribute__((always_inline)) {
		if (St.nrows == 0) return;
		if (SEEDS && St.seed != kseed) {
			kseed = St.seed;
			keys(kseed);
		}
		const uint64_t blk = St.b + r;
		const uint64_t nfull = (St.len - 1) >> 10;
		const uint32_t ns = (uint32_t)(((St.len - 1) - (nfull << 10)) >> 6);
		const bool fin = blk == nfull;
		uint64_t d0 = 0, d1 = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool last = fin && s == 15;
			const bool on = !fin || s < ns || last;
			const uint64_t x0 = St.v[i][0] ^ (last ? l0 : k0[i]);
			const uint64_t x1 = St.v[i][1] ^ (last ? l1 : k1[i]);
			const uint64_t c0 = St.v[i][1] + (uint64_t)(uint32_t)x0 * (x0 >> 32);
			const uint64_t c1 = St.v[i][0] + (uint64_t)(uint32_t)x1 * (x1 >> 32);
			d0 += on ? c0 : 0;
			d1 += on ? c1 : 0;
		}
		uint32_t lo0 = (uint32_t)d0, hi0 = (uint32_t)(d0 >> 32), lo1 = (uint32_t)d1, hi1 = (uint32_t)(d1 >> 32);
		add_dpp<0x124>(lo0, hi0);  // row_ror:4
		add_dpp<0x124>(lo1, hi1);
		add_dpp<0x128>(lo0, hi0);  // row_ror:8
		add_dpp<0x128>(lo1, hi1);
#pragma unroll
		for (uint32_t j = 0; j < kXGroup / 4; ++j)
			if ((slot >> 2) == j && (uint32_t)g == (slot & 3)) {
				e0[j] = ((uint64_t)hi0 << 32) | lo0;
				e1[j] = ((uint64_t)hi1 << 32) | lo1;
				ei[j] = St.d + r;
				ev[j] = (uint32_t)r < St.nrows;
			}
		if (++slot == kXGroup) {
			flush();
			slot = 0;
		}
	};
	AStep s0, s1, t0, t1;
#pragma unroll
	for (int i = 0; i < 4; ++i) s0.v[i][0] = s0.v[i][1] = s1.v[i][0] = s1.v[i][1] = 0;
	s0.p = s1.p = idle_p;
	s0.len = s1.len = 1025;
	s0.seed = s1.seed = 0;
	s0.b = s1.b = 0;
	s0.d = s1.d = 0;
	s0.nrows = s1.nrows = 0;
	for (;;) {
		load(t0);
		load(t1);
		__builtin_amdgcn_sched_barrier(0);
		compute(s0);
		compute(s1);
		__builtin_amdgcn_sched_barrier(0);
		if (t0.nrows == 0) break;  // (t1 is idle too: steps are loaded in order)
		load(s0);
		load(s1);
		__builtin_amdgcn_sched_barrier(0);
		compute(t0);
		compute(t1);
		__builtin_amdgcn_sched_barrier(0);
		if (s0.nrows == 0) break;
	}
	flush();
}

// ---------------------------------------------------------------------------
// Phase B: the chains, one wave per long buffer (64-thread workgroups, two
// per SIMD: more waves per SIMD slow every chain down, and the longest one
// sets the time); lane j < 8 holds acc[j].  The stripe sums
// arrive 64 blocks (4 KiB) per round by LDS-DMA (global_load_lds: no VGPR
// staging for the compiler to wait on) into a ring of four rounds, three in
// flight while the chain runs (with one in flight the chain waited on every
// round: a round's 64 scrambles take less than the DMA's latency under load).
// The chain is the only sequential part of XXH3: one scramble per 1 KiB
// block, so the batch's longest buffer sets this kernel's time.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_xsplit_b(XSplit S) {
	constexpr uint32_t NR = 4;  // rounds of 4 KiB in the LDS ring: three in flight while one is chained
	__shared__ uint64_t sd[NR * 512];
	const uint64_t nsplit = rdf64(gld64(S.sh + 0));
	const uint64_t nbig = rdf64(gld64(S.sh + 4));
	const uint32_t lane = threadIdx.x;
	const uint32_t j = lane & 7;
	const uint64_t init = j == 0 ? P32_3 : j == 1 ? P64_1 : j == 2 ? P64_2 : j == 3 ? P64_3
	                    : j == 4 ? P64_4 : j == 5 ? P32_2 : j == 6 ? P64_5 : P32_1;
	typedef __attribute__((address_space(1))) const void* gp;
	typedef __attribute__((address_space(3))) void* lp;
	auto chain = [&](uint64_t sidx) __attribute__((always_inline)) {
		const XEnt E = S.ents[sidx];
		const uint64_t len = rdf64(E.len), seed = rdf64(E.seed), idx = rdf64(E.idx);
		const uint64_t nfull = (len - 1) >> 10, nb = nfull + 1;
		const uint8_t* base = reinterpret_cast<const uint8_t*>(S.D + 8 * rdf64(E.F));
		const uint64_t last16 = 64 * nb - 16;  // the last 16 bytes of this buffer's stripe sums
		const uint64_t nround = (nb + 63) >> 6;
		const uint64_t ck = swd(16 + (int)j, seed);  // scramble key: secret + 128 + 8j
		const uint64_t gk = sat(1 + (int)j, 3, seed);  // merge key: secret + 11 + 8j
		const uint32_t cklo = (uint32_t)ck, ckhi = (uint32_t)(ck >> 32);
		// scrambleAcc (xxhash.h:3702-3718) in 32-bit halves: the high half's
		// product is off the dependent path (a ^= a >> 47 changes only the low
		// half): shift, xor3, one 32x32->64 mad and one add per block
		auto scr = [&](uint64_t a) __attribute__((always_inline)) -> uint64_t {
			const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
			const uint32_t lo2 = __builtin_amdgcn_bitop3_b32(lo, hi >> 15, cklo, 0x96);  // xor3
			const uint64_t m = (uint64_t)lo2 * (uint32_t)P32_1;
			return m + ((uint64_t)((hi ^ ckhi) * (uint32_t)P32_1) << 32);
		};
		uint64_t acc = init;
		// round c -> sd[(c % NR) * 512]: lane L's 16 bytes of quarter q land at
		// 1024 q + 16 L (the wave-uniform base + lane x 16 of the DMA)
		auto issue = [&](uint64_t c) __attribute__((always_inline)) {
			uint64_t* dst = sd + 512 * (uint32_t)(c % NR);
#pragma unroll
			for (int q = 0; q < 4; ++q) {
				const uint64_t o = 4096 * c + 1024 * q + 16 * lane;
				__builtin_amdgcn_global_load_lds((gp)(base + (o < last16 ? o : last16)), (lp)(dst + 128 * q), 16, 0, 0);
			}
		};
		// the entry's loads complete here, before any DMA is in flight (a use of
		// an ordinary load's result behind a DMA would wait for the DMA too)
		__builtin_amdgcn_s_waitcnt(0);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (uint32_t c = 0; c + 1 < NR; ++c) issue(c);
		for (uint64_t c = 0; c < nround; ++c) {
			issue(c + NR - 1);  // into round c - 1's slot (read); clamped: values past the end are never used
			__builtin_amdgcn_s_waitcnt(0x0F7C);  // vmcnt(12): round c has landed, c + 1 .. c + 3 in flight
			const uint64_t* r = sd + 512 * (uint32_t)(c % NR);
			if (lane < 8) {
				const uint64_t b0 = 64 * c;
				if (b0 + 64 <= nfull) {
#pragma unroll 16
					for (int t = 0; t < 64; ++t) acc = scr(acc + r[8 * t + j]);
				} else {
					for (uint64_t t = 0; b0 + t < nb; ++t) {
						const uint64_t x = r[8 * t + j];
						acc = b0 + t < nfull ? scr(acc + x) : acc + x;
					}
				}
			}
			// the reads of round c complete before round c + NR is issued into its slot
			__builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
		}
		__builtin_amdgcn_s_waitcnt(0);  // every DMA of this buffer landed before the next one reuses the buffers
		// mergeAccs (xxhash.h:3678-3700): lanes 2k, 2k+1 -> mulfold, summed over k
		const uint64_t a = acc ^ gk;
		const uint32_t plo = (uint32_t)__shfl_xor((int)(uint32_t)a, 1), phi = (uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), 1);
		const uint64_t bq = ((uint64_t)phi << 32) | plo;
		uint64_t m = (lane < 8 && !(j & 1)) ? (a * bq ^ __umul64hi(a, bq)) : 0;
#pragma unroll
		for (int o = 2; o < 8; o <<= 1) {
			const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)m, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(m >> 32), o);
			m += ((uint64_t)hi << 32) | lo;
		}
		uint64_t h = len * P64_1 + m;
		h ^= h >> 37;
		h *= 0x165667919E3779F9ull;
		h ^= h >> 32;
		if (lane == 0) S.out[idx] = h;
	};
	// The batch's longest chains set this kernel's time, so they start first,
	// each on a wave of its own (the planner's list of buffers of kXBig blocks
	// or more); the other buffers go to the waves without one, in entry order.
	const uint64_t W = gridDim.x, w = blockIdx.x;
	for (uint64_t q = w; q < nbig; q += W) chain(rdf64(gld64(S.big + q)));
	const bool apart = nbig < W && W - nbig >= W / 4;  // enough waves without a long chain
	const uint64_t w0 = apart ? nbig : 0, nw = apart ? W - nbig : W;
	if (w < w0) return;
	for (uint64_t e = w - w0; e < nsplit; e += nw) {
		const uint64_t len = rdf64(gld64(&S.ents[e].len));
		if (((len - 1) >> 10) + 1 < kXBig) chain(e);
	}
}

static int xsplit_a_bpc() {
	static const int bpc = [] {
		int a = 0, b = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_xsplit_a<false>, 256, 0) != hipSuccess) a = 3;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_xsplit_a<true>, 256, 0) != hipSuccess) b = 3;
		a = a < b ? a : b;
		const int c = 2 * xxh3_blocks_per_cu();  // (the workspace holds twice the row kernel's wave count of starts)
		a = a < c ? a : c;
		return a < 1 ? 1 : a;
	}();
	return bpc;
}

uint64_t xxh3_split_waves(int num_cus) { return (uint64_t)num_cus * xsplit_a_bpc() * 4; }

int launch_xxh3_split(const XSplit& S, int num_cus, bool seeds, hipStream_t stream) {
	const unsigned ga = (unsigned)((S.nwa + 3) / 4);
	if (ga == 0) return 0;
	if (seeds)
		k_xsplit_a<true><<<ga, 256, 0, stream>>>(S);
	else
		k_xsplit_a<false><<<ga, 256, 0, stream>>>(S);
	k_xsplit_b<<<(unsigned)num_cus * 8, 64, 0, stream>>>(S);  // two chains per SIMD: ~full speed each
	return 0;
}

}  // namespace fdbxxh
