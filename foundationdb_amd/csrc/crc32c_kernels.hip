// Batched CRC-32C on MI355X (gfx950).  Hand-written HIP, wave64, no MFMA.
//
// Replaces, for batches of device-resident buffers, the per-buffer loop that
// every FoundationDB caller runs over crc32c_append()
// (contrib/crc32/include/crc32/crc32c.h:36-39, contrib/crc32/crc32c.cpp:346-356).
// Results are bit-identical to that function for every (seed, bytes, length).
//
// Geometry (DESIGN.md has the derivation and the measurements behind it):
//   * A wavefront reads a buffer in BLOCKS of 4 KiB with four
//     global_load_dwordx4, each covering one contiguous KiB (fully coalesced;
//     per-lane-contiguous address patterns measured 2-3.9 TB/s and are
//     rejected).  The lanes' addresses inside each KiB are permuted so that
//     two v_permlane32_swap + two v_permlane16_swap rounds (16 VALU per
//     block) leave lane l holding the 64 CONTIGUOUS bytes [64l, 64l+64) of
//     the block in registers.
//   * Each lane runs one CRC register over its 64 bytes (4-byte slicing from
//     bank-replicated LDS tables -- every ds_read_b32 is conflict-free -- the
//     next message word folded into each step's second XOR3).
//   * Lane l then multiplies its register by x^(8*64*(63-l)) -- its distance
//     to the end of the block -- and the 64 registers are xor-reduced across
//     the wave (DPP row reduction + 4 readlanes).  Two blocks of one buffer
//     combine with x^(8*4096) (8 KiB pages).  This is append_hw's stream
//     merge (crc32c.cpp:268-269) with GPU-shaped distances.
//   * Seed: the register at the buffer's first byte is ~seed, as in
//     append_hw's pre-inversion (crc32c.cpp:197); the result is post-inverted
//     (crc32c.cpp:310).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32c_common.h"

#ifndef FDBCRC_PU
#define FDBCRC_PU 2  // pages per unit (register chains interleaved per wave)
#endif

namespace fdbcrc {

// 4 KiB pages (160 KiB LDS image, 4-byte slicing).
// U pages per unit: U independent register chains interleave (ILP U) while
// the next unit's U pages are in flight.
// WINDOW: checksum bytes [h, 4096 - t) of every page (h, t < 16): before the
// unswizzle, lane 0's first chunk (page bytes 0..15) is masked below h and
// gets the seed register at byte h (lane 32's chunk 16..31 takes the bytes
// spilling past 16), lane 63's last chunk (4080..4095) is masked from 16 - t;
// the t zero bytes are removed from the raw register when the group is stored.
template <int U, bool WINDOW, bool RAW = WINDOW>
__device__ __forceinline__ void unit_crc_b(const uint32_t* lds, int lane, uint32_t c4, uint32_t c_lane,
                                           Block (&u)[U], const uint32_t (&s)[U], uint32_t (&crc)[U],
                                           uint32_t h, uint32_t t) {
	if (WINDOW) {
#pragma unroll
		for (int j = 0; j < U; ++j) {
			const Masks mk = edge_masks(h, 16 - t, ~s[j]);
#pragma unroll
			for (int d = 0; d < 4; ++d) {
				const uint32_t m0 = lane == 0 ? mk.lm[d] : ~0u;
				const uint32_t x0 = lane == 0 ? mk.inj[d] : ((d == 0 && lane == 32) ? mk.spill : 0u);
				u[j].r[0][d] = (u[j].r[0][d] & m0) ^ x0;
				u[j].r[3][d] &= lane == 63 ? mk.tm[d] : ~0u;
			}
		}
	}
#pragma unroll
	for (int j = 0; j < U; ++j) unswizzle(u[j]);
	uint32_t x[U];
#pragma unroll
	for (int j = 0; j < U; ++j) x[j] = (!WINDOW && lane == 0) ? ~s[j] : 0u;
	// 16 word steps per chain; the next word is folded into the second XOR3
	// (x' = T3 ^ T2 ^ T1 ^ T0 ^ w': two VALU XORs per word)
#pragma unroll
	for (int j = 0; j < U; ++j) x[j] ^= u[j].r[0][0];
#pragma unroll
	for (int w = 0; w < 16; ++w)
#pragma unroll
		for (int j = 0; j < U; ++j) x[j] = word_step4_next(lds, x[j], w < 15 ? u[j].r[(w + 1) >> 2][(w + 1) & 3] : 0u, c4);
#pragma unroll
	for (int j = 0; j < U; ++j) {
		const uint32_t r = wave_xor(mul_nibbles(lds, x[j], c_lane));
		crc[j] = RAW ? r : ~r;  // raw register (WINDOW, PAIR): finished at the store
	}
}

// Strided page layout (STRIDED): lane l reads dword k of a page at byte
// 4l + 256k -- 16 global_load_dword per page, each 256 contiguous bytes -- and
// runs ONE register chain over its 16 words at a 256-byte stride:
//     r' = (r ^ w) * x^(8*256)
// four lookups per word from the stride4 tables, exactly as the contiguous
// chain's x^32 step, and no permlane swizzle.  The chain ends at 4l + 4096;
// the lane multiplies by x^(-8*4l) (lane_s) before the wave XOR.
struct BlockS {
	uint32_t w[16];
};
typedef __attribute__((address_space(1))) const uint32_t g_u32k;
__device__ __forceinline__ void load_block_s(BlockS& b, const uint8_t* page, uint32_t lane4) {
	const uint8_t* p = page + lane4;
#pragma unroll
	for (int k = 0; k < 16; ++k) b.w[k] = __builtin_nontemporal_load((g_u32k*)reinterpret_cast<uintptr_t>(p + 256 * k));
}
template <int U, bool WINDOW, bool RAW = WINDOW>
__device__ __forceinline__ void unit_crc_s(const uint32_t* lds, int lane, uint32_t c4, uint32_t c_lane,
                                           BlockS (&u)[U], const uint32_t (&s)[U], uint32_t (&crc)[U],
                                           uint32_t h, uint32_t t) {
	uint32_t x[U];
	if (WINDOW) {
		// word 0 of lane l holds bytes [4l, 4l + 4): keep those >= h and XOR in
		// ~seed at byte h (it reaches lane h/4 and, past a word boundary, the
		// next lane); word 15 holds [3840 + 4l, +4): keep those < 4096 - t
		const int d = (int)h - 4 * lane;  // ~seed's byte offset inside the word
		const uint32_t keep0 = d <= 0 ? ~0u : (d >= 4 ? 0u : ~0u << (8 * d));
		const int cut = 256 - (int)t - 4 * lane;
		const uint32_t keep15 = cut >= 4 ? ~0u : (cut <= 0 ? 0u : ~0u >> (8 * (4 - cut)));
#pragma unroll
		for (int j = 0; j < U; ++j) {
			const uint32_t sd = ~s[j];
			const uint32_t inj = (d > -4 && d < 4) ? (d >= 0 ? sd << (8 * d) : sd >> (-8 * d)) : 0u;
			x[j] = (u[j].w[0] & keep0) ^ inj;
			u[j].w[15] &= keep15;
		}
	} else {
#pragma unroll
		for (int j = 0; j < U; ++j) x[j] = (lane == 0 ? ~s[j] : 0u) ^ u[j].w[0];
	}
#pragma unroll
	for (int w = 0; w < 16; ++w)
#pragma unroll
		for (int j = 0; j < U; ++j) x[j] = word_step4_next(lds, x[j], w < 15 ? u[j].w[w + 1] : 0u, c4);
#pragma unroll
	for (int j = 0; j < U; ++j) {
		const uint32_t r = wave_xor(mul_nibbles(lds, x[j], c_lane));
		crc[j] = RAW ? r : ~r;
	}
}

// Lane-parallel multiply of a per-lane value by a constant whose nibble tables
// live in global memory (8 gathers, L2-resident).
__device__ __forceinline__ uint32_t vmul_tab(const uint32_t (*tab)[16], uint32_t v) {
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n)
		r ^= *((g_u32*)reinterpret_cast<uintptr_t>(&tab[n][(v >> (4 * n)) & 15u]));
	return r;
}

// Load balance.  The SIMD's issue arbitration favours some waves: with an
// equal static share per wave, the waves of one launch finish between 50 %
// and 100 % of the kernel time.  So each workgroup owns a contiguous range of
// GRABS (one unit pair, 2U pages, each) and its waves take them from a
// per-workgroup counter: the first two grabs of a wave are static, the next
// one is requested one grab ahead, so the atomic's return travels in the
// shadow of the data loads issued before it.  The counters (kPageCtrWords
// apart, one cache line each) belong to the launch stream and are zero
// between launches: each workgroup puts its counter back to zero once all its
// waves are done.
//
// The checksums of F = 64 / 2U consecutive grabs of a wave collect in its
// lanes (lane 2U*f + j: page j of the group's f-th grab) and leave together;
// the WINDOW / PAIR finishing multiplies run once per group.
//
// LIST: page i of the batch is page idx[i] of `base` and the batch size is
// read from *d_count (device-side compaction output, pagecheck.hip).
// PAIR: 8 KiB pages as pairs of 4 KiB blocks (block 2i+h = half h of page
// i): the seed enters the first half, and at the group store lane 2m
// combines raw(A)*x^(8*4096) ^ raw(B) with its neighbour (DPP lane swap +
// one lane-parallel table multiply).
#ifdef FDBCRC_BTIMES
// development: per-wave start / end timestamps of k_pages4k and k_bigblocks (s_memrealtime, 100 MHz)
__device__ uint64_t g_bt[16384][4];
__device__ uint64_t g_bt2[16384][4];  // prep-free start-up: after the scan's barrier, the entries' barrier, the first loads
#define FDBCRC_BT2(k) \
	{ \
		const uint64_t tk = __builtin_amdgcn_s_memrealtime(); \
		const uint32_t wk = blockIdx.x * 16 + (threadIdx.x >> 6); \
		if ((threadIdx.x & 63) == 0) __hip_atomic_store(&g_bt2[wk][k], tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
	}
#else
#define FDBCRC_BT2(k)
#endif
#ifndef FDBCRC_STRIDED
#define FDBCRC_STRIDED 0
#endif
template <int U, bool WINDOW = false, bool LIST = false, bool PAIR = false, bool STRIDED = FDBCRC_STRIDED>
__global__ __launch_bounds__(1024) void k_pages4k(const uint8_t* __restrict__ base, uint64_t stride, uint64_t count,
                                                  uint32_t seed, const uint32_t* __restrict__ seeds,
                                                  uint32_t* __restrict__ out, const DevTables* __restrict__ tabs,
                                                  uint32_t* __restrict__ ctr, uint32_t h = 0, uint32_t t = 0,
                                                  const uint32_t* __restrict__ idx = nullptr,
                                                  const uint64_t* __restrict__ d_count = nullptr) {
	if (LIST) {
		count = *d_count;
		if (count == 0) return;  // the list is empty: every wave leaves before touching the counters
	}
	if (PAIR) count *= 2;  // blocks
#ifdef FDBCRC_BTIMES
	const uint64_t pt0 = __builtin_amdgcn_s_memrealtime();
#endif
	constexpr uint32_t C = 2 * U;   // pages per grab
	constexpr uint32_t F = 64 / C;  // grabs per store group
	static_assert(64 % C == 0, "a store group fills the wave's lanes");
	__shared__ uint32_t lds[kLdsBytesB / 4];
	const LaneCtx c = make_ctx();
	const uint32_t col4 = (c.lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (c.lane >> 5) * 0x4000) | col4;
	const uint32_t wpb = blockDim.x >> 6;
	const uint32_t wi = rdfirst(threadIdx.x >> 6);
	const uint64_t ngrab = (count + C - 1) / C;
	// per-workgroup grab ranges weighted by XCD parity (xcd_range)
	uint64_t g0, g1;
	xcd_range(ngrab, blockIdx.x, gridDim.x, g0, g1);
	uint32_t* const my_ctr = ctr + kPageCtrWords * blockIdx.x;
	const uint64_t last = count - 1;
	// page index -> address, clamped into the batch: clamped duplicates are
	// computed and discarded, so every load is consumed unconditionally
	auto page = [&](uint64_t i) {
		const uint64_t j = i < count ? i : last;
		if (PAIR) return base + (j >> 1) * stride + (j & 1) * 4096;
		return base + (LIST ? (uint64_t)idx[j] : j) * stride;
	};
	typedef typename std::conditional<STRIDED, BlockS, Block>::type Blk;
	const uint32_t lane4 = 4u * (uint32_t)c.lane;
	auto load_u = [&](Blk (&u)[U], uint64_t i0) {
#pragma unroll
		for (int j = 0; j < U; ++j) {
			if constexpr (STRIDED)
				load_block_s(u[j], page(i0 + j), lane4);
			else
				load_block(u[j], page(i0 + j), c.ld_off);
		}
	};
	auto unit = [&](Blk (&u)[U], const uint32_t (&sd)[U], uint32_t (&crc)[U]) {
		if constexpr (STRIDED)
			unit_crc_s<U, WINDOW, WINDOW || PAIR>(lds, c.lane, c4, c_lane, u, sd, crc, h, t);
		else
			unit_crc_b<U, WINDOW, WINDOW || PAIR>(lds, c.lane, c4, c_lane, u, sd, crc, h, t);
	};
	auto clampg = [&](uint64_t g) { return g < g1 ? g : ngrab; };  // ngrab: nothing left
	auto request = [&]() -> uint32_t {
		uint32_t r = 0;
		if (c.lane == 0) r = atomicAdd(my_ctr, 1u);
		return r;
	};
	// lane j < C: seed of page j of grab g (an unconditional load: a branch
	// around vector memory would make the compiler wait for the loads in flight)
	auto seed_of = [&](uint64_t g) -> uint32_t {
		const uint64_t i = g * C + (uint64_t)(c.lane & (C - 1));
		const uint64_t j = i < count ? i : last;
		const uint32_t v = *(seeds ? seeds + (PAIR ? j >> 1 : j) : &tabs->slice4[0][0]);
		const uint32_t sd = seeds ? v : seed;
		return (PAIR && (c.lane & 1)) ? ~0u : sd;  // second halves carry no seed (~0 -> 0)
	};
	// Grab A is static (g0 + wi); then one request per grab, issued at the
	// grab's start and read at its middle, just before the next grab's first
	// unit is loaded (the atomic returns during the first unit's compute), so
	// a wave holds at most its grab and the next when the range runs out.
	// (Requesting a grab further ahead, as before, left the waves ~2 grabs
	// apart at the end: 1 Mi pages 672 -> 667 us, same box, 6 launches each.)
	uint64_t gA = clampg(g0 + wi), gB = ngrab;
	uint32_t sdA = seed_of(gA), sdB = 0;
	Blk u0[U], u1[U];
	load_u(u0, gA * C);  // in flight during the LDS fill
	if constexpr (STRIDED)
		fill_lds_src(lds, &tabs->stride4[0][0], &tabs->lane_s[0][0][0]);
	else
		fill_lds_b(lds, tabs);
	uint32_t mine = 0;     // lane 2U*f + j: checksum of page j of the group's f-th grab
	uint64_t myi = ~0ull;  // ... and its index in the batch (~0: none)
	uint32_t f = 0;        // grabs in the current store group
	// A store holds up every later wait on the loads issued after it until it
	// has been acknowledged (vmcnt counts stores and loads in issue order), and
	// under the read stream that takes longer than a unit's compute: the
	// groups' checksums wait in registers (raw, with 32-bit indices) and leave
	// together at the end -- or when kDefer groups are held (1 Mi pages: ~4
	// groups per wave).  Measured: the page kernel without its stores ran 2.5 %
	// faster; the WINDOW / PAIR finishing multiplies (L2 gathers) would wait
	// for every load in flight as well.
	constexpr uint32_t kDefer = 8;
	const bool defer = count < 0xFFFFFFFFull;  // (indices fit 32 bits; else each group leaves at once)
	uint32_t dm[kDefer], di[kDefer];
	uint32_t nd = 0;  // groups held
	auto finish = [&](uint32_t m, uint64_t i) {
		if (WINDOW) m = ~(t ? vmul_tab(tabs->inv_z[t], m) : m);
		if (PAIR) {
			const uint32_t other = __builtin_amdgcn_update_dpp(0u, m, 0xB1, 0xF, 0xF, false);  // lane ^ 1
			m = ~(vmul_tab(tabs->block, m) ^ other);
			if (i < count && !(c.lane & 1)) out[i >> 1] = m;
		} else if (i < count) {
			out[i] = m;
		}
	};
	auto flush_held = [&]() {
#pragma unroll
		for (uint32_t q = 0; q < kDefer; ++q)
			if (q < nd) finish(dm[q], di[q] == ~0u ? ~0ull : (uint64_t)di[q]);
		nd = 0;
	};
	auto store = [&]() {
		if (defer) {
#pragma unroll
			for (uint32_t q = 0; q < kDefer; ++q)
				if (q == nd) {
					dm[q] = mine;
					di[q] = myi < count ? (uint32_t)myi : ~0u;
				}
			if (++nd == kDefer) flush_held();
		} else {
			finish(mine, myi);
		}
		myi = ~0ull;
	};
	while (gA < ngrab) {
		const uint64_t first = gA * C;
		const uint32_t l0 = f * C;
		uint32_t sd[U], crc[U];
		const uint32_t req = request();
		load_u(u1, first + U);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int j = 0; j < U; ++j) sd[j] = rdlane(sdA, j);
		unit(u0, sd, crc);
#pragma unroll
		for (int j = 0; j < U; ++j) mine = (uint32_t)c.lane == l0 + j ? crc[j] : mine;
		__builtin_amdgcn_sched_barrier(0);
		gB = clampg(g0 + wpb + rdlane(req, 0));
		sdB = seed_of(gB);
		load_u(u0, gB * C);  // the next grab's first unit
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int j = 0; j < U; ++j) sd[j] = rdlane(sdA, U + j);
		unit(u1, sd, crc);
#pragma unroll
		for (int j = 0; j < U; ++j) mine = (uint32_t)c.lane == l0 + U + j ? crc[j] : mine;
		__builtin_amdgcn_sched_barrier(0);
		const uint32_t k = (uint32_t)c.lane - l0;
		myi = k < C ? first + k : myi;
		gA = gB;
		sdA = sdB;
		if (++f == F) {
			store();
			f = 0;
		}
	}
	if (f) store();
	flush_held();
#ifdef FDBCRC_BTIMES
	if (c.lane == 0) {
		const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
		if (w < 16384) {
			g_bt[w][0] = pt0;
			g_bt[w][1] = __builtin_amdgcn_s_memrealtime();
			g_bt[w][2] = 0;
			g_bt[w][3] = 0;
		}
	}
#endif
	// every request of every wave has returned: the counter goes back to zero
	// for the next launch on this stream
	__builtin_amdgcn_s_waitcnt(0);
	__syncthreads();
	if (threadIdx.x == 0) *my_ctr = 0;
}

// ---------------------------------------------------------------------------
// Big-buffer block route (buffers the varlen prep routed here, crc32c_varlen.hip)
// ---------------------------------------------------------------------------
// A routed buffer [P0, P1) is cut into nb 4 KiB BLOCKS aligned to its
// 16-byte-rounded end E: block k (counted from the end) is
// [E - 4096(k+1), E - 4096k).  The blocks of all routed buffers, in buffer
// order, stream exactly like 4 KiB pages (k_pages4k: same loads, swizzle,
// register chains, lane fold, dynamic per-workgroup grabs).  Edges, in the
// load layout before the swizzle (uniform branches, first/last block only):
//   * the first block's chunks before A = P0 & ~15 are not loaded (their
//     addresses clamp to A) and hold zeros -- leading zeros are free;
//   * in the lead chunk the bytes below P0 are zeroed and ~seed is XORed in
//     at P0 (append_hw's pre-inversion, crc32c.cpp:197); what spills past the
//     chunk goes into the next chunk, or into the register at the block end;
//   * in the last chunk the t = E - P1 bytes after the buffer are zeroed.
// Every block's raw register R is weighted to the buffer's end and XORed
// into out[] (prep stored ~0 there: the final inversion):
//     out ^= R * x^(8*4096*k) * x^(-8t)          (k < 2^28: spans under 1 TiB)
//
// Block -> buffer: each wave keeps a WINDOW of 64 consecutive route entries
// in its lanes; the owner of block b is the last entry whose first block is
// <= b (one ballot).  The window only moves forward (a wave's grabs
// increase) and is refilled when a grab passes its end.  The registers of a
// store group's 64 blocks (increasing block order, so a buffer's blocks sit
// in adjacent lanes) are weighted lane-parallel (global nibble tables),
// XOR-reduced per buffer (segmented scan) and leave with one atomicXor per
// buffer part.
//
// Lane and register of the 16-byte chunk at block offset o in the load
// layout (make_ctx, load_block): lane 32h + 16q + r, register ka | kb << 1.
__device__ __forceinline__ void chunk_slot(uint32_t o, uint32_t& ln, uint32_t& ri) {
	ln = 32 * ((o >> 4) & 1) + 16 * ((o >> 5) & 1) + ((o >> 6) & 15);
	ri = ((o >> 11) & 1) | (((o >> 10) & 1) << 1);
}
// ---- prep-free form: each workgroup plans its own blocks ------------------
// The kernel's arguments re-read at their use from the kernarg segment (an
// opaque pointer: the compiler cannot keep the values in SGPRs across the
// stream loop, where they spilled)
typedef __attribute__((address_space(4))) const BigParams KBig;
__device__ __forceinline__ KBig* big_kargs() {
#if defined(__HIP_DEVICE_COMPILE__)
	KBig* kp = (KBig*)__builtin_amdgcn_kernarg_segment_ptr();
	asm volatile("" : "+s"(kp));
	return kp;
#else
	return nullptr;
#endif
}
// Route geometry of one buffer on the block route alone: every buffer of 16
// bytes or more, in 4 KiB blocks aligned to its 16-byte-rounded end (a span
// of 1 TiB or more refuses the batch); shorter ones are finished byte by byte.
struct NPGeo {
	uint32_t nb;  // blocks (0: shorter than 16 bytes)
	bool refuse;
};
__device__ __forceinline__ NPGeo np_geo(uint64_t P0, uint64_t len) {
	NPGeo g;
	const uint64_t E = (P0 + len + 15) & ~uint64_t(15), A = P0 & ~uint64_t(15);
	const uint64_t span = E - A;
	g.refuse = len >= 16 && span >= kBigMax;
	g.nb = len >= 16 && !g.refuse ? (uint32_t)((span + 4095) >> 12) : 0u;
	return g;
}
__device__ __forceinline__ BigEnt np_entry(uint64_t P0, uint64_t len, uint32_t nb, uint32_t s, uint32_t idx,
                                           uint32_t seed) {
	const uint64_t E = (P0 + len + 15) & ~uint64_t(15), A = P0 & ~uint64_t(15);
	const uint32_t lo = (uint32_t)(4096ull * nb - (E - A));
	BigEnt e;
	e.E = E;
	e.s = s;
	e.idx = idx;
	e.lot = (lo >> 4) | ((uint32_t)(P0 & 15) << 8) | ((uint32_t)(E - (P0 + len)) << 12);
	e.sd = ~seed;
	return e;
}
struct NPStart {
	uint32_t count, nbig;  // blocks, entries
	uint32_t qa, qlim;     // this workgroup's first entry, and its sentinel (the entry after its last)
	uint32_t smallm;       // this thread's buffers (bit j: buffer t*m + j) shorter than 16 bytes
	uint32_t m;            // buffers per thread
	bool refused;
};
// LDS words used before the table fill (fill_commit_1024 writes wave w's
// share of round r, words [4096 r + 256 w, + 256), only after its own reads):
// round 0, wave w's first words: the hand-over (first entry, sentinel); wave
// 0's words 16..47: workgroup 0's statistics; round 1: the scan's wave sums;
// rounds 2-3: the batch's block counts.
// A workgroup barrier for LDS only: the waves' LDS writes done, global memory
// operations left in flight (__syncthreads' fence waits for them too); the
// memory clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
constexpr uint32_t kNPRing = 0;         // [128][6] route entries by q mod 128 (the waves' first windows)
constexpr uint32_t kNPScratch = 1024;   // the scan's wave sums
constexpr uint32_t kNPStats = 1088;     // u64 [4 waves][4]: workgroup 0's route statistics
constexpr uint32_t kNPHand = 1200;      // first entry, sentinel
constexpr uint32_t kNPBlocks = 2048;    // [kNPMax] blocks per buffer
constexpr uint32_t kNPGeo = kNPBlocks + kNPMax;  // [kNPMax][4] E (2 words), lo | k0 | t, ~seed: one 16-byte read
static_assert(kNPGeo + 4 * kNPMax <= kLdsBytesB / 4, "prep-free start-up: its LDS scratch fits the table image");
// Every workgroup sums the whole batch's block counts (thread t: buffers
// [8t, 8t + 8), their metadata loaded at once), writes the route entries of
// the buffers its own grab range [g0, g1) covers -- plus a sentinel entry
// holding the first block after them -- into its part of P.priv, and hands
// its first entry to its waves.  All of this runs before the table fill is
// written to LDS (the table loads are in flight meanwhile).
template <uint32_t C>
__device__ NPStart np_start(const BigParams& P, uint32_t* lds, uint32_t ngrid) {
	typedef __attribute__((address_space(1))) const uint64_t g_u64;
	auto gl64 = [](const uint64_t* p) -> uint64_t { return *((g_u64*)reinterpret_cast<uintptr_t>(p)); };
	NPStart R;
	const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
	const uint64_t n = P.nbuf;  // (<= kNPMax = 6144: at most six buffers per thread)
	const uint32_t m = (uint32_t)((n + 1023) >> 10);
	const uint64_t i0 = (uint64_t)t * m;
	uint32_t* const nbl = lds + kNPBlocks;                                // [n] blocks per buffer
	uint64_t* const sB = reinterpret_cast<uint64_t*>(lds + kNPScratch);  // [16] wave block sums
	uint32_t* const sN = lds + kNPScratch + 32;                           // [16] wave entry sums
	uint32_t* const sR = lds + kNPScratch + 48;                           // [16] wave refusals
	uint64_t B = 0;
	uint32_t N = 0, smallm = 0;
	bool refuse = false;
	for (uint32_t j0 = 0; j0 < m; j0 += 8) {
		uint64_t o[8], l[8];
		uint32_t sd[8];
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u) {
			const uint64_t ic = j0 + u < m && i0 + j0 + u < n ? i0 + j0 + u : 0;
			o[u] = gl64(P.offsets + ic);
			l[u] = gl64(P.lengths + ic);
			// (per-buffer seeds loaded here, with the metadata: a load in the
			// entry loop below made its join wait for the entries' stores)
			sd[u] = P.seeds ? P.seeds[ic] : P.seed;
		}
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u) {
			if (j0 + u < m && i0 + j0 + u < n) {
				const uint64_t P0 = reinterpret_cast<uint64_t>(P.base) + o[u];
				const NPGeo g = np_geo(P0, l[u]);
				nbl[i0 + j0 + u] = g.nb;
				const BigEnt e = np_entry(P0, l[u], g.nb, 0u, 0u, sd[u]);
				*reinterpret_cast<u32x4*>(lds + kNPGeo + 4 * (uint32_t)(i0 + j0 + u)) =
				    u32x4{(uint32_t)e.E, (uint32_t)(e.E >> 32), e.lot, e.sd};
				B += g.nb;
				N += g.nb ? 1u : 0u;
				refuse |= g.refuse;
				smallm |= (g.nb == 0 && !g.refuse ? 1u : 0u) << (j0 + u);
			}
		}
	}
	FDBCRC_BT2(0)
	uint64_t Bi = B;
	uint32_t Ni = N;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint64_t vb = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(Bi >> 32), d) << 32) |
		                    (uint32_t)__shfl_up((int)(uint32_t)Bi, d);
		const uint32_t vn = (uint32_t)__shfl_up((int)Ni, d);
		if (lane >= (uint32_t)d) {
			Bi += vb;
			Ni += vn;
		}
	}
	const bool wref = __ballot(refuse) != 0;
	if (lane == 63) {
		sB[wv] = Bi;
		sN[wv] = Ni;
		sR[wv] = wref ? 1u : 0u;
	}
	__syncthreads();
	FDBCRC_BT2(1)
	// the 16 wave sums, lane-parallel: lanes 0..15 of every wave read them
	// once and scan them (serial reads took 0.8 us)
	constexpr uint32_t nw = 16;  // (1024-thread workgroups: blockDim read from memory costs a round trip here)
	const uint32_t kl = lane & 15;
	uint64_t sb16 = sB[kl];
	uint32_t sn16 = sN[kl];
	const bool ref = __ballot(sR[kl] != 0) != 0;
#pragma unroll
	for (int d = 1; d < 16; d <<= 1) {
		const uint64_t vb = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(sb16 >> 32), d, 16) << 32) |
		                    (uint32_t)__shfl_up((int)(uint32_t)sb16, d, 16);
		const uint32_t vn = (uint32_t)__shfl_up((int)sn16, d, 16);
		if (kl >= (uint32_t)d) {
			sb16 += vb;
			sn16 += vn;
		}
	}
	const uint64_t Btot = rdlane64(sb16, 15);
	const uint32_t Ntot = rdlane(sn16, 15);
	const uint64_t Bex = Bi - B + (wv ? rdlane64(sb16, (int)wv - 1) : 0);
	const uint32_t Nex = Ni - N + (wv ? rdlane(sn16, (int)wv - 1) : 0u);
	// 32-bit block and entry numbers, as the planner's
	R.refused = ref || Btot >= 0xFFFFFFFFull;
	R.count = R.refused ? 0u : (uint32_t)Btot;
	R.nbig = Ntot;
	R.smallm = smallm;
	R.m = m;
	R.qa = R.qlim = 0;
	const uint32_t ngrab = (uint32_t)(((uint64_t)R.count + C - 1) / C);
	const uint32_t per = (ngrab + ngrid - 1) / ngrid;
	const uint32_t g0 = blockIdx.x * per, g1 = g0 + per < ngrab ? g0 + per : ngrab;
	const uint64_t blo = (uint64_t)g0 * C;
	const uint64_t bhi = g1 * (uint64_t)C < R.count ? g1 * (uint64_t)C : R.count;  // this workgroup's blocks [blo, bhi)
	BigEnt* const priv = P.priv + 2 * blockIdx.x;
	// an entry: to the ring (the first windows) and to this workgroup's part of
	// P.priv (window moves, when its range holds more entries than a window)
	auto put = [&](uint32_t q, const BigEnt& e) {
		priv[q] = e;
		uint32_t* const r = lds + kNPRing + 6 * (q & 127u);
		r[0] = (uint32_t)e.E;
		r[1] = (uint32_t)(e.E >> 32);
		r[2] = e.s;
		r[3] = e.idx;
		r[4] = e.lot;
		r[5] = e.sd;
	};
	if (!R.refused && g0 < g1 && Bex < bhi && Bex + B > blo) {
		uint64_t sb = Bex;
		uint32_t q = Nex;
		for (uint32_t j = 0; j < m; ++j) {
			const uint64_t i = i0 + j;
			if (i >= n || sb >= bhi) break;
			const uint32_t nb = nbl[i];
			if (!nb) continue;
			if (sb + nb > blo) {
				const u32x4 gq = *reinterpret_cast<const u32x4*>(lds + kNPGeo + 4 * (uint32_t)i);
				BigEnt e;
				e.E = ((uint64_t)gq[1] << 32) | gq[0];
				e.s = (uint32_t)sb;
				e.idx = (uint32_t)i;
				e.lot = gq[2];
				e.sd = gq[3];
				put(q, e);
				if (sb <= blo) lds[kNPHand] = q;  // holds the workgroup's first block
				if (bhi <= sb + nb) {  // holds its last block: the sentinel follows
					BigEnt z;
					z.E = 0;
					z.s = (uint32_t)(sb + nb);
					z.idx = ~0u;
					z.lot = 0;
					z.sd = 0;
					put(q + 1, z);
					lds[kNPHand + 1] = q + 1;
				}
			}
			sb += nb;
			++q;
		}
	}
	// workgroup 0: the route statistics of the first 256 buffers (v7_route_stats'
	// classes and packing), one buffer per thread, into wave 0's own fill words
	if (blockIdx.x == 0 && P.hstat && t < 256) {
		const uint64_t i = t;
		const bool ok = i < n;
		const uint64_t off = ok ? P.offsets[i] : 0, len = ok ? P.lengths[i] : 0;
		const bool nx = i + 1 < n;
		const uint64_t on = nx ? P.offsets[i + 1] : 0;
		const uint64_t P0 = reinterpret_cast<uint64_t>(P.base) + off;
		const uint64_t span = ok && len >= 16 ? ((P0 + len + 15) & ~uint64_t(15)) - (P0 & ~uint64_t(15)) : 0;
		const uint64_t e = off + len, gap = on - e;
		uint64_t c[4] = {span > 128 && span < 4096 ? len : 0, span >= 4096 && span < 16384 ? len : 0,
		                 span >= 16384 ? len : 0,
		                 (ok && nx && !(on >= e && gap < 4096 && gap <= (len > 256 ? len : 256))) ? 1u : 0u};
#pragma unroll
		for (int k = 0; k < 4; ++k)
			for (int o = 32; o > 0; o >>= 1)
				c[k] += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(c[k] >> 32), o) << 32) |
				        (uint32_t)__shfl_xor((int)(uint32_t)c[k], o);
		uint64_t* const s64 = reinterpret_cast<uint64_t*>(lds + kNPStats);
		if (lane == 0)
#pragma unroll
			for (int k = 0; k < 4; ++k) s64[4 * wv + k] = c[k];
	}
	// LDS only: the entries' global stores stay in flight (waited for below
	// only when this workgroup's windows will move and read them back)
	lds_barrier();
	FDBCRC_BT2(2)
	R.qa = rdfirst(lds[kNPHand]);
	R.qlim = rdfirst(lds[kNPHand + 1]);
	if (R.qlim - R.qa >= 64 && !R.refused && g0 < g1) {  // (uniform)
		__builtin_amdgcn_s_waitcnt(0);
		__syncthreads();
	}
	// parked in device memory beside the accumulators: the host-mapped words
	// are written at the kernel's end, off the start-up's path
	if (blockIdx.x == 0 && t == 0 && P.hstat) {
		const uint64_t* const s64 = reinterpret_cast<const uint64_t*>(lds + kNPStats);
		uint64_t* const park = reinterpret_cast<uint64_t*>(P.acc + 2 * kNPMax);
		for (int k = 0; k < 4; ++k) park[k] = s64[k] + s64[4 + k] + s64[8 + k] + s64[12 + k];
	}
	return R;
}

template <int U, bool NP>
__global__ __launch_bounds__(1024) void k_bigblocks(BigParams P) {
#ifdef FDBCRC_BTIMES
	const uint64_t bt0 = __builtin_amdgcn_s_memrealtime();
#endif
	typedef __attribute__((address_space(1))) const uint64_t g_u64;
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	auto gl32 = [](const uint32_t* p) -> uint32_t { return *((g_u32*)reinterpret_cast<uintptr_t>(p)); };
	auto gl64 = [](const uint64_t* p) -> uint64_t { return *((g_u64*)reinterpret_cast<uintptr_t>(p)); };
	// the LDS table loads go out first: they return while the header, the
	// entry search and the window load (dependent round trips) proceed
	// the grid size is a hidden kernel argument: read now, with the others (a
	// scalar load where it is first used put a round trip into the planning)
	const uint32_t ngrid = gridDim.x;
	asm volatile("" ::"s"(ngrid));
	FillRegs fill;
	fill_issue_1024(fill, P.tabs);
	constexpr uint32_t C = 2 * U;   // blocks per grab
	constexpr uint32_t F = 64 / C;  // grabs per store group
	__shared__ uint32_t lds[kLdsBytesB / 4];
	// (32-bit block, entry and grab numbers: the planner refuses batches of
	// 2^32 - 1 or more blocks)
	NPStart S;
	uint32_t count, nbig;
	if (NP) {
		S = np_start<C>(P, lds, ngrid);
		if (S.refused) {
			if (blockIdx.x == 0 && threadIdx.x == 0 && P.err) *P.err = 1u;
			return;
		}
		count = S.count;
		nbig = S.nbig;
	} else {
		count = (uint32_t)rdfirst64(gl64(P.hdr + 2));  // blocks
		if (count == 0) return;
		nbig = (uint32_t)rdfirst64(gl64(P.hdr + 3));   // entries
	}
	const DevTables* __restrict__ T = P.tabs;
	const LaneCtx c = make_ctx();
	const uint32_t lane = (uint32_t)c.lane;
	const uint32_t col4 = (lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (lane >> 5) * 0x4000) | col4;
	constexpr uint32_t wpb = 16;  // waves per workgroup (launched with 1024 threads)
	const uint32_t wi = rdfirst(threadIdx.x >> 6);
	const uint32_t ngrab = (uint32_t)(((uint64_t)count + C - 1) / C);
	const uint32_t per = (ngrab + ngrid - 1) / ngrid;
	const uint32_t g0 = blockIdx.x * per;
	const uint32_t g1 = g0 + per < ngrab ? g0 + per : ngrab;
	uint32_t* const my_ctr = P.ctr + kPageCtrWords * blockIdx.x;
	const uint32_t last = (uint32_t)(count - 1);

	// ---- window of route entries [wj, wj + 64) ----------------------------
	uint32_t wj = 0;
	uint32_t ws = 0, wI = 0, wL = 0, wS = 0, wend = 0;  // first block (~0: none), output index, lo | k0 | t, ~seed
	uint64_t wE = 0;                                   // 16-byte-rounded end
	// (prep-free: this workgroup's own entries, read past the L1 -- a line
	// cached there by an earlier launch would be stale)
	auto ent = [&](uint32_t q) -> BigEnt {
		const uint64_t* w = reinterpret_cast<const uint64_t*>(NP ? big_kargs()->priv + 2 * blockIdx.x + q : P.ent + q);
		uint64_t w0, w1, w2;
		if (NP) {
			w0 = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			w1 = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			w2 = __hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		} else {
			w0 = gl64(w);
			w1 = gl64(w + 1);
			w2 = gl64(w + 2);
		}
		BigEnt e;
		e.E = w0;
		e.s = (uint32_t)w1;
		e.idx = (uint32_t)(w1 >> 32);
		e.lot = (uint32_t)w2;
		e.sd = (uint32_t)(w2 >> 32);
		return e;
	};
	auto ent_s = [&](uint32_t q) -> uint32_t {
		if (NP)
			return __hip_atomic_load(&big_kargs()->priv[2 * blockIdx.x + q].s, __ATOMIC_RELAXED,
			                         __HIP_MEMORY_SCOPE_AGENT);
		return gl32(&P.ent[q].s);
	};
	// prep-free: entries past this workgroup's sentinel are never read
	const uint32_t qtop = NP ? S.qlim : nbig - 1;
	auto load_window = [&](uint32_t j0) {
		const uint32_t q = j0 + lane;
		const uint32_t qc = q <= qtop ? q : qtop;  // clamped: every load is unconditional
		const BigEnt e = ent(qc);
		const uint32_t s = e.s;
		wE = e.E;
		wI = e.idx;
		wL = e.lot;
		wS = e.sd;
		if (NP) {  // entries qa .. qlim (the sentinel's first block closes the last one)
			const uint32_t qe = (uint64_t)j0 + 64 <= qtop ? j0 + 64 : qtop;
			const uint32_t se = ent_s(qe);
			ws = q <= qtop ? s : ~0u;
			wend = (uint64_t)j0 + 64 <= qtop ? rdfirst(se) : count;
		} else {
			const uint32_t qe = (uint64_t)j0 + 64 < nbig ? j0 + 64 : nbig - 1;
			const uint32_t se = ent_s(qe);
			ws = q < nbig ? s : (q == nbig ? count : ~0u);
			wend = (uint64_t)j0 + 64 < nbig ? rdfirst(se) : count;
		}
		wj = j0;
	};
	// the entry holding block b: the last q with es[q] <= b (64-ary narrowing)
	// (256-ary narrowing: four samples per lane per round trip -- two rounds
	// up to 16 Ki entries, three up to 4 Mi)
	auto find = [&](uint32_t b) -> uint32_t {
		uint32_t q0 = 0, n = nbig;  // es[q0] <= b
		for (;;) {
			if (n <= 64) {
				const uint32_t v = ent_s(q0 + (lane < n ? lane : 0));
				const bool le = lane < n && v <= b;
				return q0 + (uint32_t)__builtin_popcountll(__ballot(le)) - 1;
			}
			const uint32_t stp = (n + 255) >> 8;
			uint32_t v[4];
#pragma unroll
			for (uint32_t u = 0; u < 4; ++u) {
				const uint64_t k = (4 * (uint64_t)lane + u) * stp;
				v[u] = ent_s(q0 + (uint32_t)(k < n ? k : 0));
			}
			uint32_t cnt = 0;
#pragma unroll
			for (uint32_t u = 0; u < 4; ++u) {
				const uint64_t k = (4 * (uint64_t)lane + u) * stp;
				cnt += (uint32_t)__builtin_popcountll(__ballot(k < n && v[u] <= b));
			}
			if (stp == 1) return q0 + cnt - 1;
			q0 += (cnt - 1) * stp;
			n = n - (cnt - 1) * stp < stp ? n - (cnt - 1) * stp : stp;
		}
	};

	// ---- per-grab metadata, one block per lane -----------------------------
	// Lane j < C holds block j of the grab: its address, its index from the
	// buffer's end | t << 28, its first-block lead (lo/16 | k0 << 8), ~seed and
	// output index.  (Held as wave-uniform values -- 24 SGPRs per grab, two
	// grabs live -- they spilled 113 SGPRs.)  A block's fields are read with
	// v_readlane where it is loaded and checksummed.
	struct Meta {
		uint32_t alo, ahi, kt, ek, sd, idx, nbt;  // (nbt: the buffer's blocks, prep-free form)
	};
	auto rd = [](uint32_t v, uint32_t j) { return rdlane(v, (int)j); };
	// lane j (< C): block b0 + j (past the batch's last block: a duplicate
	// of it, result discarded); its entry e = the last window entry whose
	// first block is <= b, one ballot per block
	auto pick = [&](Meta& M, uint32_t b0) {
		const uint32_t j = lane & (C - 1);
		int e = 0;
#pragma unroll
		for (uint32_t t = 0; t < C; ++t) {
			const uint32_t bt = b0 + t <= last ? b0 + t : last;
			const int et = (int)__builtin_popcountll(__ballot(ws <= bt)) - 1;
			e = j == t ? et : e;
		}
		const uint32_t b = b0 + j <= last ? b0 + j : last;
		const int src = e << 2;
		const uint32_t se = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)ws);
		const uint32_t sn1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4, (int)ws);
		const uint32_t sn = e < 63 ? sn1 : wend;
		const uint32_t lot = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wL);
		const uint32_t eEl = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)wE);
		const uint32_t eEh = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(wE >> 32));
		const uint32_t sdv = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wS);
		const uint32_t ixv = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wI);
		const uint32_t m = b - se;           // block index from the buffer's start
		const uint32_t k = sn - se - 1 - m;  // ... from its end
		const uint64_t a = (((uint64_t)eEh << 32) | eEl) - 4096ull * (k + 1);
		M.alo = (uint32_t)a;
		M.ahi = (uint32_t)(a >> 32);
		M.kt = k | ((lot >> 12) << 28);
		M.ek = m == 0 ? lot & 0xFFFu : 0u;
		M.sd = m == 0 ? sdv : 0u;
		M.idx = b0 + j <= last ? ixv : ~0u;
		M.nbt = sn - se;
	};
	auto meta_of = [&](uint32_t g, Meta& M) {
		const uint64_t bf = (uint64_t)g * C;
		if (bf >= count) {  // nothing left: duplicates of the window's first entry's last block, discarded
			const uint64_t a0 = rdlane64(wE, 0) - 4096;
			// a buffer of one block starts lo bytes into it: its loads clamp there
			const uint32_t lo16 = rdlane(ws, 1) - rdlane(ws, 0) == 1 ? rdlane(wL, 0) & 0xFFu : 0u;
			M.alo = (uint32_t)a0;
			M.ahi = (uint32_t)(a0 >> 32);
			M.kt = 0;
			M.ek = lo16;
			M.sd = 0;
			M.idx = ~0u;
			M.nbt = 0;
			return;
		}
		const uint32_t b0 = (uint32_t)bf;
		const uint32_t bl = bf + C - 1 < count ? b0 + C - 1 : last;
		// The window moves (rarely): its loads are waited for on that path
		// only.  With one path the compiler's wait before the lookups below
		// assumed the window had just been loaded and drained every block load
		// in flight, once per grab.
		if (bl >= wend) {
			do {
				const uint32_t adv = b0 < wend ? (uint32_t)__builtin_popcountll(__ballot(ws <= b0)) - 1u : 64u;
				load_window(wj + adv);
			} while (bl >= wend);
			pick(M, b0);
		} else {
			pick(M, b0);
		}
	};
	auto load_u = [&](Block (&u)[U], const Meta& M, uint32_t j0) {
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) {
			const uint8_t* blk = reinterpret_cast<const uint8_t*>(((uint64_t)rd(M.ahi, j0 + j) << 32) | rd(M.alo, j0 + j));
			const uint32_t lo = (rd(M.ek, j0 + j) & 0xFFu) << 4;
			// load k = 2kb + ka reads block bytes ld_off + 2048ka + 1024kb
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				uint32_t off = c.ld_off + 2048u * (k & 1) + 1024u * (k >> 1);
				off = off > lo ? off : lo;
				u[j].r[k] = ld16(blk + off);
			}
		}
	};
	auto crc_u = [&](Block (&u)[U], const Meta& M, uint32_t j0, uint32_t (&crc)[U]) {
		uint32_t spill[U];
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) {
			const uint32_t kt = rd(M.kt, j0 + j), ek = rd(M.ek, j0 + j), sd = rd(M.sd, j0 + j);
			spill[j] = 0;
			if (ek | sd) {  // first block
				const uint32_t lo = (ek & 0xFFu) << 4, k0 = ek >> 8;
#pragma unroll
				for (int k = 0; k < 4; ++k) {  // chunks before the lead chunk
					const bool z = c.ld_off + 2048u * (k & 1) + 1024u * (k >> 1) < lo;
#pragma unroll
					for (int d = 0; d < 4; ++d) u[j].r[k][d] = z ? 0u : u[j].r[k][d];
				}
				const Masks mk = edge_masks(k0, 16u, sd);
				uint32_t ln, ri;
				chunk_slot(lo, ln, ri);
				const bool lead_lane = lane == ln;
#pragma unroll
				for (uint32_t k = 0; k < 4; ++k) {
					const bool on = lead_lane && k == ri;
#pragma unroll
					for (int d = 0; d < 4; ++d) u[j].r[k][d] = on ? ((u[j].r[k][d] & mk.lm[d]) ^ mk.inj[d]) : u[j].r[k][d];
				}
				// ~seed past the lead chunk: into the next chunk, or the register at the block end
				const bool in_blk = lo + 16 < 4096;
				chunk_slot((lo + 16) & 4095u, ln, ri);
				const bool sp_lane = in_blk && lane == ln;
#pragma unroll
				for (uint32_t k = 0; k < 4; ++k) u[j].r[k][0] ^= (sp_lane && k == ri) ? mk.spill : 0u;
				spill[j] = in_blk ? 0u : mk.spill;
			}
			const uint32_t t = kt >> 28;
			if ((kt & 0xFFFFFFFu) == 0 && t) {  // last block: the bytes after the buffer (lane 63, register 3)
				const Masks mt = edge_masks(0u, 16u - t, 0u);
#pragma unroll
				for (int d = 0; d < 4; ++d) u[j].r[3][d] &= lane == 63 ? mt.tm[d] : ~0u;
			}
		}
		uint32_t sd[U];
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) sd[j] = ~0u;  // no register at the block start: ~sd = 0
		unit_crc_b<U, false, true>(lds, c.lane, c4, c_lane, u, sd, crc, 0, 0);
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) crc[j] ^= spill[j];
	};

	uint32_t mine = 0, mkt = 0, midx = ~0u, mnbt = 0;  // lane f*C + j: block j of the group's f-th grab
	auto store = [&]() {
		const uint32_t k = mkt & 0xFFFFFFFu, t = mkt >> 28;
		uint32_t w = vmul_tab(T->bpow[0][k & 255u], mine);
		if (__ballot(k >= (1u << 8))) w = vmul_tab(T->bpow[1][(k >> 8) & 255u], w);
		if (__ballot(k >= (1u << 16))) w = vmul_tab(T->bpow[2][(k >> 16) & 255u], w);
		if (__ballot(k >= (1u << 24))) w = vmul_tab(T->bpow[3][k >> 24], w);
		w = vmul_tab(T->inv_z[t], w);
		// segmented inclusive XOR over runs of equal output index (and, prep-free,
		// the run's block count)
		uint32_t nrun = 1;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t y = (uint32_t)__shfl_up((int)w, d);
			const uint32_t yi = (uint32_t)__shfl_up((int)midx, d);
			const uint32_t yn = NP ? (uint32_t)__shfl_up((int)nrun, d) : 0u;
			if ((int)lane >= d && yi == midx) {
				w ^= y;
				nrun += yn;
			}
		}
		const uint32_t ni = (uint32_t)__shfl_down((int)midx, 1);
		if (midx != ~0u && (lane == 63 || ni != midx)) {
			if (!NP) {
				atomicXor(P.out + midx, w);
			} else {
				// The part's XOR, performed (its return awaited) before its block
				// count is added: the part whose count completes the buffer reads
				// every part's XOR back, writes ~acc to out[] and leaves both words
				// zero for the next launch.  (No out[] initialisation ahead of the
				// stream: that took a kernel of its own.)
				uint32_t* const acc = big_kargs()->acc + midx;
				uint32_t* const cnt = acc + kNPMax;
				const uint32_t old = atomicXor(acc, w);
				asm volatile("" ::"v"(old));
				const uint32_t done = atomicAdd(cnt, nrun) + nrun;
				if (done == mnbt) {
					const uint32_t v = atomicExch(acc, 0u);
					atomicExch(cnt, 0u);
					big_kargs()->out[midx] = ~v;
				}

			}
		}
		midx = ~0u;
	};

	auto clampg = [&](uint32_t g) { return g < g1 ? g : ngrab; };  // ngrab: nothing left
	auto request = [&]() -> uint32_t {
		uint32_t r = 0;
		if (lane == 0) r = atomicAdd(my_ctr, 1u);
		return r;
	};
	// grab A static (g0 + wi), then one request per grab, issued at its start
	// and read at its middle (k_pages4k)
	uint32_t gA = clampg(g0 + wi);
	// prep-free: a workgroup without grabs (or a batch without blocks) streams
	// nothing -- its window would hold no entry of its own
	const bool run = !NP || (count > 0 && g0 < g1);
	if (!NP) {
		// One entry search per workgroup (wave 0; every wave searching put 16x the
		// scattered entry loads at the kernel's start), handed to each wave in an
		// LDS word of its OWN table-fill share: wave w reads it before its
		// fill_commit overwrites it, so no wave's fill races another's read.  (The
		// barrier's fence waits for the table loads in flight: they return during
		// the search anyway.)
		if (wi == 0) {
			const uint32_t q = find(g0 * C < count ? (uint32_t)(g0 * C) : last);
			if (lane < wpb) lds[kS4Off / 4 + 256 * lane] = q;  // (thread 64w's first fill word)
		}
		__syncthreads();
		load_window(rdfirst(lds[kS4Off / 4 + 256 * wi]));
	} else if (run) {
		if (S.qlim - S.qa < 64) {
			// the whole range fits one window: from the LDS ring, and it never
			// moves (no round trip)
			const uint32_t q = S.qa + lane, qc = q <= S.qlim ? q : S.qlim;
			const uint32_t* const r = lds + kNPRing + 6 * (qc & 127u);
			wE = ((uint64_t)r[1] << 32) | r[0];
			ws = q <= S.qlim ? r[2] : ~0u;
			wI = r[3];
			wL = r[4];
			wS = r[5];
			wend = count;
			wj = S.qa;
		} else {
			load_window(S.qa);
		}

	}
	Meta MA, MB;
	Block u0[U], u1[U];
	if (run) {
		meta_of(gA, MA);
		load_u(u0, MA, 0);  // in flight while the tables are written
	}
	FDBCRC_BT2(3)
	if (NP) lds_barrier();  // every wave has read the ring before any table word overwrites it
	fill_commit_1024(fill, lds);
#ifdef FDBCRC_BTIMES
	const uint64_t bt1 = __builtin_amdgcn_s_memrealtime();
#endif
	uint32_t f = 0;
	// one grab: X is its metadata; Y becomes the next grab's (its first unit
	// is loaded here)
	auto step = [&](Meta& X, Meta& Y) {
		const uint32_t l0 = f * C;
		uint32_t crc[U];
		const uint32_t req = request();
		load_u(u1, X, U);
		__builtin_amdgcn_sched_barrier(0);
		crc_u(u0, X, 0, crc);
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) mine = lane == l0 + j ? crc[j] : mine;
		{  // lanes l0 .. l0 + C - 1 take the grab's blocks' kt and output index from lanes 0 .. C - 1
			const bool mine_grab = lane - l0 < C;
			const int src = (int)(((lane - l0) & (C - 1)) << 2);
			const uint32_t kt = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)X.kt);
			const uint32_t ix = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)X.idx);
			mkt = mine_grab ? kt : mkt;
			midx = mine_grab ? ix : midx;
			if (NP) {
				const uint32_t nt = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)X.nbt);
				mnbt = mine_grab ? nt : mnbt;
			}
		}
		__builtin_amdgcn_sched_barrier(0);
		const uint32_t gB = clampg(g0 + wpb + rdlane(req, 0));
		meta_of(gB, Y);
		load_u(u0, Y, 0);  // the next grab's first unit
		__builtin_amdgcn_sched_barrier(0);
		crc_u(u1, X, U, crc);
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) mine = lane == l0 + U + j ? crc[j] : mine;
		__builtin_amdgcn_sched_barrier(0);
		gA = gB;
		if (++f == F) {
			store();
			f = 0;
		}
	};
	// two grabs per iteration: the metadata registers swap roles instead of
	// being copied
	if (run) {
		while (gA < ngrab) {
			step(MA, MB);
			if (gA >= ngrab) break;
			step(MB, MA);
		}
		if (f) store();
	}
#ifdef FDBCRC_BTIMES
	const uint64_t bt2 = __builtin_amdgcn_s_memrealtime();
#endif
	if (NP) {
		// buffers shorter than 16 bytes, byte by byte (the 1-byte table of the
		// LDS image), spread over the workgroups by index
		KBig* const K = big_kargs();
		const uint64_t i0 = (uint64_t)threadIdx.x * S.m;
		for (uint32_t msk = S.smallm; msk;) {
			const uint32_t j = (uint32_t)__builtin_ctz(msk);
			msk &= msk - 1;
			const uint64_t i = i0 + j;
			if (i % ngrid != blockIdx.x) continue;
			const uint8_t* b = K->base + K->offsets[i];
			const uint32_t len = (uint32_t)K->lengths[i];
			uint32_t r = ~(K->seeds ? K->seeds[i] : K->seed);
			for (uint32_t k = 0; k < len; ++k)
				r = (r >> 8) ^ lds_rd(lds, (0x10000u | (((r ^ ld1(b + k)) & 255u) << 8) | col4) + 128);
			K->out[i] = ~r;
		}
		// the stream's route statistics for its next batch (v7_route_stats)
		uint64_t* const hs = K->hstat;
		if (blockIdx.x == 0 && threadIdx.x == 0 && hs) {
			const uint64_t* const park = reinterpret_cast<const uint64_t*>(K->acc + 2 * kNPMax);
			for (int k = 0; k < 3; ++k) hs[k] = park[k];
			hs[kHstatPacked] = park[3] ? 0 : 1;
			if (hs[kHstatXfail] > 0 && hs[kHstatXfail] <= kXfailBackoff) --hs[kHstatXfail];
		}
	}
#ifdef FDBCRC_BTIMES
	if (lane == 0) {  // start, stream end, stream start, kernel end (after the prep-free tail)
		const uint32_t w = blockIdx.x * wpb + wi;
		g_bt[w][0] = bt0;
		g_bt[w][1] = bt2;
		g_bt[w][2] = bt1;
		g_bt[w][3] = __builtin_amdgcn_s_memrealtime();
	}
#endif
	// every request of every wave has returned: the counter goes back to zero
	__builtin_amdgcn_s_waitcnt(0);
	__syncthreads();
	if (threadIdx.x == 0) *my_ctr = 0;
}

int launch_bigblocks(const BigParams& P, int num_cus, hipStream_t stream) {
	// the block count lives on the device: one workgroup per CU, waves
	// without a grab leave at once
	k_bigblocks<FDBCRC_PU, false><<<(unsigned)num_cus, 1024, 0, stream>>>(P);
	return 0;
}

int launch_bigblocks_np(const BigParams& P, int num_cus, hipStream_t stream) {
	if (P.nbuf == 0 || P.nbuf > kNPMax || !P.offsets || !P.lengths || !P.acc || !P.priv || !P.ctr) return -1;
	k_bigblocks<FDBCRC_PU, true><<<(unsigned)num_cus, 1024, 0, stream>>>(P);
	return 0;
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// At most one workgroup per CU, and at least one grab per wave.
static unsigned page_grid(uint64_t pages, int num_cus) {
	const uint64_t grabs = (pages + 2 * FDBCRC_PU - 1) / (2 * FDBCRC_PU);
	uint64_t grid = (grabs + 15) / 16;
	if (grid > (uint64_t)num_cus) grid = num_cus;
	return grid ? (unsigned)grid : 1u;
}

int launch_pages(int blocks_per_page, const uint8_t* base, uint64_t stride, uint64_t count, uint32_t seed,
                 const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream) {
	if (count == 0) return 0;  // the kernels clamp page indices into a non-empty batch
	uint32_t* ctr;
	if (page_counters(stream, num_cus, &ctr)) return -1;
	switch (blocks_per_page) {
		case 1:
			k_pages4k<FDBCRC_PU><<<page_grid(count, num_cus), 1024, 0, stream>>>(base, stride, count, seed, seeds, out,
			                                                                      tabs, ctr);
			break;
		case 2:  // 8 KiB pages as block pairs on the 4 KiB kernel
			k_pages4k<FDBCRC_PU, false, false, true><<<page_grid(2 * count, num_cus), 1024, 0, stream>>>(
			    base, stride, count, seed, seeds, out, tabs, ctr);
			break;
		default: return -1;
	}
	return 0;
}

// Bytes [h, 4096 - t) of 4 KiB pages; `pages` is 16-byte aligned (the page
// start, h bytes before the caller's window).
int launch_pages_window(const uint8_t* pages, uint64_t stride, uint64_t count, uint32_t h, uint32_t t, uint32_t seed,
                        const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream) {
	if (count == 0) return 0;
	uint32_t* ctr;
	if (page_counters(stream, num_cus, &ctr)) return -1;
	k_pages4k<FDBCRC_PU, true><<<page_grid(count, num_cus), 1024, 0, stream>>>(pages, stride, count, seed, seeds, out,
	                                                                          tabs, ctr, h, t);
	return 0;
}

// Same over a device-side list: page j of the batch = page idx[j], j < *d_count
// (max_count bounds the grid).
int launch_pages_window_list(const uint8_t* pages, uint64_t stride, const uint32_t* idx, const uint64_t* d_count,
                             uint64_t max_count, uint32_t h, uint32_t t, uint32_t seed, uint32_t* out,
                             const DevTables* tabs, int num_cus, hipStream_t stream) {
	if (max_count == 0) return 0;
	uint32_t* ctr;
	if (page_counters(stream, num_cus, &ctr)) return -1;
	k_pages4k<FDBCRC_PU, true, true><<<page_grid(max_count, num_cus), 1024, 0, stream>>>(
	    pages, stride, max_count, seed, nullptr, out, tabs, ctr, h, t, idx, d_count);
	return 0;
}

#ifdef FDBCRC_DEBUG
// Debug builds: this file's copy of the load window (crc32c_common.h keeps one
// per translation unit), set and read together with the varlen file's.
__global__ void k_dbg_set_pages(unsigned long long lo, unsigned long long hi) {
	g_dbg[0] = lo; g_dbg[1] = hi;
	for (int k = 2; k < 8; ++k) g_dbg[k] = 0;
}
__global__ void k_dbg_get_pages(unsigned long long* out) {
	for (int k = 0; k < 8; ++k) out[k] = g_dbg[k];
}
void dbg_set_pages(uint64_t lo, uint64_t hi) { k_dbg_set_pages<<<1, 1>>>(lo, hi); }
void dbg_get_pages(uint64_t* d_out8) { k_dbg_get_pages<<<1, 1>>>(reinterpret_cast<unsigned long long*>(d_out8)); }
#endif

__global__ void k_fill_seeds(uint64_t count, uint32_t seed, const uint32_t* __restrict__ seeds,
                             uint32_t* __restrict__ out) {
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
		out[i] = seeds ? seeds[i] : seed;
}

// Zero-length buffers: crc32c_append(seed, p, 0) == seed.
int launch_fill_seeds(uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out, hipStream_t stream) {
	uint64_t grid = (count + 255) / 256;
	if (grid > 4096) grid = 4096;
	k_fill_seeds<<<(unsigned)grid, 256, 0, stream>>>(count, seed, seeds, out);
	return 0;
}

}  // namespace fdbcrc

#ifdef FDBCRC_BTIMES
extern "C" int fdbcrc_debug_btimes(void* host, uint64_t nwave) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbcrc::g_bt), nwave * 32, 0, hipMemcpyDeviceToHost);
}
extern "C" int fdbcrc_debug_btimes2(void* host, uint64_t nwave) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbcrc::g_bt2), nwave * 32, 0, hipMemcpyDeviceToHost);
}
#endif
