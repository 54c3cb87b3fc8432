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
template <int U, bool WINDOW = false, bool LIST = false, bool PAIR = false>
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
	const uint64_t per = (ngrab + gridDim.x - 1) / gridDim.x;
	const uint64_t g0 = (uint64_t)blockIdx.x * per;
	const uint64_t g1 = g0 + per < ngrab ? g0 + per : ngrab;
	uint32_t* const my_ctr = ctr + kPageCtrWords * blockIdx.x;
	const uint64_t last = count - 1;
	// page index -> address, clamped into the batch: clamped duplicates are
	// computed and discarded, so every load is consumed unconditionally
	auto page = [&](uint64_t i) {
		const uint64_t j = i < count ? i : last;
		if (PAIR) return base + (j >> 1) * stride + (j & 1) * 4096;
		return base + (LIST ? (uint64_t)idx[j] : j) * stride;
	};
	auto load_u = [&](Block (&u)[U], uint64_t i0) {
#pragma unroll
		for (int j = 0; j < U; ++j) load_block(u[j], page(i0 + j), c.ld_off);
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
	uint64_t gA = clampg(g0 + wi), gB = clampg(g0 + wi + wpb);
	uint32_t req = request();  // grab g0 + 2*wpb + req: becomes gB after grab A
	uint32_t sdA = seed_of(gA), sdB = seed_of(gB);
	Block u0[U], u1[U];
	load_u(u0, gA * C);  // in flight during the LDS fill
	fill_lds_b(lds, tabs);
	uint32_t mine = 0;     // lane 2U*f + j: checksum of page j of the group's f-th grab
	uint64_t myi = ~0ull;  // ... and its index in the batch (~0: none)
	uint32_t f = 0;        // grabs in the current store group
	auto store = [&]() {
		if (WINDOW) mine = ~(t ? vmul_tab(tabs->inv_z[t], mine) : mine);
		if (PAIR) {
			const uint32_t other = __builtin_amdgcn_update_dpp(0u, mine, 0xB1, 0xF, 0xF, false);  // lane ^ 1
			mine = ~(vmul_tab(tabs->block, mine) ^ other);
			if (myi < count && !(c.lane & 1)) out[myi >> 1] = mine;
		} else if (myi < count) {
			out[myi] = mine;
		}
		myi = ~0ull;
	};
	while (gA < ngrab) {
		const uint64_t first = gA * C;
		const uint32_t l0 = f * C;
		uint32_t sd[U], crc[U];
		load_u(u1, first + U);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int j = 0; j < U; ++j) sd[j] = rdlane(sdA, j);
		unit_crc_b<U, WINDOW, WINDOW || PAIR>(lds, c.lane, c4, c_lane, u0, sd, crc, h, t);
#pragma unroll
		for (int j = 0; j < U; ++j) mine = (uint32_t)c.lane == l0 + j ? crc[j] : mine;
		__builtin_amdgcn_sched_barrier(0);
		load_u(u0, gB * C);  // the next grab's first unit
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int j = 0; j < U; ++j) sd[j] = rdlane(sdA, U + j);
		unit_crc_b<U, WINDOW, WINDOW || PAIR>(lds, c.lane, c4, c_lane, u1, sd, crc, h, t);
#pragma unroll
		for (int j = 0; j < U; ++j) mine = (uint32_t)c.lane == l0 + U + j ? crc[j] : mine;
		__builtin_amdgcn_sched_barrier(0);
		const uint32_t k = (uint32_t)c.lane - l0;
		myi = k < C ? first + k : myi;
		gA = gB;
		sdA = sdB;
		gB = clampg(g0 + 2 * wpb + rdlane(req, 0));
		req = request();
		sdB = seed_of(gB);
		if (++f == F) {
			store();
			f = 0;
		}
	}
	if (f) store();
	// every request of every wave has returned: the counter goes back to zero
	// for the next launch on this stream
	__builtin_amdgcn_s_waitcnt(0);
	__syncthreads();
	if (threadIdx.x == 0) *my_ctr = 0;
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
