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
//   * Each lane runs one CRC register over its 64 bytes (2-byte slicing from
//     bank-replicated LDS tables: every ds_read_b32 is conflict-free).
//   * Lane l then multiplies its register by x^(8*64*(63-l)) -- its distance
//     to the end of the block -- and the 64 registers are xor-reduced across
//     the wave (DPP row reduction + 4 readlanes).  Consecutive blocks of one
//     buffer fold Horner-style with x^(8*4096).  This is append_hw's stream
//     merge (crc32c.cpp:268-269) with GPU-shaped distances.
//   * Seed: the register at the buffer's first byte is ~seed, as in
//     append_hw's pre-inversion (crc32c.cpp:197); the result is post-inverted
//     (crc32c.cpp:310).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace fdbcrc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// LDS image (byte offsets).  Lane l always reads bank column l%32.
// ---------------------------------------------------------------------------
constexpr uint32_t kSliceOff = 0x00000;  // [256 idx][2 tab][32 col]         64 KiB
constexpr uint32_t kBlockOff = 0x10000;  // [8 nib][16 v][32 col]            16 KiB  x^(8*4096)
constexpr uint32_t kLaneOff = 0x14000;   // [2 half][8 nib][16 v][32 col]    32 KiB  x^(8*64*(63-l))
constexpr uint32_t kLdsBytes = 0x1C000;  // 112 KiB -> one 1024-thread workgroup per CU
constexpr uint32_t kTabT1 = 0;           // slice table: byte followed by one zero byte
constexpr uint32_t kTabT0 = 128;         // slice table: single byte

// Layout B (4 KiB page kernel only): 4-byte slicing, 160 KiB = all of LDS.
//   region 0 [idx][T3,T2][col], region 1 [idx][T1,T0][col], then lane tables.
constexpr uint32_t kS4Off = 0x00000;     // 2 x 64 KiB
constexpr uint32_t kS4LaneOff = 0x20000; // [2 half][8 nib][16 v][32 col]    32 KiB  x^(8*64*(63-l))
constexpr uint32_t kLdsBytesB = 0x28000; // 160 KiB

__device__ __forceinline__ uint32_t lds_rd(const uint32_t* lds, uint32_t byte_addr) {
	return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Expand the compact tables into the bank-replicated LDS image.  Each thread
// first issues all of its (independent) global loads, then writes: slice and
// block-shift values go to all 32 bank columns, lane-combine values to the
// one column (lane%32) of the lane they belong to.
__device__ void fill_lds(uint32_t* lds, const DevTables* __restrict__ t) {
	constexpr uint32_t kSlice = 512, kBlock = 128, kLane = 64 * 128;
	constexpr uint32_t kCompact = kSlice + kBlock + kLane;  // 8832 words
	constexpr uint32_t kPer = (kCompact + 1023) / 1024;
	const uint32_t* src = reinterpret_cast<const uint32_t*>(t);
	uint32_t v[kPer];
#pragma unroll
	for (uint32_t i = 0; i < kPer; ++i) {
		const uint32_t q = threadIdx.x + i * blockDim.x;
		v[i] = q < kCompact ? src[q] : 0u;
	}
#pragma unroll
	for (uint32_t i = 0; i < kPer; ++i) {
		const uint32_t q = threadIdx.x + i * blockDim.x;
		if (q < kSlice) {  // slice[tab][idx] -> [idx][tab][col]
			const uint32_t tab = q >> 8, idx = q & 255;
			uint32_t* d = lds + (kSliceOff / 4) + (idx * 2 + tab) * 32;
#pragma unroll
			for (int c = 0; c < 32; ++c) d[c] = v[i];
		} else if (q < kSlice + kBlock) {  // block[nib][v] -> [nib][v][col]
			uint32_t* d = lds + (kBlockOff / 4) + (q - kSlice) * 32;
#pragma unroll
			for (int c = 0; c < 32; ++c) d[c] = v[i];
		} else if (q < kCompact) {  // lane[l][nib][v] -> [l/32][nib][v][l%32]
			const uint32_t r = q - kSlice - kBlock;
			const uint32_t l = r >> 7, nv = r & 127;
			lds[(kLaneOff / 4) + (l >> 5) * 4096 + nv * 32 + (l & 31)] = v[i];
		}
	}
	__syncthreads();
}

// Layout B fill: slice4 (1024 words) to all 32 columns, lane tables to their column.
__device__ void fill_lds_b(uint32_t* lds, const DevTables* __restrict__ t) {
	constexpr uint32_t kSlice = 1024, kLane = 64 * 128;
	constexpr uint32_t kCompact = kSlice + kLane;  // 9216 words
	constexpr uint32_t kPer = (kCompact + 1023) / 1024;
	const uint32_t* s4 = &t->slice4[0][0];
	const uint32_t* ln = &t->lane[0][0][0];
	uint32_t v[kPer];
#pragma unroll
	for (uint32_t i = 0; i < kPer; ++i) {
		const uint32_t q = threadIdx.x + i * blockDim.x;
		v[i] = q < kSlice ? s4[q] : (q < kCompact ? ln[q - kSlice] : 0u);
	}
#pragma unroll
	for (uint32_t i = 0; i < kPer; ++i) {
		const uint32_t q = threadIdx.x + i * blockDim.x;
		if (q < kSlice) {  // slice4[k][idx], k = 0..3 -> T3,T2 | T1,T0 regions
			const uint32_t k = q >> 8, idx = q & 255;
			uint32_t* d = lds + (kS4Off / 4) + (k >> 1) * 16384 + (idx * 2 + (k & 1)) * 32;
#pragma unroll
			for (int c = 0; c < 32; ++c) d[c] = v[i];
		} else if (q < kCompact) {
			const uint32_t r = q - kSlice;
			const uint32_t l = r >> 7, nv = r & 127;
			lds[(kS4LaneOff / 4) + (l >> 5) * 4096 + nv * 32 + (l & 31)] = v[i];
		}
	}
	__syncthreads();
}

struct LaneCtx {
	uint32_t c_slice;  // col*4
	uint32_t c_block;  // kBlockOff | col*4
	uint32_t c_lane;   // kLaneOff + half*16 KiB | col*4
	uint32_t ld_off;   // byte offset of this lane's first 16 B load inside a block
	int lane;
};

__device__ __forceinline__ LaneCtx make_ctx() {
	LaneCtx c;
	c.lane = threadIdx.x & 63;
	const uint32_t col4 = (c.lane & 31) * 4;
	c.c_slice = kSliceOff | col4;
	c.c_block = kBlockOff | col4;
	c.c_lane = (kLaneOff + (c.lane >> 5) * 0x4000) | col4;
	// lane m = 32h + 16q + r loads, for load k = 2kb + ka, the 16 bytes at
	//   2048*ka + 1024*kb + 64r + 32q + 16h
	// which after the swap network (unswizzle) puts block bytes
	// [64l, 64l+64) into lane l as registers r[0..3].
	const uint32_t h = c.lane >> 5, q = (c.lane >> 4) & 1, r = c.lane & 15;
	c.ld_off = 64 * r + 32 * q + 16 * h;
	return c;
}

// Two bytes of register update: x already holds (register ^ data).
//   x' = (x >> 16) ^ T1[x.b0] ^ T0[x.b1]
__device__ __forceinline__ uint32_t half_step(const uint32_t* lds, uint32_t x, uint32_t c_slice) {
	const uint32_t a0 = __builtin_amdgcn_perm(x, c_slice, 0x0c0c0400u);  // (x.b0 << 8) | col*4
	const uint32_t a1 = __builtin_amdgcn_perm(x, c_slice, 0x0c0c0500u);  // (x.b1 << 8) | col*4
	return xor3(x >> 16, lds_rd(lds, a0 + kTabT1), lds_rd(lds, a1 + kTabT0));
}

// Feed 16 bytes into register s.
__device__ __forceinline__ uint32_t feed16(const uint32_t* lds, uint32_t s, u32x4 w, uint32_t c_slice) {
	s = half_step(lds, half_step(lds, s ^ w.x, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.y, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.z, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.w, c_slice), c_slice);
	return s;
}

// Layout B: four bytes per step, s' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]
// with x = s ^ word.  c4 = col*4 | 0x10000 (byte 2 selects region 1).
__device__ __forceinline__ uint32_t word_step4(const uint32_t* lds, uint32_t x, uint32_t c4) {
	const uint32_t a3 = __builtin_amdgcn_perm(x, c4, 0x0c0c0400u);  // (x.b0 << 8) | col*4
	const uint32_t a2 = __builtin_amdgcn_perm(x, c4, 0x0c0c0500u);  // (x.b1 << 8) | col*4
	const uint32_t a1 = __builtin_amdgcn_perm(x, c4, 0x0c020600u);  // 0x10000 | (x.b2 << 8) | col*4
	const uint32_t a0 = __builtin_amdgcn_perm(x, c4, 0x0c020700u);  // 0x10000 | (x.b3 << 8) | col*4
	return xor3(lds_rd(lds, a3), lds_rd(lds, a2 + 128), lds_rd(lds, a1)) ^ lds_rd(lds, a0 + 128);
}

__device__ __forceinline__ uint32_t feed16_b(const uint32_t* lds, uint32_t s, u32x4 w, uint32_t c4) {
	s = word_step4(lds, s ^ w.x, c4);
	s = word_step4(lds, s ^ w.y, c4);
	s = word_step4(lds, s ^ w.z, c4);
	s = word_step4(lds, s ^ w.w, c4);
	return s;
}

// Multiply a register by the constant whose nibble tables start at `base`
// (base already carries the lane's column).
__device__ __forceinline__ uint32_t mul_nibbles(const uint32_t* lds, uint32_t s, uint32_t base) {
	uint32_t r[8];
#pragma unroll
	for (int n = 0; n < 8; ++n) {
		const uint32_t v = (s >> (4 * n)) & 15u;
		r[n] = lds_rd(lds, ((v << 7) | base) + n * 2048);
	}
	return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// XOR of v over all 64 lanes, returned wave-uniform.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false);  // row_ror:4
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
	return __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^
	       __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
	return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// ---------------------------------------------------------------------------
// 4 KiB blocks
// ---------------------------------------------------------------------------
struct Block {
	u32x4 r[4];
};

__device__ __forceinline__ void load_block(Block& b, const uint8_t* block, uint32_t ld_off) {
	const uint8_t* p = block + ld_off;
	b.r[0] = ld16(p);
	b.r[1] = ld16(p + 2048);
	b.r[2] = ld16(p + 1024);
	b.r[3] = ld16(p + 3072);
}

__device__ __forceinline__ void swap32(u32x4& x, u32x4& y) {
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const auto t = __builtin_amdgcn_permlane32_swap(x[i], y[i], false, false);
		x[i] = t[0];
		y[i] = t[1];
	}
}

__device__ __forceinline__ void swap16(u32x4& x, u32x4& y) {
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const auto t = __builtin_amdgcn_permlane16_swap(x[i], y[i], false, false);
		x[i] = t[0];
		y[i] = t[1];
	}
}

// After this, lane l holds block bytes [64l, 64l+64) in r[0..3].
__device__ __forceinline__ void unswizzle(Block& b) {
	swap32(b.r[0], b.r[1]);
	swap32(b.r[2], b.r[3]);
	swap16(b.r[0], b.r[2]);
	swap16(b.r[1], b.r[3]);
}

// Register of this lane after its 64 bytes, starting from s.
__device__ __forceinline__ uint32_t chain64(const uint32_t* lds, uint32_t s, const Block& b, uint32_t c_slice) {
	s = feed16(lds, s, b.r[0], c_slice);
	s = feed16(lds, s, b.r[1], c_slice);
	s = feed16(lds, s, b.r[2], c_slice);
	s = feed16(lds, s, b.r[3], c_slice);
	return s;
}

// ---------------------------------------------------------------------------
// Fixed-stride pages of NB*4 KiB (16-byte aligned base and stride).
// Every wave owns a contiguous run of pages and works on UNIT = 2 blocks at a
// time (two 4 KiB pages, or one 8 KiB page) while the next unit's loads are
// in flight.  The two blocks' register chains interleave (ILP 2).  Control
// flow is scalar (readfirstlane'd wave id); seeds arrive as one vector load
// per 64 pages, checksums leave as one coalesced store per 64 pages.
// ---------------------------------------------------------------------------
template <int NB>  // 4 KiB blocks per page: 1 or 2
__device__ __forceinline__ void unit_crc(const uint32_t* lds, const LaneCtx& c, Block (&u)[2], uint32_t sa,
                                         uint32_t sb, uint32_t& ca, uint32_t& cb) {
	unswizzle(u[0]);
	unswizzle(u[1]);
	if (NB == 1) {  // two pages
		const uint32_t x0 = chain64(lds, c.lane == 0 ? ~sa : 0u, u[0], c.c_slice);
		const uint32_t x1 = chain64(lds, c.lane == 0 ? ~sb : 0u, u[1], c.c_slice);
		ca = ~wave_xor(mul_nibbles(lds, x0, c.c_lane));
		cb = ~wave_xor(mul_nibbles(lds, x1, c.c_lane));
	} else {  // one 8 KiB page
		const uint32_t x0 = chain64(lds, c.lane == 0 ? ~sa : 0u, u[0], c.c_slice);
		const uint32_t x1 = chain64(lds, 0u, u[1], c.c_slice);
		const uint32_t acc = mul_nibbles(lds, x0, c.c_block) ^ x1;
		ca = ~wave_xor(mul_nibbles(lds, acc, c.c_lane));
		cb = ca;
	}
}

template <int NB>
__device__ __forceinline__ void load_unit(Block (&u)[2], const uint8_t* p0, const uint8_t* p1, uint32_t ld_off) {
	if (NB == 1) {
		load_block(u[0], p0, ld_off);
		load_block(u[1], p1, ld_off);
	} else {
		load_block(u[0], p0, ld_off);
		load_block(u[1], p0 + 4096, ld_off);
	}
}

template <int NB>
__global__ __launch_bounds__(1024) void k_pages(const uint8_t* __restrict__ base, uint64_t stride, uint64_t count,
                                                uint32_t seed, const uint32_t* __restrict__ seeds,
                                                uint32_t* __restrict__ out, const DevTables* __restrict__ tabs) {
	__shared__ uint32_t lds[kLdsBytes / 4];
	constexpr uint64_t PPU = NB == 1 ? 2 : 1;  // pages per unit
	const LaneCtx c = make_ctx();
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t wave = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint64_t waves = (uint64_t)gridDim.x * wpb;
	uint64_t per = (count + waves - 1) / waves;
	per = per > 64 ? (per + 63) & ~uint64_t(63) : (per + PPU - 1) / PPU * PPU;
	const uint64_t begin = wave * per;
	const uint64_t end = begin + per < count ? begin + per : count;
	const uint64_t last = end ? end - 1 : 0;
	// page index -> address, clamped into this wave's run (clamped duplicates
	// are computed and discarded, so every load is consumed unconditionally)
	auto page = [&](uint64_t i) { return base + (i < end ? i : (begin < end ? last : 0)) * stride; };
	Block u0[2], u1[2];
	load_unit<NB>(u0, page(begin), page(begin + 1), c.ld_off);  // in flight during the LDS fill
	fill_lds(lds, tabs);
	if (begin >= end) return;
	for (uint64_t first = begin; first < end; first += 64) {
		const uint64_t n = end - first < 64 ? end - first : 64;
		const uint32_t my_seed = seeds ? seeds[first + ((uint64_t)c.lane < n ? c.lane : 0)] : seed;
		uint32_t mine = 0;  // lane k keeps the checksum of page first+k
		for (uint64_t k = 0; k < n; k += 2 * PPU) {
			uint32_t ca, cb;
			load_unit<NB>(u1, page(first + k + PPU), page(first + k + PPU + 1), c.ld_off);
			__builtin_amdgcn_sched_barrier(0);
			unit_crc<NB>(lds, c, u0, __builtin_amdgcn_readlane(my_seed, (int)k),
			             __builtin_amdgcn_readlane(my_seed, (int)(k + 1) & 63), ca, cb);
			mine = (uint64_t)c.lane == k ? ca : mine;
			if (PPU == 2) mine = (uint64_t)c.lane == k + 1 ? cb : mine;
			__builtin_amdgcn_sched_barrier(0);
			load_unit<NB>(u0, page(first + k + 2 * PPU), page(first + k + 2 * PPU + 1), c.ld_off);
			__builtin_amdgcn_sched_barrier(0);
			unit_crc<NB>(lds, c, u1, __builtin_amdgcn_readlane(my_seed, (int)(k + PPU) & 63),
			             __builtin_amdgcn_readlane(my_seed, (int)(k + PPU + 1) & 63), ca, cb);
			mine = (uint64_t)c.lane == k + PPU ? ca : mine;
			if (PPU == 2) mine = (uint64_t)c.lane == k + PPU + 1 ? cb : mine;
			__builtin_amdgcn_sched_barrier(0);
		}
		if ((uint64_t)c.lane < n) out[first + c.lane] = mine;
	}
}

// 4 KiB pages with the layout-B image (4-byte slicing: half the dependent
// LDS round trips and a third less VALU than layout A).
__device__ __forceinline__ uint32_t chain64_b(const uint32_t* lds, uint32_t s, const Block& b, uint32_t c4) {
	s = feed16_b(lds, s, b.r[0], c4);
	s = feed16_b(lds, s, b.r[1], c4);
	s = feed16_b(lds, s, b.r[2], c4);
	s = feed16_b(lds, s, b.r[3], c4);
	return s;
}

__device__ __forceinline__ void unit_crc_b(const uint32_t* lds, int lane, uint32_t c4, uint32_t c_lane,
                                           Block (&u)[2], uint32_t sa, uint32_t sb, uint32_t& ca, uint32_t& cb) {
	unswizzle(u[0]);
	unswizzle(u[1]);
	const uint32_t x0 = chain64_b(lds, lane == 0 ? ~sa : 0u, u[0], c4);
	const uint32_t x1 = chain64_b(lds, lane == 0 ? ~sb : 0u, u[1], c4);
	ca = ~wave_xor(mul_nibbles(lds, x0, c_lane));
	cb = ~wave_xor(mul_nibbles(lds, x1, c_lane));
}

__global__ __launch_bounds__(1024) void k_pages4k(const uint8_t* __restrict__ base, uint64_t stride, uint64_t count,
                                                  uint32_t seed, const uint32_t* __restrict__ seeds,
                                                  uint32_t* __restrict__ out, const DevTables* __restrict__ tabs) {
	__shared__ uint32_t lds[kLdsBytesB / 4];
	const LaneCtx c = make_ctx();
	const uint32_t col4 = (c.lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (c.lane >> 5) * 0x4000) | col4;
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t wave = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint64_t waves = (uint64_t)gridDim.x * wpb;
	uint64_t per = (count + waves - 1) / waves;
	per = per > 64 ? (per + 63) & ~uint64_t(63) : (per + 1) & ~uint64_t(1);
	const uint64_t begin = wave * per;
	const uint64_t end = begin + per < count ? begin + per : count;
	const uint64_t last = end ? end - 1 : 0;
	auto page = [&](uint64_t i) { return base + (i < end ? i : (begin < end ? last : 0)) * stride; };
	Block u0[2], u1[2];
	load_unit<1>(u0, page(begin), page(begin + 1), c.ld_off);  // in flight during the LDS fill
	fill_lds_b(lds, tabs);
	if (begin >= end) return;
	for (uint64_t first = begin; first < end; first += 64) {
		const uint64_t n = end - first < 64 ? end - first : 64;
		const uint32_t my_seed = seeds ? seeds[first + ((uint64_t)c.lane < n ? c.lane : 0)] : seed;
		uint32_t mine = 0;  // lane k keeps the checksum of page first+k
		for (uint64_t k = 0; k < n; k += 4) {
			uint32_t ca, cb;
			load_unit<1>(u1, page(first + k + 2), page(first + k + 3), c.ld_off);
			__builtin_amdgcn_sched_barrier(0);
			unit_crc_b(lds, c.lane, c4, c_lane, u0, __builtin_amdgcn_readlane(my_seed, (int)k),
			           __builtin_amdgcn_readlane(my_seed, (int)(k + 1) & 63), ca, cb);
			mine = (uint64_t)c.lane == k ? ca : mine;
			mine = (uint64_t)c.lane == k + 1 ? cb : mine;
			__builtin_amdgcn_sched_barrier(0);
			load_unit<1>(u0, page(first + k + 4), page(first + k + 5), c.ld_off);
			__builtin_amdgcn_sched_barrier(0);
			unit_crc_b(lds, c.lane, c4, c_lane, u1, __builtin_amdgcn_readlane(my_seed, (int)(k + 2) & 63),
			           __builtin_amdgcn_readlane(my_seed, (int)(k + 3) & 63), ca, cb);
			mine = (uint64_t)c.lane == k + 2 ? ca : mine;
			mine = (uint64_t)c.lane == k + 3 ? cb : mine;
			__builtin_amdgcn_sched_barrier(0);
		}
		if ((uint64_t)c.lane < n) out[first + c.lane] = mine;
	}
}

// ---------------------------------------------------------------------------
// General buffer: any alignment, any length.  Wave-uniform in (p, len, seed).
//   head  [p, A)      A = p rounded up to 16       (<= 15 bytes, serial)
//   body  [A, B)      B = end rounded down to 16   (4 KiB blocks, end-aligned)
//   tail  [B, end)                                 (<= 15 bytes, serial)
// The body's blocks are aligned to its END: block 0 is front-padded with
// `pad` virtual 16-byte chunks that read as zero.  Zeros fed into a zero
// register leave it zero, so the padding is free; the head's register is
// injected at the body's first real chunk.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_step(const uint32_t* lds, uint32_t s, uint32_t b, uint32_t c_slice) {
	const uint32_t a = __builtin_amdgcn_perm(s ^ b, c_slice, 0x0c0c0400u);
	return (s >> 8) ^ lds_rd(lds, a + kTabT0);
}

__device__ uint32_t feed_bytes(const uint32_t* lds, uint32_t s, const uint8_t* p, const uint8_t* e, uint32_t c_slice) {
	for (; p < e; ++p) s = byte_step(lds, s, *p, c_slice);
	return s;
}

__device__ __forceinline__ u32x4 ld16_if(const uint8_t* p, bool ok) {
	return ok ? ld16(p) : u32x4{0u, 0u, 0u, 0u};
}

__device__ uint32_t crc_buffer_wave(const uint32_t* lds, const LaneCtx& c, const uint8_t* p, uint64_t len,
                                    uint32_t seed) {
	if (len == 0) return seed;
	const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
	const uintptr_t ea = pa + len;
	const uintptr_t A = (pa + 15) & ~uintptr_t(15);
	const uintptr_t B = ea & ~uintptr_t(15);
	uint32_t s = ~seed;
	const uintptr_t head_end = A < ea ? A : ea;
	s = feed_bytes(lds, s, p, reinterpret_cast<const uint8_t*>(head_end), c.c_slice);
	if (B > A) {
		const uint64_t m = (B - A) >> 4;  // 16-byte chunks in the body
		const uint64_t nblk = (m + 255) >> 8;
		const uint32_t pad = (uint32_t)(nblk * 256 - m);
		// virtual block 0 starts pad chunks before the body
		const uint8_t* vbase = reinterpret_cast<const uint8_t*>(A) - 16 * (uint64_t)pad;
		const uint32_t o0 = c.ld_off, o1 = c.ld_off + 2048, o2 = c.ld_off + 1024, o3 = c.ld_off + 3072;
		const uint32_t pad_bytes = 16 * pad;
		// the first real chunk lands in lane pad/4, slot pad%4 after unswizzle
		const uint32_t inj_lane = pad >> 2, inj_slot = pad & 3;
		uint32_t acc = 0;
		Block b;
		b.r[0] = ld16_if(vbase + o0, o0 >= pad_bytes);
		b.r[1] = ld16_if(vbase + o1, o1 >= pad_bytes);
		b.r[2] = ld16_if(vbase + o2, o2 >= pad_bytes);
		b.r[3] = ld16_if(vbase + o3, o3 >= pad_bytes);
		for (uint64_t blk = 0; blk < nblk; ++blk) {
			Block nb;
			const uint8_t* next = vbase + 4096 * (blk + 1 < nblk ? blk + 1 : blk);
			load_block(nb, next, c.ld_off);
			unswizzle(b);
			uint32_t x = 0;
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				if (blk == 0 && (uint32_t)c.lane == inj_lane && (uint32_t)j == inj_slot) x ^= s;
				x = feed16(lds, x, b.r[j], c.c_slice);
			}
			acc = blk ? mul_nibbles(lds, acc, c.c_block) ^ x : x;
			b = nb;
		}
		s = wave_xor(mul_nibbles(lds, acc, c.c_lane));
	}
	const uintptr_t tail_start = A > B ? A : B;
	if (tail_start < ea)
		s = feed_bytes(lds, s, reinterpret_cast<const uint8_t*>(tail_start), reinterpret_cast<const uint8_t*>(ea),
		               c.c_slice);
	return ~s;
}

// Fixed-stride or offset-addressed batch, one wave per buffer (grid-stride).
__global__ __launch_bounds__(1024) void k_general(const uint8_t* __restrict__ base, uint64_t stride, uint64_t length,
                                                  const uint64_t* __restrict__ offsets,
                                                  const uint64_t* __restrict__ lengths, uint64_t count, uint32_t seed,
                                                  const uint32_t* __restrict__ seeds, uint32_t* __restrict__ out,
                                                  const DevTables* __restrict__ tabs) {
	__shared__ uint32_t lds[kLdsBytes / 4];
	fill_lds(lds, tabs);
	const LaneCtx c = make_ctx();
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t waves = (uint64_t)gridDim.x * wpb;
	for (uint64_t i = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); i < count;
	     i += waves) {
		const uint8_t* p = offsets ? base + offsets[i] : base + i * stride;
		const uint64_t n = lengths ? lengths[i] : length;
		const uint32_t s0 = seeds ? seeds[i] : seed;
		const uint32_t r = crc_buffer_wave(lds, c, p, n, s0);
		if (c.lane == 0) out[i] = r;
	}
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
int launch_pages(int blocks_per_page, const uint8_t* base, uint64_t stride, uint64_t count, uint32_t seed,
                 const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream) {
	const int threads = 1024;
	const uint64_t units = (count + 63) / 64;
	uint64_t grid = (units + 15) / 16;
	if (grid > (uint64_t)num_cus) grid = num_cus;
	if (grid == 0) grid = 1;
	switch (blocks_per_page) {
		case 1: k_pages4k<<<(unsigned)grid, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		case 2: k_pages<2><<<(unsigned)grid, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		default: return -1;
	}
	return 0;
}

int launch_general(const uint8_t* base, uint64_t stride, uint64_t length, const uint64_t* offsets,
                   const uint64_t* lengths, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                   const DevTables* tabs, int num_cus, hipStream_t stream) {
	const int threads = 1024;
	uint64_t grid = (count + 15) / 16;
	if (grid > (uint64_t)num_cus) grid = num_cus;
	if (grid == 0) grid = 1;
	k_general<<<(unsigned)grid, threads, 0, stream>>>(base, stride, length, offsets, lengths, count, seed, seeds, out,
	                                                 tabs);
	return 0;
}

}  // namespace fdbcrc
