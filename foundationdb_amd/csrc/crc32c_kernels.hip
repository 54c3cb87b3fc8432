// Batched CRC-32C on MI355X (gfx950).  Hand-written HIP, wave64, no MFMA.
//
// Replaces, for batches of device-resident buffers, the per-buffer loop that
// every FoundationDB caller runs over crc32c_append()
// (contrib/crc32/include/crc32/crc32c.h:36-39, contrib/crc32/crc32c.cpp:346-356).
// Results are bit-identical to that function for every (seed, bytes, length).
//
// Geometry (see DESIGN.md for the derivation and the measurements behind it):
//   * One wavefront owns one buffer at a time.  The buffer is read in ROWS of
//     1 KiB: lane l loads the 16 bytes at row*1024 + 16*l with one
//     global_load_dwordx4, so every load instruction is a fully coalesced
//     1 KiB window (measured 7.2 TB/s read on MI355X; per-lane-contiguous
//     layouts measured 2-3.9 TB/s and are rejected).
//   * Each lane keeps a raw CRC register over its column of 16-byte chunks.
//     Moving from row r to row r+1 multiplies the register by x^(8*1008)
//     (the 1008 bytes of other lanes' chunks between two of this lane's
//     chunks) and then feeds the next 16 bytes.  This is append_hw's stream
//     merge (crc32c.cpp:268-269) with a GPU-shaped distance.
//   * After the last row lane l multiplies by x^(128*(63-l)) (its distance to
//     the end of the row) and the 64 registers are xor-reduced across the
//     wave (DPP row reductions + 4 readlanes).
//   * All table lookups hit LDS images that are replicated across the 32
//     banks (lane l reads column l%32), so every ds_read_b32 is conflict-free.
//     The data path uses 2-byte slicing (two 256-entry tables, 64 KiB image),
//     the two shift operators use 4-bit nibble tables (16 KiB + 32 KiB).
//   * Seed: lane 0 starts from ~seed instead of 0 (the register value at the
//     first byte), exactly the pre-inversion of append_hw (crc32c.cpp:197);
//     the result is post-inverted (crc32c.cpp:310).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace fdbcrc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// LDS image
// ---------------------------------------------------------------------------
// byte offsets into the LDS image
constexpr uint32_t kSliceOff = 0x00000;   // [256 idx][2 tab][32 col]  64 KiB
constexpr uint32_t kHornerOff = 0x10000;  // [8 nib][16 v][32 col]     16 KiB
constexpr uint32_t kLaneOff = 0x14000;    // [2 half][8 nib][16 v][32 col] 32 KiB
constexpr uint32_t kLdsBytes = 0x1C000;   // 112 KiB
constexpr uint32_t kTabT1 = 0;            // slice table: byte followed by one zero byte
constexpr uint32_t kTabT0 = 128;          // slice table: single byte

__device__ __forceinline__ uint32_t lds_rd(const uint32_t* lds, uint32_t byte_addr) {
	return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Copy the compact tables into the bank-replicated LDS image.
__device__ void fill_lds(uint32_t* lds, const DevTables* __restrict__ t) {
	constexpr uint32_t kWords = kLdsBytes / 4;
	for (uint32_t q = threadIdx.x; q < kWords; q += blockDim.x) {
		uint32_t v;
		const uint32_t col = q & 31;
		if (q < 16384) {
			v = t->slice[(q >> 5) & 1][q >> 6];
		} else if (q < 20480) {
			const uint32_t r = q - 16384;
			v = t->horner[r >> 9][(r >> 5) & 15];
		} else {
			const uint32_t r = q - 20480;
			v = t->lane[(r >> 12) * 32 + col][(r >> 9) & 7][(r >> 5) & 15];
		}
		lds[q] = v;
	}
	__syncthreads();
}

struct LaneCtx {
	uint32_t c_slice;   // col*4                        (slice image, perm byte 0)
	uint32_t c_horner;  // kHornerOff | col*4
	uint32_t c_lane;    // kLaneOff + half*16 KiB | col*4
	int lane;
};

__device__ __forceinline__ LaneCtx make_ctx() {
	LaneCtx c;
	c.lane = threadIdx.x & 63;
	const uint32_t col4 = (c.lane & 31) * 4;
	c.c_slice = kSliceOff | col4;
	c.c_horner = kHornerOff | col4;
	c.c_lane = (kLaneOff + (c.lane >> 5) * 0x4000) | col4;
	return c;
}

// Two bytes of register update: x already holds (register ^ data).
//   x' = (x >> 16) ^ T1[x.b0] ^ T0[x.b1]
__device__ __forceinline__ uint32_t half_step(const uint32_t* lds, uint32_t x, uint32_t c_slice) {
	const uint32_t a0 = __builtin_amdgcn_perm(x, c_slice, 0x0c0c0400u);  // (x.b0 << 8) | col*4
	const uint32_t a1 = __builtin_amdgcn_perm(x, c_slice, 0x0c0c0500u);  // (x.b1 << 8) | col*4
	return xor3(x >> 16, lds_rd(lds, a0 + kTabT1), lds_rd(lds, a1 + kTabT0));
}

// Feed 16 bytes (one chunk) into register s.
__device__ __forceinline__ uint32_t feed16(const uint32_t* lds, uint32_t s, u32x4 w, uint32_t c_slice) {
	s = half_step(lds, half_step(lds, s ^ w.x, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.y, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.z, c_slice), c_slice);
	s = half_step(lds, half_step(lds, s ^ w.w, c_slice), c_slice);
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

// One register byte step, wave-uniform (every lane computes the same value;
// lane l reads column l%32 so the lookup stays conflict-free).
__device__ __forceinline__ uint32_t byte_step(const uint32_t* lds, uint32_t s, uint32_t b, uint32_t c_slice) {
	const uint32_t a = __builtin_amdgcn_perm(s ^ b, c_slice, 0x0c0c0400u);
	return (s >> 8) ^ lds_rd(lds, a + kTabT0);
}

__device__ uint32_t feed_bytes(const uint32_t* lds, uint32_t s, const uint8_t* p, const uint8_t* e, uint32_t c_slice) {
	for (; p < e; ++p) s = byte_step(lds, s, *p, c_slice);
	return s;
}

// ---------------------------------------------------------------------------
// General buffer: any alignment, any length.  Wave-uniform in (p, len, seed).
//   head  [p, A)      A = p rounded up to 16       (<= 15 bytes, serial)
//   body  [A, B)      B = end rounded down to 16   (1 KiB rows, end-aligned)
//   tail  [B, end)                                 (<= 15 bytes, serial)
// The body's rows are aligned to its END: row 0 is front-padded with `pad`
// virtual chunks that read as zero.  Zeros in front of a zero register leave
// it zero, so the padding is free; the lane holding the body's first real
// chunk starts from the head's register instead of zero.
// ---------------------------------------------------------------------------
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
		const uint64_t m = (B - A) >> 4;                      // chunks in the body
		const uint32_t pad = (uint32_t)((64 - (m & 63)) & 63);
		const uint64_t rows = (m + pad) >> 6;
		const uint8_t* body = reinterpret_cast<const uint8_t*>(A);
		int64_t j = (int64_t)c.lane - (int64_t)pad;            // chunk index of this lane in row 0
		uint32_t acc = ((uint32_t)c.lane == pad) ? s : 0u;
		u32x4 cur = j >= 0 ? ld16(body + 16 * j) : u32x4{0u, 0u, 0u, 0u};
		for (uint64_t r = 0; r < rows; ++r) {
			u32x4 nxt = u32x4{0u, 0u, 0u, 0u};
			if (r + 1 < rows) nxt = ld16(body + 16 * (j + 64));
			if (r) acc = mul_nibbles(lds, acc, c.c_horner);
			acc = feed16(lds, acc, cur, c.c_slice);
			cur = nxt;
			j += 64;
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
	const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < count; i += waves) {
		const uint8_t* p = offsets ? base + offsets[i] : base + i * stride;
		const uint64_t n = lengths ? lengths[i] : length;
		const uint32_t s0 = seeds ? seeds[i] : seed;
		const uint32_t r = crc_buffer_wave(lds, c, p, n, s0);
		if (c.lane == 0) out[i] = r;
	}
}

// Fast path: 16-byte aligned buffers of exactly ROWS KiB at a 16-byte aligned
// stride (4 KiB pages: ROWS = 4; 8 KiB sqlite pages: ROWS = 8).
// A wave walks GROUP consecutive buffers, prefetching buffer i+1 while it
// folds buffer i, and stores the GROUP checksums as one coalesced write.
template <int ROWS>
__global__ __launch_bounds__(1024) void k_pages(const uint8_t* __restrict__ base, uint64_t stride, uint64_t count,
                                                uint32_t seed, const uint32_t* __restrict__ seeds,
                                                uint32_t* __restrict__ out, const DevTables* __restrict__ tabs) {
	__shared__ uint32_t lds[kLdsBytes / 4];
	fill_lds(lds, tabs);
	const LaneCtx c = make_ctx();
	constexpr uint64_t GROUP = 64;
	const uint64_t groups = (count + GROUP - 1) / GROUP;
	const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < groups; g += waves) {
		const uint64_t first = g * GROUP;
		const uint64_t n = count - first < GROUP ? count - first : GROUP;
		const uint8_t* p = base + first * stride + 16 * c.lane;
		u32x4 cur[ROWS], nxt[ROWS];
#pragma unroll
		for (int r = 0; r < ROWS; ++r) cur[r] = ld16(p + 1024 * r);
		uint32_t mine = 0;  // lane k keeps the checksum of buffer first+k
		for (uint64_t k = 0; k < n; ++k) {
			if (k + 1 < n) {
#pragma unroll
				for (int r = 0; r < ROWS; ++r) nxt[r] = ld16(p + stride + 1024 * r);
			}
			const uint32_t s0 = seeds ? seeds[first + k] : seed;
			uint32_t acc = c.lane == 0 ? ~s0 : 0u;
			acc = feed16(lds, acc, cur[0], c.c_slice);
#pragma unroll
			for (int r = 1; r < ROWS; ++r) acc = feed16(lds, mul_nibbles(lds, acc, c.c_horner), cur[r], c.c_slice);
			const uint32_t crc = ~wave_xor(mul_nibbles(lds, acc, c.c_lane));
			if ((uint64_t)c.lane == k) mine = crc;
#pragma unroll
			for (int r = 0; r < ROWS; ++r) cur[r] = nxt[r];
			p += stride;
		}
		if ((uint64_t)c.lane < n) out[first + c.lane] = mine;
	}
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
int launch_pages(int rows, const uint8_t* base, uint64_t stride, uint64_t count, uint32_t seed,
                 const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream) {
	const uint64_t groups = (count + 63) / 64;
	const int threads = 1024;
	uint64_t blocks = (groups + 15) / 16;
	if (blocks > (uint64_t)num_cus) blocks = num_cus;
	if (blocks == 0) blocks = 1;
	switch (rows) {
		case 1: k_pages<1><<<(unsigned)blocks, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		case 2: k_pages<2><<<(unsigned)blocks, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		case 4: k_pages<4><<<(unsigned)blocks, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		case 8: k_pages<8><<<(unsigned)blocks, threads, 0, stream>>>(base, stride, count, seed, seeds, out, tabs); break;
		default: return -1;
	}
	return 0;
}

int launch_general(const uint8_t* base, uint64_t stride, uint64_t length, const uint64_t* offsets,
                   const uint64_t* lengths, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                   const DevTables* tabs, int num_cus, hipStream_t stream) {
	const int threads = 1024;
	uint64_t blocks = (count + 15) / 16;
	if (blocks > (uint64_t)num_cus) blocks = num_cus;
	if (blocks == 0) blocks = 1;
	k_general<<<(unsigned)blocks, threads, 0, stream>>>(base, stride, length, offsets, lengths, count, seed, seeds, out,
	                                                   tabs);
	return 0;
}

}  // namespace fdbcrc
