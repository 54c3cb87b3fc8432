// Device-side building blocks shared by the page and variable-length kernels:
// LDS images of the operator tables, the 2-/4-byte sliced register update,
// nibble-table constant multiplies, the wave XOR reduction and the 4 KiB
// block load + permlane swizzle.  See crc32c_kernels.hip for the geometry.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace fdbcrc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// LDS image (byte offsets).  Lane l always reads bank column l%32.
// ---------------------------------------------------------------------------
// 4-byte slicing, 160 KiB = all of LDS:
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

// LDS fill: slice4 (1024 words) to all 32 columns, lane tables to their column.
// Every entry of the image is written (a kernel must never depend on what an
// earlier kernel left in LDS), for any block size.  Threads write consecutive
// 16-byte quads of the image (ds_write_b128, conflict-free): the transposed
// order -- one thread writing a table word's 32 replicas -- puts all lanes of
// a write on the same banks and cost ~15 us per launch.  The loads of a round
// are all issued before its writes.
// (s4: the four 256-entry word-step tables, ln: the 64 lanes' nibble tables --
// slice4 / lane for the contiguous 64-byte lane spans, stride4 / lane_s for
// the strided page layout)
__device__ inline void fill_lds_src(uint32_t* lds, const uint32_t* __restrict__ s4, const uint32_t* __restrict__ ln) {
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	auto gl = [](const uint32_t* p) -> uint32_t { return *((g_u32*)reinterpret_cast<uintptr_t>(p)); };
	constexpr uint32_t kSliceQ = 0x20000 / 16;  // quads of the two slicing regions
	constexpr uint32_t kLaneQ = 0x8000 / 16;    // quads of the lane tables
	constexpr uint32_t kPer = 8;
	u32x4* q4 = reinterpret_cast<u32x4*>(lds);
	// slicing regions: word W = region*16384 + (idx*2 + (k&1))*32 + col holds
	// slice4[2*region + (k&1)][idx]; a quad's four words share one value
	for (uint32_t Q0 = 0; Q0 < kSliceQ; Q0 += kPer * blockDim.x) {
		uint32_t v[kPer];
#pragma unroll
		for (uint32_t i = 0; i < kPer; ++i) {
			const uint32_t Q = Q0 + threadIdx.x + i * blockDim.x;
			const uint32_t W = 4 * (Q < kSliceQ ? Q : 0);
			const uint32_t pair = (W & 16383u) >> 5;
			v[i] = gl(s4 + (((W >> 14) * 2 + (pair & 1)) << 8) + (pair >> 1));
		}
#pragma unroll
		for (uint32_t i = 0; i < kPer; ++i) {
			const uint32_t Q = Q0 + threadIdx.x + i * blockDim.x;
			if (Q < kSliceQ) q4[(kS4Off / 16) + Q] = u32x4{v[i], v[i], v[i], v[i]};
		}
	}
	// lane tables: word V = half*4096 + nv*32 + (l & 31) holds lane[l][nv] (l = 32*half + (l & 31))
	for (uint32_t Q0 = 0; Q0 < kLaneQ; Q0 += 2 * blockDim.x) {
		u32x4 v[2];
#pragma unroll
		for (uint32_t i = 0; i < 2; ++i) {
			const uint32_t Q = Q0 + threadIdx.x + i * blockDim.x;
			const uint32_t V = 4 * (Q < kLaneQ ? Q : 0);
			const uint32_t nv = (V >> 5) & 127u, l = (V >> 12) * 32 + (V & 31u);
#pragma unroll
			for (uint32_t e = 0; e < 4; ++e) v[i][e] = gl(ln + (l + e) * 128 + nv);
		}
#pragma unroll
		for (uint32_t i = 0; i < 2; ++i) {
			const uint32_t Q = Q0 + threadIdx.x + i * blockDim.x;
			if (Q < kLaneQ) q4[(kS4LaneOff / 16) + Q] = v[i];
		}
	}
	__syncthreads();
}
__device__ inline void fill_lds_b(uint32_t* lds, const DevTables* __restrict__ t) {
	fill_lds_src(lds, &t->slice4[0][0], &t->lane[0][0][0]);
}

// The same fill split in two for 1024-thread workgroups, so a kernel can put
// the table loads in flight first and write them to LDS once its own start-up
// loads have returned: fill_issue_1024 loads each thread's share (8 slicing
// quads' values, 2 lane-table quads), fill_commit_1024 writes them and syncs.
struct FillRegs {
	uint32_t v[8];
	u32x4 lv[2];
};
__device__ __forceinline__ void fill_issue_1024(FillRegs& R, const DevTables* __restrict__ t) {
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	auto gl = [](const uint32_t* p) -> uint32_t { return *((g_u32*)reinterpret_cast<uintptr_t>(p)); };
	const uint32_t* s4 = &t->slice4[0][0];
	const uint32_t* ln = &t->lane[0][0][0];
#pragma unroll
	for (uint32_t i = 0; i < 8; ++i) {
		const uint32_t W = 4 * (threadIdx.x + i * 1024);
		const uint32_t pair = (W & 16383u) >> 5;
		R.v[i] = gl(s4 + (((W >> 14) * 2 + (pair & 1)) << 8) + (pair >> 1));
	}
#pragma unroll
	for (uint32_t i = 0; i < 2; ++i) {
		const uint32_t V = 4 * (threadIdx.x + i * 1024);
		const uint32_t nv = (V >> 5) & 127u, l = (V >> 12) * 32 + (V & 31u);
#pragma unroll
		for (uint32_t e = 0; e < 4; ++e) R.lv[i][e] = gl(ln + (l + e) * 128 + nv);
	}
}
__device__ __forceinline__ void fill_commit_1024(const FillRegs& R, uint32_t* lds) {
	u32x4* q4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
	for (uint32_t i = 0; i < 8; ++i) q4[(kS4Off / 16) + threadIdx.x + i * 1024] = u32x4{R.v[i], R.v[i], R.v[i], R.v[i]};
#pragma unroll
	for (uint32_t i = 0; i < 2; ++i) q4[(kS4LaneOff / 16) + threadIdx.x + i * 1024] = R.lv[i];
	__syncthreads();
}

struct LaneCtx {
	uint32_t ld_off;   // byte offset of this lane's first 16 B load inside a block
	int lane;
};

__device__ __forceinline__ LaneCtx make_ctx() {
	LaneCtx c;
	c.lane = threadIdx.x & 63;
	// lane m = 32h + 16q + r loads, for load k = 2kb + ka, the 16 bytes at
	//   2048*ka + 1024*kb + 64r + 32q + 16h
	// which after the swap network (unswizzle) puts block bytes
	// [64l, 64l+64) into lane l as registers r[0..3].
	const uint32_t h = c.lane >> 5, q = (c.lane >> 4) & 1, r = c.lane & 15;
	c.ld_off = 64 * r + 32 * q + 16 * h;
	return c;
}

// Four bytes per step, s' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]
// with x = s ^ word.  c4 = col*4 | 0x10000 (byte 2 selects region 1).
__device__ __forceinline__ uint32_t word_step4(const uint32_t* lds, uint32_t x, uint32_t c4) {
	const uint32_t a3 = __builtin_amdgcn_perm(x, c4, 0x0c0c0400u);  // (x.b0 << 8) | col*4
	const uint32_t a2 = __builtin_amdgcn_perm(x, c4, 0x0c0c0500u);  // (x.b1 << 8) | col*4
	const uint32_t a1 = __builtin_amdgcn_perm(x, c4, 0x0c020600u);  // 0x10000 | (x.b2 << 8) | col*4
	const uint32_t a0 = __builtin_amdgcn_perm(x, c4, 0x0c020700u);  // 0x10000 | (x.b3 << 8) | col*4
	return xor3(lds_rd(lds, a3), lds_rd(lds, a2 + 128), lds_rd(lds, a1)) ^ lds_rd(lds, a0 + 128);
}

// word_step4 with the next message word folded in: returns s' ^ next.
__device__ __forceinline__ uint32_t word_step4_next(const uint32_t* lds, uint32_t x, uint32_t next, uint32_t c4) {
	const uint32_t a3 = __builtin_amdgcn_perm(x, c4, 0x0c0c0400u);
	const uint32_t a2 = __builtin_amdgcn_perm(x, c4, 0x0c0c0500u);
	const uint32_t a1 = __builtin_amdgcn_perm(x, c4, 0x0c020600u);
	const uint32_t a0 = __builtin_amdgcn_perm(x, c4, 0x0c020700u);
	return xor3(xor3(lds_rd(lds, a3), lds_rd(lds + 32, a2), lds_rd(lds, a1)), lds_rd(lds + 32, a0), next);
}

// Multiply a register by the constant whose nibble tables start at `base`
// (base already carries the lane's column).
__device__ __forceinline__ uint32_t mul_nibbles(const uint32_t* lds, uint32_t s, uint32_t base) {
	uint32_t r[8];
#pragma unroll
	for (int n = 0; n < 8; ++n) {  // nibble n of s at bits 7..10, table n at bits 11..13 (zero in base)
		const uint32_t v = n == 0 ? (s << 7) : (4 * n >= 7 ? (s >> (4 * n - 7)) : (s << (7 - 4 * n)));
		// (v & 0x780) | (base | n << 11) as one v_bitop3 (truth table 0xEA = (S0 & S1) | S2): written
		// as a plain expression, LLVM turns the OR into an add against hoisted per-n constants
		r[n] = lds_rd(lds, __builtin_amdgcn_bitop3_b32(v, 0x780u, base | ((uint32_t)n << 11), 0xEA));
	}
	return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// Byte masks of a 16-byte chunk from 64-bit shifts: keep bytes >= k0 (lead),
// keep bytes < k1 (tail), and the register value s0 placed at byte k0
// (its bytes past the chunk end spill into the next chunk).
struct Masks {
	uint32_t lm[4], tm[4], inj[4], spill;
};
__device__ __forceinline__ Masks edge_masks(uint32_t k0, uint32_t k1, uint32_t s0) {
	const uint64_t ones = ~uint64_t(0), s = s0;
	const uint64_t lmLo = k0 >= 8 ? 0 : ones << (8 * k0);
	const uint64_t lmHi = k0 <= 8 ? ones : ones << (8 * (k0 - 8));
	const uint64_t tmLo = k1 >= 8 ? ones : ones >> (64 - 8 * k1);
	const uint64_t tmHi = k1 <= 8 ? 0 : ones >> (128 - 8 * k1);
	const uint64_t injLo = k0 >= 8 ? 0 : s << (8 * k0);
	const uint64_t injHi = k0 >= 8 ? s << (8 * (k0 - 8)) : (k0 > 4 ? s >> (8 * (8 - k0)) : 0);
	Masks m;
	m.lm[0] = (uint32_t)lmLo; m.lm[1] = (uint32_t)(lmLo >> 32); m.lm[2] = (uint32_t)lmHi; m.lm[3] = (uint32_t)(lmHi >> 32);
	m.tm[0] = (uint32_t)tmLo; m.tm[1] = (uint32_t)(tmLo >> 32); m.tm[2] = (uint32_t)tmHi; m.tm[3] = (uint32_t)(tmHi >> 32);
	m.inj[0] = (uint32_t)injLo; m.inj[1] = (uint32_t)(injLo >> 32); m.inj[2] = (uint32_t)injHi; m.inj[3] = (uint32_t)(injHi >> 32);
	m.spill = k0 > 12 ? s0 >> (8 * (16 - k0)) : 0u;
	return m;
}

// Cross-lane reads with unsigned results.  The builtins return `int`: widening
// that to 64 bits sign-extends, so every 64-bit value is rebuilt from
// explicitly unsigned halves.
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int k) {
	return (uint32_t)__builtin_amdgcn_readlane((int)v, k);
}
__device__ __forceinline__ uint32_t rdfirst(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int k) {
	return ((uint64_t)rdlane((uint32_t)(v >> 32), k) << 32) | (uint64_t)rdlane((uint32_t)v, k);
}
__device__ __forceinline__ uint64_t rdfirst64(uint64_t v) {
	return ((uint64_t)rdfirst((uint32_t)(v >> 32)) << 32) | (uint64_t)rdfirst((uint32_t)v);
}

// XOR of v over each 16-lane row; every lane of the row gets its row's value.
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false);  // row_ror:4
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
	return v;
}

// Inclusive prefix XOR of v over the wave (DPP row shifts, then the row
// broadcasts of lanes 15 and 31): lane l gets v[0] ^ ... ^ v[l].
__device__ __forceinline__ uint32_t wave_scanx(uint32_t v) {
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
	return v;
}

// XOR of v over all 64 lanes, returned wave-uniform.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false);  // row_ror:4
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
	return rdlane(v, 0) ^ rdlane(v, 16) ^ rdlane(v, 32) ^ rdlane(v, 48);
}

#ifdef FDBCRC_DEBUG
// Debug builds (make debug): every data load is bounds-checked against the
// window set by crc32c_debug_bounds(); violations are counted and skipped
// instead of faulting.  [0] lo, [1] hi, [2] violations, [3] first bad address
static __device__ unsigned long long g_dbg[8];
__device__ __forceinline__ bool dbg_ok(const void* p, uint64_t n, int site) {
	const uint64_t a = reinterpret_cast<uint64_t>(p);
	// aligned 16-byte chunks may extend past the data to the next 16-byte
	// boundary (same page, cannot fault): allow the 16-byte-rounded window
	if (g_dbg[1] == 0 || (a >= (g_dbg[0] & ~15ull) && a + n <= ((g_dbg[1] + 15) & ~15ull))) return true;
	if (atomicAdd(&g_dbg[2], 1ull) == 0) {
		g_dbg[3] = a;
		g_dbg[4] = (unsigned long long)site;
	}
	return false;
}
#define DBG_OK(p, n, site) dbg_ok((p), (n), (site))
#else
#define DBG_OK(p, n, site) true
#endif

// Every data load goes through the global address space (global_load_*,
// in-order vmcnt), never a FLAT load: addresses computed from integers would
// otherwise lose their address space.
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
	if (!DBG_OK(p, 16, 1)) return u32x4{0u, 0u, 0u, 0u};
	return __builtin_nontemporal_load((g_u32x4*)(reinterpret_cast<uintptr_t>(p)));
}

__device__ __forceinline__ uint32_t ld1(const uint8_t* p) {
	if (!DBG_OK(p, 1, 2)) return 0u;
	return *((g_u8*)(reinterpret_cast<uintptr_t>(p)));
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

}  // namespace fdbcrc
