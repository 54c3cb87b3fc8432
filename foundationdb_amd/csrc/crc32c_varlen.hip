// Variable-length / unaligned batched CRC-32C (gfx950).
//
// Serves every batch the 4 KiB page kernel does not: any alignment, any
// length, offsets in any order (overlaps allowed), per-buffer seeds, and
// fixed-stride batches of odd lengths.  Reference semantics: crc32c_append
// (contrib/crc32/crc32c.cpp:346-356) per buffer; the chained/streaming callers
// (fdbrpc/FileTransfer.cpp:29-37) reduce to the same thing through
// crc32c_combine.  The design (v7) is described where its kernels start below.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "crc32c_common.h"

namespace fdbcrc {

// ---------------------------------------------------------------------------
// tile scan (batches of more than kScanTiles tiles)
// ---------------------------------------------------------------------------
// quantum: ceil(total / nwave), at least qmin, rounded up to a multiple of qalign
__global__ __launch_bounds__(1024) void k_scan(uint64_t* __restrict__ prefix, uint64_t ntile,
                                               uint32_t* __restrict__ wave_tile, uint64_t nwave,
                                               uint64_t* __restrict__ hdr, uint64_t qmin = 4096,
                                               uint64_t qalign = 64, uint64_t* __restrict__ aux0 = nullptr,
                                               uint64_t* __restrict__ aux1 = nullptr) {
	constexpr uint32_t C = 8192;  // tiles per LDS chunk
	__shared__ uint64_t buf[C];
	__shared__ uint64_t wsum[16];
	__shared__ uint64_t carry_s;
	const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
	// pass 1: total
	uint64_t acc = 0;
	for (uint64_t k = t; k < ntile; k += blockDim.x) acc += prefix[k];
	for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
	if (lane == 0) wsum[w] = acc;
	__syncthreads();
	uint64_t total = 0;
	for (int k = 0; k < 16; ++k) total += wsum[k];
	uint64_t q = (total + nwave - 1) / nwave;
	q = q < qmin ? qmin : (q + qalign - 1) / qalign * qalign;
	__syncthreads();
	if (t == 0) carry_s = 0;
	__syncthreads();
	// pass 2: chunked exclusive scan + wave -> tile
	for (uint64_t c0 = 0; c0 < ntile; c0 += C) {
		const uint32_t n = (uint32_t)(ntile - c0 < C ? ntile - c0 : C);
		for (uint32_t k = t; k < n; k += blockDim.x) buf[k] = prefix[c0 + k];
		__syncthreads();
		// each thread scans a contiguous run of 8 entries
		const uint32_t r0 = t * (C / 1024);
		uint64_t run = 0;
		for (uint32_t k = 0; k < C / 1024; ++k) {
			const uint32_t idx = r0 + k;
			const uint64_t x = idx < n ? buf[idx] : 0;
			if (idx < n) buf[idx] = run;
			run += x;
		}
		// exclusive scan of the 1024 run totals
		uint64_t inc = run;
		for (int o = 1; o < 64; o <<= 1) {
			const uint64_t y = __shfl_up(inc, o);
			if ((int)lane >= o) inc += y;
		}
		if (lane == 63) wsum[w] = inc;
		__syncthreads();
		uint64_t wbase = 0;
		for (uint32_t k = 0; k < w; ++k) wbase += wsum[k];
		const uint64_t carry = carry_s;
		const uint64_t excl = carry + wbase + inc - run;
		for (uint32_t k = 0; k < C / 1024; ++k) {
			const uint32_t idx = r0 + k;
			if (idx < n) buf[idx] += excl;
		}
		__syncthreads();
		for (uint32_t k = t; k < n; k += blockDim.x) prefix[c0 + k] = buf[k];
		// waves whose first byte lies in this chunk's byte range
		const uint64_t lo_b = buf[0];
		uint64_t chunk_total = 0;
		for (int k = 0; k < 16; ++k) chunk_total += wsum[k];
		const uint64_t hi_b = carry + chunk_total;  // exclusive end of this chunk's bytes
		const bool last_chunk = c0 + n >= ntile;
		const uint64_t w_lo = c0 == 0 ? 0 : (lo_b + q - 1) / q;
		const uint64_t w_hi = last_chunk ? nwave : (hi_b + q - 1) / q;
		for (uint64_t wv = w_lo + t; wv < w_hi && wv < nwave; wv += blockDim.x) {
			const uint64_t lo = wv * q;
			// last index k in [0, n) with buf[k] <= lo
			uint32_t a = 0, b = n;
			while (b - a > 1) {
				const uint32_t mid = (a + b) >> 1;
				if (buf[mid] <= lo) a = mid; else b = mid;
			}
			wave_tile[wv] = (uint32_t)(c0 + a);
		}
		__syncthreads();
		if (t == 0) carry_s = hi_b;
		__syncthreads();
	}
	if (t == 0) {
		prefix[ntile] = total;
		hdr[0] = total;
		hdr[1] = q;
	}
	// the block route's tile sums (blocks, entries): plain exclusive scans
	for (int a = 0; a < 2; ++a) {
		uint64_t* arr = a == 0 ? aux0 : aux1;
		if (!arr) continue;
		__syncthreads();
		if (t == 0) carry_s = 0;
		for (uint64_t c0 = 0; c0 < ntile; c0 += C) {
			const uint32_t n = (uint32_t)(ntile - c0 < C ? ntile - c0 : C);
			__syncthreads();
			for (uint32_t k = t; k < n; k += blockDim.x) buf[k] = arr[c0 + k];
			__syncthreads();
			const uint32_t r0 = t * (C / 1024);
			uint64_t run = 0;
			for (uint32_t k = 0; k < C / 1024; ++k) {
				const uint32_t idx = r0 + k;
				const uint64_t x = idx < n ? buf[idx] : 0;
				if (idx < n) buf[idx] = run;
				run += x;
			}
			uint64_t inc = run;
			for (int o = 1; o < 64; o <<= 1) {
				const uint64_t y = __shfl_up(inc, o);
				if ((int)lane >= o) inc += y;
			}
			if (lane == 63) wsum[w] = inc;
			__syncthreads();
			uint64_t wbase = 0, ctot = 0;
			for (uint32_t k = 0; k < 16; ++k) {
				wbase += k < w ? wsum[k] : 0;
				ctot += wsum[k];
			}
			const uint64_t excl = carry_s + wbase + inc - run;
			for (uint32_t k = 0; k < C / 1024; ++k) {
				const uint32_t idx = r0 + k;
				if (idx < n) buf[idx] += excl;
			}
			__syncthreads();
			for (uint32_t k = t; k < n; k += blockDim.x) arr[c0 + k] = buf[k];
			__syncthreads();
			if (t == 0) carry_s += ctot;
		}
	}
}

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
// Uniform (wave-wide) multiply through nibble tables in global memory: the
// value is uniform, so these are scalar-cache loads, off the LDS path.
// The table is read through the constant address space with a uniform
// index, so these are s_load (lgkmcnt): as vector loads they would share the
// in-order vmcnt with the data prefetch and every multiply would wait for it.
__device__ __forceinline__ uint32_t umul(const uint32_t (*tab)[16], uint32_t v) {
	typedef __attribute__((address_space(4))) const uint32_t c_u32;
	const c_u32* t = (const c_u32*)reinterpret_cast<uintptr_t>(&tab[0][0]);
	v = rdfirst(v);
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= t[n * 16 + ((v >> (4 * n)) & 15u)];
	return rdfirst(r);
}

// Uniform value times x^(8d), d >= 0: one table multiply per set bit of d.
__device__ uint32_t mul_xpow(const DevTables* __restrict__ t, uint32_t v, uint64_t d) {
	for (int m = 0; d; ++m, d >>= 1)
		if (d & 1) v = umul(t->pow2[m], v);
	return v;
}

// Register chain over the lane's 64 contiguous bytes (layout B, 4-byte
// slicing), each step folding in the next word (word_step4_next).
__device__ __forceinline__ uint32_t chain64_b(const uint32_t* lds, uint32_t s, const Block& b, uint32_t c4) {
	s ^= b.r[0][0];
#pragma unroll
	for (int w = 0; w < 16; ++w) s = word_step4_next(lds, s, w < 15 ? b.r[(w + 1) >> 2][(w + 1) & 3] : 0u, c4);
	return s;
}
__device__ __forceinline__ uint32_t shup(uint32_t v, int d) { return (uint32_t)__shfl_up((int)v, d); }

// Inclusive prefix sum of a 32-bit value over the wave on DPP (row shifts,
// then the row broadcasts of lanes 15 and 31): six VALU adds, no LDS traffic.
__device__ __forceinline__ uint32_t scan_add(uint32_t v) {
	v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
	v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
	v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
	v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
	v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
	v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
	return v;
}

// Saturating 32-bit add (UINT32_MAX absorbs): the planner's slot and block
// counts are 32-bit; a batch whose totals reach 2^32 - 1 is refused (the
// last prep tile sees the saturated total, so overflow anywhere is caught).
__device__ __forceinline__ uint32_t sadd(uint32_t a, uint32_t b) {
	const uint32_t s = a + b;
	return s < a ? 0xFFFFFFFFu : s;
}
__device__ __forceinline__ uint32_t sat32(uint64_t v) { return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v; }
// scan_add with saturation at every step.
__device__ __forceinline__ uint32_t scan_sadd(uint32_t v) {
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false));
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false));
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false));
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false));
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false));
	v = sadd(v, __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false));
	return v;
}

// Inclusive prefix sum of a 64-bit value over the wave.
__device__ __forceinline__ uint64_t scan64(uint64_t v, int lane) {
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint64_t y = ((uint64_t)shup((uint32_t)(v >> 32), d) << 32) | shup((uint32_t)v, d);
		if (lane >= d) v += y;
	}
	return v;
}

__device__ __forceinline__ uint32_t gld32(const uint32_t* p) {
	typedef __attribute__((address_space(1))) const uint32_t g_u32;
	return *((g_u32*)reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ uint64_t gld64(const uint64_t* p) {
	typedef __attribute__((address_space(1))) const uint64_t g_u64;
	return *((g_u64*)reinterpret_cast<uintptr_t>(p));
}

// Lane-parallel multiply by the per-lane constant whose nibble tables start
// at `tab` (global memory, 8 x 16 words).
__device__ __forceinline__ uint32_t vmul(const uint32_t* tab, uint32_t v) {
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= gld32(tab + n * 16 + ((v >> (4 * n)) & 15u));
	return r;
}

// ---------------------------------------------------------------------------
// v7: window slots, prepared per buffer, streamed per wave
// ---------------------------------------------------------------------------
// Every buffer of >= 16 bytes is cut into W = ceil((E - A) / 1024) windows of
// 1 KiB ALIGNED TO ITS END E = ceil16(P1) (A = P0 & ~15): window m covers
// [E - 1024(W-m), E - 1024(W-m-1)); window 0 starts lo = 1024W - (E - A)
// bytes before A, and those leading bytes are not loaded (leading zeros are
// free).  The windows of all buffers, in index order, are the batch's SLOTS
// (global slot g_i + m for window m of buffer i).  Shorter buffers are
// finished byte-serially by the prep kernel.
//
//  k_v7prep   per tile of 256 buffers: W and the tile's slot prefix (single-pass
//             decoupled look-back over the tiles), then per buffer g_i, the lead
//             and tail EDGE TERMS (below), short buffers finished; zeroes out[]
//             of windowed buffers; the last tile writes the total and the
//             per-wave quantum (whole passes)
//  k_varlen7  wave w checksums slots [w*Qs, (w+1)*Qs): slot k of a pass is
//             window k%4 of 4 (one 16-lane team each, page-kernel layout), so a
//             pass always carries four windows whatever the buffer sizes.
//
// Edge terms (CRC linearity: the chain of a XOR b is chain(a) ^ chain(b)):
// the pass checksums the garbage bytes [A, P0) before the buffer and
// [P1, E) after it, and no seed.  The lead term is the register of the lead
// lane's 64-byte span fed with only those garbage bytes, with the register
// ~seed injected at P0 (crc32c.cpp:197) -- XORed in, it cancels the garbage
// and adds the seed; the tail term cancels the trailing garbage.  Both are
// stored as TEAM-SUM terms (already multiplied by their lane's constant), so
// the streaming kernel only XORs them into the slot sums.
//
// Combining, per table of 64 slots (16 passes) of a wave, lane-parallel: the
// 64-lane constant tables give slot sum S_k = Rw_k * x^(8*1024*(3 - k%4));
// weighted by x^(8*4096*(15 - k/4)) it becomes Rw_k * x^(8*1024*(63-k)); a
// prefix XOR over the lanes then yields every buffer's total at its last slot
// kl, normalised by x^(-8*(1024*(63-kl) + zt)) (zt = E - P1 trailing zeros).
// A buffer open at a table's end carries into the next table as one uniform
// register times x^(8*65536); a buffer cut by the wave range is finished as a
// part shifted to its end and XOR-merged (atomicXor) with its other parts.
constexpr uint32_t kTileW = 256;
#ifndef FDBCRC_V7_THREADS
#define FDBCRC_V7_THREADS 768  // 12 waves per CU: 155 VGPRs per lane, no VGPR spills
#endif
// One static slot range per wave (dynamic ranges grabbed from per-workgroup
// counters were measured slower: each range restart -- tile search, first
// table build, pipeline refill -- costs more than the balance gains).
constexpr uint64_t kV7RangesPerBlock = FDBCRC_V7_THREADS / 64;
#ifndef FDBCRC_SELFSUM_TILES
#define FDBCRC_SELFSUM_TILES 32
#endif
constexpr uint64_t kSelfSumTiles = FDBCRC_SELFSUM_TILES;
#ifndef FDBCRC_SCAN_TILES
#define FDBCRC_SCAN_TILES 8192
#endif
constexpr uint64_t kScanTiles = FDBCRC_SCAN_TILES;
#ifndef FDBCRC_SMALL_SPAN
#define FDBCRC_SMALL_SPAN 128
#endif
// Buffers whose 16-byte chunks span at most kSmallSpan bytes get no window
// slots: the prep kernel finishes them, one lane each (a 1 KiB window would
// mostly checksum lanes of zeros for them).
constexpr uint32_t kSmallSpan = FDBCRC_SMALL_SPAN;
__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) {
	return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
	return ((uint64_t)shfl32((uint32_t)(v >> 32), src) << 32) | shfl32((uint32_t)v, src);
}
// Inclusive prefix XOR over the wave.
// (DPP row shifts and row broadcasts, like scan_add: no LDS round trips)
__device__ __forceinline__ uint32_t scanx(uint32_t v, int lane) {
	(void)lane;
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
	v ^= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
	return v;
}
// Byte mask of a 16-byte chunk keeping bytes < k1 (1..15).
__device__ __forceinline__ void keep_below7(uint32_t k1, uint32_t (&tm)[4]) {
	const uint64_t ones = ~uint64_t(0);
	const uint64_t lo = k1 >= 8 ? ones : ones >> (64 - 8 * k1);
	const uint64_t hi = k1 <= 8 ? 0 : ones >> (128 - 8 * k1);
	tm[0] = (uint32_t)lo; tm[1] = (uint32_t)(lo >> 32); tm[2] = (uint32_t)hi; tm[3] = (uint32_t)(hi >> 32);
}
struct Geo7 {
	uint64_t A;    // P0 & ~15
	uint32_t W;    // windows (0: shorter than 16 bytes, small, or routed to blocks)
	uint32_t lo;   // bytes of window 0 before A (multiple of 16, < 1024)
	uint32_t k0;   // P0 % 16
	uint32_t zt;   // E - P1
	uint32_t nb;   // 4 KiB blocks of the big-buffer route (0: not routed)
};
// bigmin: spans of at least this many bytes (below kBigMax) go to the block
// route (crc32c_kernels.hip, k_bigblocks); 0 disables it.
__device__ __forceinline__ Geo7 geo7(uint64_t P0, uint64_t len, uint64_t bigmin = 0) {
	Geo7 g;
	const uint64_t P1 = P0 + len;
	const uint64_t E = (P1 + 15) & ~uint64_t(15);
	g.A = P0 & ~uint64_t(15);
	const uint64_t span = E - g.A;
	const bool big = bigmin && len >= 16 && span >= bigmin && span < kBigMax;
	g.nb = big ? (uint32_t)((span + 4095) >> 12) : 0u;
	// (saturated: a span of 4 TiB or more alone overflows the slot count)
	g.W = (!big && len >= 16 && span > kSmallSpan) ? sat32((span >> 10) + ((span & 1023) != 0)) : 0u;
	g.lo = (uint32_t)(1024 * (uint64_t)g.W - span) & 1023u;
	g.k0 = (uint32_t)(P0 & 15);
	g.zt = (uint32_t)(E - P1);
	return g;
}
#ifndef FDBCRC_SELFSUM_UB
#define FDBCRC_SELFSUM_UB 2
#endif
#ifndef FDBCRC_SELFSUM_UW
#define FDBCRC_SELFSUM_UW 4
#endif
struct V7Params {
	const uint8_t* base;
	const uint64_t* offsets;   // nullptr: fixed stride
	const uint64_t* lengths;   // nullptr: fixed length
	uint64_t stride, length, count;
	uint32_t seed;
	const uint32_t* seeds;
	uint32_t* out;
	uint64_t* hdr;             // [0] total slots, [1] slots per wave
	uint64_t* tsum;            // per tile: windows of its buffers (exclusive prefix after k_scan)
	uint64_t* incl;            // per tile: inclusive slot prefix
	uint64_t ntile, nwave;
	bool scanned;              // tsum already holds exclusive prefixes (large batches: k_scan ran)
	bool selfsum;              // small batches: no count kernel, each prep block counts its predecessors' windows
	uint32_t* gs;              // first slot of each buffer
	uint32_t* cl;              // lead edge term (team-sum form)
	uint32_t* dummy;           // 64 words per wave: target of the no-op XORs
	const DevTables* tabs;
	uint32_t qalign;           // slots per wave rounded to a multiple of this (power of two)
	// big-buffer block route (bigmin = 0: off; hdr[2] blocks and hdr[3] entries in total)
	uint64_t bigmin;
	uint64_t* bsum;            // per tile: blocks of its routed buffers (like tsum)
	uint64_t* nsum;            // per tile: routed buffers
	BigEnt* ent;               // per entry (routed buffer): end, first block, index, lo | k0 | t, ~seed
	uint32_t* bctr;            // block kernel grab counters (zeroed here)
	uint32_t nbctr;            // ... words
	uint64_t* hstat;           // route statistics of tile 0 (host-mapped, may be null): RouteStat
	uint32_t* err;             // sticky refusal flag of the stream (host-mapped, may be null)
	// extent route (kRouteExtent, crc32c_extent.hip): the count kernel checks
	// the packing (the extent kernels follow it; prep and the window kernel
	// are not launched)
	uint32_t* xhdr;            // [0] / [1]: epoch of the last launch found not packed / over kXMaxExtent
	uint32_t epoch;
	uint32_t* xwq;             // per grab of k_xgrab: the first buffer ending past its start (may be null)
	uint64_t xcapg;            // ... grabs it holds
};
// hdr[6]: 1 if the planner refused the batch (2^32 - 1 or more windows or
// blocks: 32-bit slot indices); the streaming kernels then do nothing.
constexpr int kHdrRefused = 6;
__device__ __forceinline__ void v7_buffer(const V7Params& P, uint64_t i, uint64_t& off, uint64_t& len) {
	off = P.offsets ? P.offsets[i] : i * P.stride;
	len = P.lengths ? P.lengths[i] : P.length;
}
// Buffers i and i + 1 are PACKED (the extent route's condition): in order,
// no overlap, and a gap below 4096 bytes and at most max(len_i, 256) (the gap
// is read: bounded waste, and every gap byte lies in a page that holds buffer
// bytes).  tests/extent_model.py: eligible().
__device__ __forceinline__ bool v7_packed_pair(const V7Params& P, uint64_t i, uint64_t off, uint64_t len) {
	if (i + 1 >= P.count) return true;
	uint64_t on, ln;
	v7_buffer(P, i + 1, on, ln);
	(void)ln;
	const uint64_t e = off + len;
	const uint64_t gap = on - e;
	return on >= e && gap < 4096 && gap <= (len > 256 ? len : 256);
}
// The first 256 buffers' bytes by span class and whether they are packed,
// for the stream's next route choice (tile 0 of prep, or of the count kernel
// on the extent route).  All threads of the block call it.
// st: where the statistics go (hstat's layout: the stream's host-mapped words,
// or the extent route's device staging, kXStage); backoff: count the extent
// route's back-off down (host-mapped words only: on the extent route k_xfin
// sets that word from the batch's own check).
__device__ void v7_route_stats(const V7Params& P, uint64_t i, uint64_t off, uint64_t len, uint64_t (*s_stat)[4],
                               uint64_t* st, bool backoff) {
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const bool ok = i < P.count;
	const uint64_t P0 = reinterpret_cast<uint64_t>(P.base) + off;
	const uint64_t span = ok && len >= 16 ? ((P0 + len + 15) & ~uint64_t(15)) - (P0 & ~uint64_t(15)) : 0;
	uint64_t c[4] = {span > kSmallSpan && span < 4096 ? len : 0, span >= 4096 && span < 16384 ? len : 0,
	                 span >= 16384 ? len : 0, (ok && !v7_packed_pair(P, i, off, len)) ? 1u : 0u};
#pragma unroll
	for (int k = 0; k < 4; ++k)
		for (int o = 32; o > 0; o >>= 1) c[k] += __shfl_xor(c[k], o);
	if (lane == 0)
#pragma unroll
		for (int k = 0; k < 4; ++k) s_stat[wv][k] = c[k];
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int k = 0; k < 3; ++k) st[k] = s_stat[0][k] + s_stat[1][k] + s_stat[2][k] + s_stat[3][k];
		st[kHstatPacked] = (s_stat[0][3] | s_stat[1][3] | s_stat[2][3] | s_stat[3][3]) ? 0 : 1;
		// a window/block-route batch counts the extent route's back-off down
		if (backoff && P.hstat[kHstatXfail] > 0 && P.hstat[kHstatXfail] <= kXfailBackoff) --P.hstat[kHstatXfail];
	}
}
__global__ __launch_bounds__(256) void k_v7count(V7Params P) {
	__shared__ uint32_t part[3][4];
	__shared__ uint64_t s_stat[4][4];
	const uint64_t i = (uint64_t)blockIdx.x * kTileW + threadIdx.x;
	uint32_t W = 0, B = 0, N = 0;
	uint64_t off = 0, len = 0;
	if (i < P.count) {
		v7_buffer(P, i, off, len);
		const Geo7 g = geo7(reinterpret_cast<uint64_t>(P.base) + off, len, P.bigmin);
		W = g.W;
		B = g.nb;
		N = g.nb ? 1u : 0u;
	}
	if (P.xhdr) {  // extent route: the packing check, epoch-tagged (no flag is ever reset)
		const bool bad = i < P.count && !v7_packed_pair(P, i, off, len);
		if (__ballot(bad) && (threadIdx.x & 63) == 0) P.xhdr[0] = P.epoch;
		if (blockIdx.x == 0 && threadIdx.x == 0) {
			uint64_t o0, l0, o1, l1;
			v7_buffer(P, 0, o0, l0);
			v7_buffer(P, P.count - 1, o1, l1);
			const uint64_t S = (reinterpret_cast<uint64_t>(P.base) + o0) & ~uint64_t(15);
			const uint64_t E = (reinterpret_cast<uint64_t>(P.base) + o1 + l1 + 15) & ~uint64_t(15);
			// (an unordered batch may give E < S: the packing check refuses it anyway)
			const uint64_t nblk = E > S ? (E - S + 4095) >> 12 : 0;
			if (E - S >= kXMaxExtent) P.xhdr[1] = P.epoch;
			if (P.hstat) reinterpret_cast<uint64_t*>(P.xhdr)[kXStage + kHstatNblk] = nblk;
		}
		if (blockIdx.x == 0 && P.hstat)
			v7_route_stats(P, i, off, len, s_stat, reinterpret_cast<uint64_t*>(P.xhdr) + kXStage, false);
		// k_xgrab's grab map: buffer i is the first to end past the start T(g)
		// of grabs g with end(i-1) <= T(g) < end(i); the last buffer also
		// covers the grabs after its end.  Only ordered pairs write (a batch
		// that is not packed is never streamed), at most the grabs that exist.
		if (P.xwq && i < P.count) {
			uint64_t o0, l0, o1, l1;
			v7_buffer(P, 0, o0, l0);
			v7_buffer(P, P.count - 1, o1, l1);
			const uint64_t S = (reinterpret_cast<uint64_t>(P.base) + o0) & ~uint64_t(15);
			const uint64_t E = (reinterpret_cast<uint64_t>(P.base) + o1 + l1 + 15) & ~uint64_t(15);
			const uint64_t nblk = E > S ? (E - S + 4095) >> 12 : 0;
			const uint64_t gsz = x_gsz(nblk, P.xcapg), ngrab = (nblk + gsz - 1) / gsz;
			const uint32_t lt = 12 + x_log2(gsz);  // bytes per grab: 2^lt
			const uint64_t Pe = reinterpret_cast<uint64_t>(P.base) + off + len;
			uint64_t pe = 0;
			if (i) {
				uint64_t op, lp;
				v7_buffer(P, i - 1, op, lp);
				pe = reinterpret_cast<uint64_t>(P.base) + op + lp;
			}
			if (nblk && E - S < kXMaxExtent && Pe >= S && (i == 0 || (pe >= S && pe <= Pe))) {
				const uint64_t ep = i ? pe - S : 0, ei = Pe - S;
				const uint64_t glo = (ep + (1ull << lt) - 1) >> lt;
				uint64_t ghi = (ei + (1ull << lt) - 1) >> lt;
				if (i + 1 == P.count) ghi = ngrab;
				for (uint64_t g = glo; g < ghi && g < ngrab; ++g) P.xwq[g] = (uint32_t)i;
			}
		}
	}
	W = scan_sadd(W);
	B = scan_sadd(B);
	N = scan_add(N);
	if ((threadIdx.x & 63) == 63) {
		part[0][threadIdx.x >> 6] = W;
		part[1][threadIdx.x >> 6] = B;
		part[2][threadIdx.x >> 6] = N;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		P.tsum[blockIdx.x] = (uint64_t)part[0][0] + part[0][1] + part[0][2] + part[0][3];
		if (P.bigmin) {
			P.bsum[blockIdx.x] = (uint64_t)part[1][0] + part[1][1] + part[1][2] + part[1][3];
			P.nsum[blockIdx.x] = (uint64_t)part[2][0] + part[2][1] + part[2][2] + part[2][3];
		}
	}
}

// wq[g] = v for g in [lo, hi): a lane writes a short range itself; a range of
// more than 64 grabs (a buffer spanning them, e.g. one of a few huge buffers)
// is written by the whole wave, 64 entries per store -- one lane writing a
// 1.1 GB buffer's 34 k entries took 581 us.  Every lane of the wave calls it
// (on = false: no range of its own).
__device__ __forceinline__ void fill_grab_map(uint32_t* wq, uint64_t lo, uint64_t hi, uint32_t v, bool on) {
	const bool lng = on && hi > lo + 64;
	if (on && !lng)
		for (uint64_t g = lo; g < hi; ++g) wq[g] = v;
	uint64_t m = __ballot(lng);
	const uint32_t lane = threadIdx.x & 63;
	while (m) {
		const int j = __builtin_ctzll(m);
		m &= m - 1;
		const uint64_t a = __shfl(lo, j), b = __shfl(hi, j);
		const uint32_t x = (uint32_t)__shfl((int)v, j);
		for (uint64_t g = a + lane; g < b; g += 64) wq[g] = x;
	}
}

// The extent route's only planning pass (crc32c_extent.hip): the packing and
// extent checks (epoch-tagged flags), the stream's route statistics (tile 0)
// and k_xgrab's grab map, from one coalesced load of each buffer's offset and
// length (the next buffer's come from the neighbouring lane).  Buffer i + 1 is
// the first to end past the start T(g) of the grabs with end(i) <= T(g) <
// end(i + 1); buffer 0 covers the grabs before its end, the last buffer's
// index + 1 (= count) the grabs after it.
__global__ __launch_bounds__(256) void k_xcount(V7Params P) {
	__shared__ uint64_t s_stat[4][4];
	const uint64_t i = (uint64_t)blockIdx.x * kTileW + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63;
	const bool in = i < P.count;
	uint64_t off = 0, len = 0, on = 0, ln = 0;
	const bool has_next = i + 1 < P.count;
	// the next buffer's metadata loaded directly (beside this one's, one round
	// trip) rather than shuffled down, which left lane 63's own load behind it
	if (in) v7_buffer(P, i, off, len);
	if (has_next) v7_buffer(P, i + 1, on, ln);
	const uint64_t e = off + len;
	const bool bad = in && has_next && !(on >= e && on - e < 4096 && on - e <= (len > 256 ? len : 256));
	if (__ballot(bad) && lane == 0) P.xhdr[0] = P.epoch;
	uint64_t o0, l0, o1, l1;
	v7_buffer(P, 0, o0, l0);
	v7_buffer(P, P.count - 1, o1, l1);
	const uint64_t S = (reinterpret_cast<uint64_t>(P.base) + o0) & ~uint64_t(15);
	const uint64_t E = (reinterpret_cast<uint64_t>(P.base) + o1 + l1 + 15) & ~uint64_t(15);
	// (an unordered batch may give E < S: the packing check refuses it anyway)
	const uint64_t nblk = E > S ? (E - S + 4095) >> 12 : 0;
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		if (E - S >= kXMaxExtent) P.xhdr[1] = P.epoch;
		if (P.hstat) reinterpret_cast<uint64_t*>(P.xhdr)[kXStage + kHstatNblk] = nblk;
	}
	if (blockIdx.x == 0 && P.hstat)
		v7_route_stats(P, i, off, len, s_stat, reinterpret_cast<uint64_t*>(P.xhdr) + kXStage, false);
	// (every lane reaches both calls: a wave fills long ranges together)
	const bool act = P.xwq && in && nblk && E - S < kXMaxExtent && !bad;
	uint64_t lo0 = 0, hi0 = 0, glo = 0, ghi = 0;
	uint32_t v = 0;
	if (act) {
		const uint64_t gsz = x_gsz(nblk, P.xcapg), ngrab = (nblk + gsz - 1) / gsz;
		const uint32_t lt = 12 + x_log2(gsz);  // bytes per grab: 2^lt
		const uint64_t base = reinterpret_cast<uint64_t>(P.base);
		const uint64_t ei = base + e - S;  // (>= 0 for an ordered pair)
		auto ceil_g = [&](uint64_t p) { return (p + (1ull << lt) - 1) >> lt; };
		if (i == 0) hi0 = min(ceil_g(ei), ngrab);
		glo = ceil_g(ei);
		ghi = min(has_next ? ceil_g(base + on + ln - S) : ngrab, ngrab);
		v = has_next ? (uint32_t)(i + 1) : (uint32_t)P.count;
	}
	fill_grab_map(P.xwq, lo0, hi0, 0u, act && i == 0);
	fill_grab_map(P.xwq, glo, ghi, v, act);
}

#ifdef FDBCRC_PTIMES
// development: per-tile timestamps of the prep kernels (s_memrealtime, 100 MHz):
// start, tables and chunks in, prefixes known, entries out
__device__ uint64_t g_pt[4096][4];
#define FDBCRC_PT(k) \
	if (threadIdx.x == 0 && blockIdx.x < 4096) g_pt[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
#else
#define FDBCRC_PT(k)
#endif

// BIG: the block route is on (bigmin != 0); without it the route's sums
// and entries are compiled out (fewer registers: 8 blocks per CU).
template <bool BIG>
__device__ __forceinline__ void v7prep(const V7Params& P) {
	FDBCRC_PT(0)
	const uint64_t bigmin = BIG ? P.bigmin : 0;
	__shared__ uint32_t s4[4][256];    // slice4 tables (no bank replication: this kernel is not LDS-bound)
	__shared__ uint32_t iz[16 * 128];  // inv_z nibble tables: x^(-8z), z < 16 (small buffers' trailing zeros)
	__shared__ uint32_t wsum[3][4];
	__shared__ uint32_t s_pre[3][4];
	__shared__ uint64_t s_stat[4][4];
	const DevTables* T = P.tabs;
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	// Latency chain: the table loads, this thread's metadata and the first
	// round of predecessor tile sums go out together; the small buffers' chunk
	// loads follow as soon as the metadata is back, in the shadow of the tile
	// sums, and the one barrier of the kernel waits for all of them.
	uint32_t tv[12];
#pragma unroll
	for (int k = 0; k < 4; ++k) tv[k] = gld32(&T->slice4[k][threadIdx.x]);
#pragma unroll
	for (int k = 0; k < 8; ++k) tv[4 + k] = gld32(&T->inv_z[0][0][0] + threadIdx.x + 256 * k);
	const uint32_t tile = blockIdx.x;
	const uint64_t i = (uint64_t)tile * kTileW + threadIdx.x;
	const bool ok = i < P.count;
	uint64_t off = 0, len = 0;
	v7_buffer(P, ok ? i : P.count - 1, off, len);
	const uint32_t sdv = P.seeds ? P.seeds[ok ? i : P.count - 1] : P.seed;
	if (!ok) len = 0;
	// general path (neither scanned nor self-summed): eight tile sums per thread
	// in flight at once (one load latency per 2048 predecessor tiles)
	const bool tl = !P.scanned && !P.selfsum;
	uint32_t v[8], vB[8], vN[8];
	auto tile_loads = [&](uint32_t k0) {
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u) {
			const uint32_t k = k0 + u * blockDim.x;
			const uint32_t kc = k < tile ? k : 0;
			v[u] = sat32(gld64(P.tsum + kc));
			vB[u] = bigmin ? sat32(gld64(P.bsum + kc)) : 0u;
			vN[u] = bigmin ? (uint32_t)gld64(P.nsum + kc) : 0u;
		}
	};
	if (tl) tile_loads(threadIdx.x);
#pragma unroll
	for (int k = 0; k < 4; ++k) s4[k][threadIdx.x] = tv[k];
#pragma unroll
	for (int k = 0; k < 8; ++k) iz[threadIdx.x + 256 * k] = tv[4 + k];
	if (tile == 0)
		for (uint32_t k = threadIdx.x; k < P.nbctr; k += 256) P.bctr[k] = 0;
	const uint64_t P0 = reinterpret_cast<uint64_t>(P.base) + off;
	const Geo7 g = geo7(P0, len, bigmin);
	// small buffer (16-byte chunks spanning at most kSmallSpan bytes): its
	// chunks, loaded now (exec-masked: chunks past the buffer's last are not
	// read; 1 Mi x 64 B packets 0.057 -> 0.048 ms against clamped re-reads)
	// A windowed buffer ending inside its last chunk (zt != 0) takes the same
	// path with that one chunk, its own bytes masked: the result is its tail
	// term (below, where out[] is initialised).
	constexpr uint32_t NC = kSmallSpan / 16;
	const bool small = ok && len >= 16 && !g.W && !g.nb;
	// (not for a span of 4 TiB or more: W saturates, the batch is refused, and
	// its end is not memory anyone holds)
	const bool tailw = ok && g.W && g.W != 0xFFFFFFFFu && g.zt;
	const uint64_t E16 = (P0 + len + 15) & ~uint64_t(15);
	const uint32_t nch = small ? (uint32_t)(E16 - g.A) >> 4 : (tailw ? 1u : 0u);
	const uint64_t cb = small ? g.A : E16 - 16;
	u32x4 ch[NC];
#pragma unroll
	for (uint32_t j = 0; j < NC; ++j)
		ch[j] = j < nch ? ld16(reinterpret_cast<const uint8_t*>(cb + 16 * j)) : u32x4{0u, 0u, 0u, 0u};
	// The tables are in LDS once every thread's writes are: the barrier (its
	// fence waits for every load in flight) also collects the chunks and the
	// first round of tile sums, which were all in flight together.
	__syncthreads();
	FDBCRC_PT(1)
	// small buffer: its chunks [A, E) as 4-byte words from a zero register,
	// the bytes before P0 zeroed and ~seed injected at P0 (crc32c.cpp:197),
	// the zt bytes after P1 zeroed and then divided out (x^(-8 zt), LDS
	// nibble tables).  Finished here, so the chunks are dead before the scans.
	uint32_t pre = 0, preB = 0, preN = 0;
	if (tl) {  // the first round of tile sums (the rest, for batches past 2048 tiles, below)
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u) {
			const bool in = threadIdx.x + u * blockDim.x < tile;
			pre = sadd(pre, in ? v[u] : 0u);
			preB = sadd(preB, in ? vB[u] : 0u);
			preN += in ? vN[u] : 0u;
		}
	}
	uint32_t xs = 0;
	if (nch) {
		// small: bytes from k0 on, ~seed at k0, bytes up to 16 - zt in the last
		// chunk; tail term: only the zt bytes after the end, no seed
		const Masks mk = small ? edge_masks(g.k0, 16u - g.zt, ~sdv) : edge_masks(16u - g.zt, 16u, 0u);
#pragma unroll
		for (uint32_t j = 0; j < NC; ++j) {
			if (j < nch) {
#pragma unroll
				for (int d = 0; d < 4; ++d) {
					uint32_t w = ch[j][d];
					if (j == 0) w = (w & mk.lm[d]) ^ mk.inj[d];
					if (j == 1 && d == 0) w ^= mk.spill;
					if (j == nch - 1) w &= mk.tm[d];
					xs ^= w;
					xs = s4[0][xs & 255u] ^ s4[1][(xs >> 8) & 255u] ^ s4[2][(xs >> 16) & 255u] ^ s4[3][xs >> 24];
				}
			}
		}
		if (g.zt) {
			const uint32_t* t = iz + 128 * g.zt;
			uint32_t r = 0;
#pragma unroll
			for (int n = 0; n < 8; ++n) r ^= t[16 * n + ((xs >> (4 * n)) & 15u)];
			xs = r;
		}
	}
	// exclusive prefixes of this tile (window slots, route blocks, route
	// entries): the sums of all earlier tiles, read in parallel by the whole
	// block (no inter-block waiting).  The engine's slot and block indices are
	// 32-bit, so the sums are 32-bit and saturating: a batch whose total
	// reaches 2^32 - 1 is refused by the last tile.
	if (P.scanned) {
		if (threadIdx.x == 0) {
			pre = sat32(P.tsum[tile]);
			if (bigmin) {
				preB = sat32(P.bsum[tile]);
				preN = (uint32_t)P.nsum[tile];
			}
		}
	} else if (P.selfsum) {
		// the predecessors' geometry recomputed here, eight buffers per thread
		// in flight at once
		const uint64_t n = (uint64_t)tile * kTileW;
		// (SU buffers in flight per thread: 8 spilled 36 SGPRs with the block
		// route's geometry, 2 spill none there; the windows-only form takes 4)
		constexpr uint32_t SU = BIG ? FDBCRC_SELFSUM_UB : FDBCRC_SELFSUM_UW;
		// (The loads sit behind v7_buffer's stride/list branch, so each pair is
		// waited for where the paths join; unconditional loads, 3-8 in flight,
		// measured the same on the chunks batch -- its prep is ~7 us of
		// dispatch and barriers, `tools/probe_ptimes.py` -- and spilled SGPRs.)
		for (uint64_t j0 = threadIdx.x; j0 < n; j0 += SU * blockDim.x) {
			uint64_t o[SU], l[SU];
#pragma unroll
			for (uint32_t u = 0; u < SU; ++u) {
				const uint64_t j = j0 + u * blockDim.x;
				v7_buffer(P, j < n ? j : 0, o[u], l[u]);
			}
#pragma unroll
			for (uint32_t u = 0; u < SU; ++u) {
				const Geo7 gj = geo7(reinterpret_cast<uint64_t>(P.base) + o[u], l[u], bigmin);
				const bool in = j0 + u * blockDim.x < n;
				pre = sadd(pre, in ? gj.W : 0u);
				preB = sadd(preB, in ? gj.nb : 0u);
				preN += in && gj.nb ? 1u : 0u;
			}
		}
	} else {
		for (uint32_t k0 = threadIdx.x + 8 * blockDim.x; k0 < tile; k0 += 8 * blockDim.x) {
			tile_loads(k0);
#pragma unroll
			for (uint32_t u = 0; u < 8; ++u) {
				const bool in = k0 + u * blockDim.x < tile;
				pre = sadd(pre, in ? v[u] : 0u);
				preB = sadd(preB, in ? vB[u] : 0u);
				preN += in ? vN[u] : 0u;
			}
		}
	}
	pre = rdlane(scan_sadd(pre), 63);
	preB = rdlane(scan_sadd(preB), 63);
	preN = rdlane(scan_add(preN), 63);
	if (lane == 0) {
		s_pre[0][wv] = pre;
		s_pre[1][wv] = preB;
		s_pre[2][wv] = preN;
	}
	const uint32_t W = ok ? g.W : 0u, B = ok ? g.nb : 0u, N = (ok && g.nb) ? 1u : 0u;
	if (tile == 0 && P.hstat && !P.xhdr) v7_route_stats(P, i, off, len, s_stat, P.hstat, true);
	const uint32_t incl = scan_sadd(W), inclB = scan_sadd(B), inclN = scan_add(N);
	if (lane == 63) {
		wsum[0][wv] = incl;
		wsum[1][wv] = inclB;
		wsum[2][wv] = inclN;
	}
	__syncthreads();
	uint32_t inwave = 0, agg = 0, inB = 0, aggB = 0, inN = 0, aggN = 0;
	for (int k = 0; k < 4; ++k) {
		inwave = sadd(inwave, k < wv ? wsum[0][k] : 0u);
		agg = sadd(agg, wsum[0][k]);
		inB = sadd(inB, k < wv ? wsum[1][k] : 0u);
		aggB = sadd(aggB, wsum[1][k]);
		inN += k < wv ? wsum[2][k] : 0u;
		aggN += wsum[2][k];
	}
	FDBCRC_PT(2)
	const uint32_t excl = sadd(sadd(s_pre[0][0], s_pre[0][1]), sadd(s_pre[0][2], s_pre[0][3]));
	const uint32_t exclB = sadd(sadd(s_pre[1][0], s_pre[1][1]), sadd(s_pre[1][2], s_pre[1][3]));
	const uint32_t exclN = s_pre[2][0] + s_pre[2][1] + s_pre[2][2] + s_pre[2][3];
	if (threadIdx.x == 0) {
		P.incl[tile] = (uint64_t)excl + agg;
		if (tile + 1 == P.ntile) {
			const uint32_t total = sadd(excl, agg), blocks = sadd(exclB, aggB);
			// 32-bit slot / block indices: 2^32 - 1 or more of either refuses the
			// batch (the saturated totals stick at the limit)
			const bool refused = total == 0xFFFFFFFFu || blocks == 0xFFFFFFFFu;
			uint64_t q = ((uint64_t)total + P.nwave - 1) / P.nwave;
			q = q < P.qalign ? P.qalign : (q + P.qalign - 1) & ~uint64_t(P.qalign - 1);
			P.hdr[0] = refused ? 0 : total;
			P.hdr[1] = q;
			P.hdr[2] = refused ? 0 : blocks;
			P.hdr[3] = (uint64_t)exclN + aggN;
			P.hdr[kHdrRefused] = refused ? 1 : 0;
			if (refused && P.err) *P.err = 1u;
		}
	}
	FDBCRC_PT(3)
	if (!ok) return;
	const uint32_t gi = excl + inwave + incl - W;
	P.gs[i] = gi;
	const uint32_t s0 = ~sdv;
	if (g.nb) {
		// block route: the buffer's entry; out[] starts at ~0 (the final
		// inversion) and every block XORs its weighted register in
		const uint64_t q = exclN + inN + inclN - 1;
		const uint64_t E = (P0 + len + 15) & ~uint64_t(15);
		const uint32_t lo = (uint32_t)(4096ull * g.nb - (E - g.A));
		BigEnt ent;
		ent.E = E;
		ent.s = (uint32_t)(exclB + inB + inclB - B);
		ent.idx = (uint32_t)i;
		ent.lot = (lo >> 4) | (g.k0 << 8) | (g.zt << 12);
		ent.sd = s0;
		P.ent[q] = ent;
		P.out[i] = ~0u;
		return;
	}
	if (!W) {
		if (len < 16) {  // byte-serial
			uint32_t r = s0;
			for (uint64_t q = 0; q < len; ++q) r = (r >> 8) ^ s4[3][(r ^ ld1(P.base + off + q)) & 255u];
			P.out[i] = ~r;
			return;
		}
		P.out[i] = ~xs;  // small buffer, finished before the prefixes
		return;
	}
	// Windowed buffers are finished in parts (atomicXor into out[]).  The
	// window kernel does not mask the zt bytes after the buffer's end (they sit
	// in its last chunk): their contribution is cancelled here instead.  Fed
	// alone into the register at E = P1 + zt they give G (four slicing steps
	// over the chunk's last zt bytes), which the kernel's x^(-8 zt) carries to
	// G * x^(-8 zt) at P1 -- independent of where the window sits -- so out[]
	// starts at that term (~(R ^ T) = ~R ^ T: the final inversion is unaffected).
	P.out[i] = xs;  // the tail term (computed with the small buffers above; 0 if zt = 0)
	// a buffer starting on a 16-byte boundary inside its first window (lo != 0:
	// the streaming kernel masks that window anyway) has no garbage before it:
	// the streaming kernel injects its ~seed, stored here, itself
	if (!g.k0 && g.lo) {
		P.cl[i] = s0;
		return;
	}
	// lead term: the lead chunk's bytes below k0 (read only when the buffer
	// starts inside its chunk) with the register ~seed injected at k0, carried
	// to the end of the pass block (chunkpow).  The garbage after the buffer's
	// end is masked by the streaming kernel (it always sits in lane 63).
	u32x4 lc = u32x4{0u, 0u, 0u, 0u};
	if (g.k0) lc = ld16(reinterpret_cast<const uint8_t*>(g.A));
	// Four 4-byte steps: the garbage bytes below k0 kept (~lm), ~seed XORed in
	// at byte k0 (inj); for k0 > 12 the part of ~seed past the chunk is still
	// in the register after it (spill).
	const Masks mk = edge_masks(g.k0, 16u, s0);
	uint32_t x = 0;
#pragma unroll
	for (int d = 0; d < 4; ++d) {
		x ^= (lc[d] & ~mk.lm[d]) ^ mk.inj[d];
		x = s4[0][x & 255u] ^ s4[1][(x >> 8) & 255u] ^ s4[2][(x >> 16) & 255u] ^ s4[3][x >> 24];
	}
	x ^= mk.spill;
	P.cl[i] = vmul(&T->chunkpow[64u * (gi & 3u) + (g.lo >> 4)][0][0], x);
}

// Windows only: at most 72 VGPRs, so 7 blocks per CU hold a whole zipf
// batch (1587 tiles) in one round; with the block route the register demand
// is higher and the tile counts are small.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void k_v7prep_w(V7Params P) {
	v7prep<false>(P);
}
__global__ __launch_bounds__(256) void k_v7prep_b(V7Params P) { v7prep<true>(P); }

// Streaming kernel.  Tables of 64 slots (wave-relative), passes of 4 slots.
constexpr uint32_t k7_LO = 0x7F0u;          // bytes of the window not loaded at its start (1024: empty slot)
constexpr uint32_t k7_INJ = 1u;             // lead slot of an aligned buffer: S holds ~seed, injected at its first byte
constexpr uint32_t k7_ZT = 11;              // trailing zeros of the buffer, when it ends in this table (4 bits)
constexpr uint32_t k7_FIN = 1u << 15;       // the buffer's last slot in this wave
constexpr uint32_t k7_PEND = 1u << 16;      // ... because the wave ends there: the buffer continues
constexpr uint32_t k7_SPLIT = 1u << 17;     // buffer shared with another wave: XOR-merge the part
constexpr uint32_t k7_INV = 1u << 18;       // this part holds window 0 (applies the final inversion)
constexpr uint32_t k7_CONT = 1u << 19;      // buffer began before this table
constexpr uint32_t k7_KF = 20;              // first slot of the buffer inside the table (6 bits)
constexpr uint32_t k7_KL = 26;              // last slot of the buffer's part in the table, 63 if open (6 bits)
// s_waitcnt vmcnt(6) (gfx9 encoding: vmcnt[3:0], expcnt[6:4] = 7, lgkmcnt[11:8] = 15, vmcnt[5:4] at [15:14])
__device__ __forceinline__ void kWaitVm6() { __builtin_amdgcn_s_waitcnt(0x0F76); }
// s_waitcnt vmcnt(8)
__device__ __forceinline__ void kWaitVm8() { __builtin_amdgcn_s_waitcnt(0x0F78); }
struct Tab7 {
	uint64_t wa;   // window address
	uint32_t f;
	uint32_t oi;   // output index relative to the wave's first tile
	uint32_t S;    // team sum of the slot, XORed onto the slot's edge terms (team-sum form)
	uint64_t em;   // (uniform) slots that need masking: window 0 (lo != 0), tail bytes, empty slots
};
// A slot whose chunks all hold its buffer's own bytes needs no masking.
__device__ __forceinline__ bool slot_edge(uint32_t f) { return f & k7_LO; }

// The kernel's arguments read again from the kernarg segment through an
// opaque pointer: s_load at the use (scalar cache, lgkmcnt -- never waits for
// the block loads in flight), so fields used once per 64-buffer batch or per
// table are not held in SGPRs across the whole pass loop (held, they spilled:
// 24 SGPRs into VGPR lanes).
typedef __attribute__((address_space(4))) const V7Params KV7;
__device__ __forceinline__ KV7* v7_kargs() {
#if defined(__HIP_DEVICE_COMPILE__)
	KV7* kp = (KV7*)__builtin_amdgcn_kernarg_segment_ptr();
	asm volatile("" : "+s"(kp));
	return kp;
#else
	return nullptr;
#endif
}

__global__ __launch_bounds__(FDBCRC_V7_THREADS) void k_varlen7(V7Params P) {
	constexpr uint32_t kTS = kV7TabSlots;  // slots per table
	__shared__ uint32_t lds[kLdsBytesB / 4];
	const DevTables* __restrict__ T = P.tabs;
	const LaneCtx c = make_ctx();
	const int lane = c.lane;
	const uint32_t col4 = (lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (lane >> 5) * 0x4000) | col4;
	const uint64_t wpb = blockDim.x >> 6;
	typedef __attribute__((address_space(1))) const uint64_t g_u64;
	const g_u64* hp = (const g_u64*)reinterpret_cast<uintptr_t>(P.hdr);
	const uint64_t total = rdfirst64(hp[0]), Qs = rdfirst64(hp[1]);
	const uint64_t r_base = (uint64_t)blockIdx.x * kV7RangesPerBlock;
	// no slots for this workgroup (e.g. every buffer went to the block route):
	// leave before the table fill
	if (r_base * Qs >= total) return;
	fill_lds_b(lds, T);
	const uint64_t w = r_base + rdfirst(threadIdx.x >> 6);
	const uint64_t lo_s64 = w * Qs;
	if (lo_s64 >= total) return;
	const uint32_t lo_s = (uint32_t)lo_s64;
	const uint32_t hi_s = (uint32_t)(lo_s64 + Qs < total ? lo_s64 + Qs : total);
	// the tile holding slot lo_s: the number of tiles whose inclusive prefix is
	// <= lo_s, narrowed 64 segments at a time
	uint64_t t_lo = 0, t_n = P.ntile;
	while (t_n > 64) {
		const uint64_t stp = (t_n + 63) >> 6;
		const uint64_t k = (uint64_t)lane * stp;
		bool le = false;
		if (k < t_n) {
			const uint64_t idx = t_lo + (k + stp - 1 < t_n ? k + stp - 1 : t_n - 1);
			le = gld64(&P.incl[idx]) <= lo_s;
		}
		const uint64_t cnt = __builtin_popcountll(__ballot(le));
		t_lo += cnt * stp;
		t_n = cnt * stp + stp <= t_n ? stp : t_n - cnt * stp;
	}
	const bool le = (uint64_t)lane < t_n && gld64(&P.incl[t_lo + lane]) <= lo_s;
	const uint64_t bi_w = (t_lo + __builtin_popcountll(__ballot(le))) * kTileW;  // output indices are relative to this

	// ---- batch: 64 buffers, lane j <-> buffer bi0 + j ---------------------
	uint64_t nb_bi0 = bi_w;
	bool more = true;
	uint64_t B_bi0 = 0;
	uint64_t B_wb;          // window 0 address
	uint32_t B_g, B_W, B_f; // first slot, windows, lo | zt << 11
	uint32_t B_cl;
	uint32_t Gb1 = 0;       // wave-relative end of the batch's slots
	uint64_t p_shift = 0;   // bytes from the end of the wave's last window to its buffer's end
	// The metadata of the next 64-buffer batch is loaded one batch ahead: when
	// build() consumes it, the loads have long returned, so they never make the
	// table build wait for the data loads in flight (vmcnt is in order).
	uint64_t pf_off = 0, pf_len = 0;
	uint32_t pf_g = 0, pf_cl = 0;
	auto prefetch = [&](uint64_t bi0) {  // unconditional, clamped into the batch
		KV7* kp = v7_kargs();
		const uint64_t cnt = kp->count;
		const uint64_t j = bi0 + lane < cnt ? bi0 + lane : cnt - 1;
		const uint64_t* const offs = kp->offsets;
		const uint64_t* const lens = kp->lengths;
		pf_off = offs ? offs[j] : j * kp->stride;
		pf_len = lens ? lens[j] : kp->length;
		pf_g = gld32(kp->gs + j);
		pf_cl = gld32(kp->cl + j);
	};
	auto build = [&]() {
		KV7* kp = v7_kargs();
		const uint64_t cnt = kp->count;
		const uint64_t bi0 = nb_bi0;
		const uint64_t j = bi0 + lane;
		const bool ok = j < cnt;
		const uint64_t off = pf_off, len = ok ? pf_len : 0;
		const uint32_t g = ok ? pf_g : 0xFFFFFFFFu, cl = ok ? pf_cl : 0u;
		const Geo7 ge = geo7(reinterpret_cast<uint64_t>(kp->base) + off, len, kp->bigmin);
		const uint32_t W = ok ? ge.W : 0u;
		B_bi0 = bi0;
		B_wb = ge.A - ge.lo;
		B_g = g;
		B_W = W;
		B_f = ge.lo | (ge.zt << k7_ZT) | ((!ge.k0 && ge.lo) ? k7_INJ : 0u);
		// a buffer starting on a 16-byte boundary inside its first window has no
		// lead term: prep stored its ~seed instead, injected into its first word
		// where that window is masked anyway (k7_INJ)
		B_cl = cl;
		nb_bi0 = bi0 + 64;
		prefetch(nb_bi0 < cnt ? nb_bi0 : bi0);
		// end of the slots of this batch: g + W is non-decreasing over the
		// batch's buffers (pieces are in order; W = 0 pieces add nothing), so it
		// is the last buffer's
		const uint64_t nv = cnt - bi0;
		const uint32_t emax = rdlane(g + W, nv < 64 ? (int)nv - 1 : 63);
		Gb1 = (emax > hi_s ? hi_s : emax) - lo_s;
		if (emax < lo_s) Gb1 = 0;
		more = nb_bi0 < cnt && emax < hi_s;
	};
	// slots [sb + k_lo, min(Gb1, sb + 64)) of the current batch into table lanes
	auto expand = [&](Tab7& X, uint32_t sb, uint32_t k_lo) -> uint32_t {
		const uint32_t k_hi = Gb1 - sb < kTS ? Gb1 - sb : kTS;
		const uint32_t ts = lo_s + sb;  // global slot of table lane 0
		// buffer start inside the table, clamped (non-decreasing in j); the
		// owner of lane k is the largest j with st_j <= k
		const uint32_t st = B_g == 0xFFFFFFFFu ? 64u : (B_g <= ts ? 0u : (B_g - ts < 64u ? B_g - ts : 64u));
		uint32_t jj = 0;
#pragma unroll
		for (uint32_t step = 32; step; step >>= 1)
			if (shfl32(st, jj + step) <= (uint32_t)lane) jj += step;
		const uint64_t wb = shfl64(B_wb, jj);
		const uint32_t g = shfl32(B_g, jj), W = shfl32(B_W, jj), bf = shfl32(B_f, jj);
		const uint32_t cl = shfl32(B_cl, jj);
		const uint32_t slot = ts + (uint32_t)lane;
		const uint32_t m = slot - g;
		const uint32_t gend = g + W - 1;                          // the buffer's last slot
		const uint32_t wend = gend < hi_s - 1 ? gend : hi_s - 1;  // ... in this wave
		const bool lead = m == 0;
		const bool fin = slot == wend, pend = fin && wend != gend;
		const bool split = g < lo_s || g + W > hi_s;
		const bool cont = g < ts;
		const bool ends = wend - ts < kTS;  // the part ends inside this table
		const uint32_t f = (lead ? (bf & (1023u | k7_INJ)) : 0u) | ((ends && wend == gend) ? (bf & (15u << k7_ZT)) : 0u) |
		                   (fin ? k7_FIN : 0u) | (pend ? k7_PEND : 0u) | (split ? k7_SPLIT : 0u) |
		                   (g >= lo_s ? k7_INV : 0u) | (cont ? k7_CONT : 0u) | ((cont ? 0u : g - ts) << k7_KF) |
		                   ((ends ? wend - ts : kTS - 1) << k7_KL);
		if ((uint32_t)lane >= k_lo && (uint32_t)lane < k_hi) {
			X.wa = wb + 1024 * (uint64_t)m;
			X.f = f;
			X.S = lead ? cl : 0u;
			X.oi = (uint32_t)(B_bi0 - bi_w) + jj;
		}
		// bytes from the end of the wave's last window to the buffer's end
		const uint64_t pm = __ballot(pend && (uint32_t)lane >= k_lo && (uint32_t)lane < k_hi);
		if (pm) {
			const int k = __builtin_ctzll(pm);
			p_shift = 1024 * (uint64_t)(rdlane(W, k) - 1 - rdlane(m, k)) - ((rdlane(bf, k) >> k7_ZT) & 15u);
		}
		return k_hi;
	};
	auto build_table = [&](Tab7& X, uint32_t sb) -> uint32_t {
		X.wa = 0;
		X.f = 1024u;
		X.oi = 0;
		X.S = 0;
		uint32_t filled = 0;
		for (;;) {
			if (Gb1 > sb + filled) filled = expand(X, sb, filled);
			if (filled == kTS || !more) break;
			build();
		}
		if (filled && filled < kTS) {  // empty slots re-read a chunk of slot 0 (never used)
			const uint64_t w0 = rdlane64(X.wa, 0);
			if ((uint32_t)lane >= filled) X.wa = w0;
		}
		X.em = __ballot(slot_edge(X.f));  // (slots with sd have lo != 0)
		return filled;
	};
	// load k of a pass fetches team {0,2,1,3}[k]'s window.  Every load is
	// issued unconditionally (a branch around a load defeats the compiler's
	// wait counting): chunks of window 0 before the buffer's first chunk, and
	// empty slots, re-read the lead chunk (empty slots: slot 0's last chunk)
	// and are zeroed at compute time.
	auto load = [&](Block& nb, const Tab7& X, uint32_t p) {
		const bool edge = (X.em >> (4 * p)) & 15u;  // uniform: plain passes skip the lead clamp
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint32_t s = 4 * p + (((k & 1) << 1) | (k >> 1));
			const uint64_t wa = rdlane64(X.wa, (int)s);
			uint32_t off = c.ld_off;
			if (edge) {
				const uint32_t lo = rdlane(X.f, (int)s) & k7_LO;
				const uint32_t lc = lo < 1008u ? lo : 1008u;
				off = off > lc ? off : lc;
			}
			nb.r[k] = ld16(reinterpret_cast<const uint8_t*>(wa + off));
		}
	};
	auto compute = [&](Block& b, Tab7& X, uint32_t p) {
		if ((X.em >> (4 * p)) & 15u) {  // a slot of this pass holds an edge, or nothing
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint32_t f = rdlane(X.f, (int)(4 * p + (((k & 1) << 1) | (k >> 1))));
			const uint32_t lo = f & k7_LO;
			if (lo) {  // window 0: chunks before the buffer's first chunk
				const bool z = c.ld_off < lo;
#pragma unroll
				for (int d = 0; d < 4; ++d) b.r[k][d] = z ? 0u : b.r[k][d];
				if (f & k7_INJ) {  // aligned buffer: ~seed (held in S) into the first word of its lead chunk (window offset lo)
					const int s = (int)(4 * p + (((k & 1) << 1) | (k >> 1)));
					const uint32_t sd = rdlane(X.S, s);
					const uint32_t ln = 32 * ((lo >> 4) & 1) + 16 * ((lo >> 5) & 1) + ((lo >> 6) & 15);
					b.r[k][0] ^= (uint32_t)lane == ln ? sd : 0u;
					X.S = lane == s ? 0u : X.S;
				}
			}
			// (the bytes after a buffer's end, in lane 63's chunk of its last
			// window, are not masked: prep's tail term in out[] cancels them)
		}
		}
		unswizzle(b);
		const uint32_t R = row_xor(mul_nibbles(lds, chain64_b(lds, 0u, b, c4), c_lane));
		const uint32_t v = shfl32(R, ((uint32_t)lane & 3u) * 16u);
		X.S ^= ((uint32_t)lane >> 2) == p ? v : 0u;
	};
	// Combining a table: one round of table lookups weights every slot sum
	// straight to its buffer's end (slotw[kl - 4p][zt]), so a prefix XOR over
	// the lanes leaves each buffer's final register at its last slot.  The
	// lookups (global gathers, which share the in-order vmcnt with the data
	// loads) are issued after the table's last pass (phase 1) and consumed in
	// the next table's first pass, right after its next loads (phase 2): the
	// wait then coincides with one the pipeline does anyway.  Every vector
	// memory operation here is unconditional (lanes with nothing to finish XOR
	// 0 into a dummy word): a load or store skipped by a branch would make the
	// compiler wait for all loads in flight.
	uint32_t carry = 0;     // register of the buffer open across the table boundary (relative to the table end)
	uint32_t pend_filled = 0;
	uint32_t gv[8];         // nibble-table words in flight (never live across a pass's compute)
	auto phase1 = [&](Tab7& X, uint32_t filled) {
		const uint32_t f = X.f;
		const uint32_t d = (((f >> k7_KL) & 63u) - ((uint32_t)lane >> 2) * 4u) & 63u;
		const uint32_t(*tab)[16] = v7_kargs()->tabs->slotw[d][(f >> k7_ZT) & 15u];
		const uint32_t v = X.S;
#pragma unroll
		for (int n = 0; n < 8; ++n) gv[n] = gld32(&tab[n][(v >> (4 * n)) & 15u]);
		pend_filled = filled;
	};
	auto phase2 = [&](Tab7& X) {
		const uint32_t D = xor3(xor3(gv[0], gv[1], gv[2]), xor3(gv[3], gv[4], gv[5]), gv[6] ^ gv[7]);
		const uint32_t Pp = scanx(D, lane);
		const uint32_t f = X.f;
		const uint32_t kf = (f >> k7_KF) & 63u;
		const bool cont = f & k7_CONT;
		const uint32_t pk = shfl32(Pp, kf ? kf - 1 : 0u);
		uint32_t v = Pp ^ ((!cont && kf) ? pk : 0u);
		// the register carried in from the previous table belongs to the buffer
		// holding slot 0 (CONT): to its finishing slot, or across this table
		const uint32_t f0 = rdlane(f, 0);
		const uint32_t kl0 = (f0 >> k7_KL) & 63u;
		const bool fin0 = (f0 & k7_CONT) && (rdlane(f, (int)kl0) & k7_FIN);
		uint32_t cc = 0;
		if (carry) {
			const DevTables* Tk = v7_kargs()->tabs;
			cc = umul(fin0 ? Tk->carryw[kl0][(f0 >> k7_ZT) & 15u] : Tk->table_shift, carry);
		}
		const bool fin = (f & k7_FIN) && (uint32_t)lane < pend_filled;
		v ^= (cont && (fin || lane == (int)kTS - 1)) ? cc : 0u;
		carry = (pend_filled == kTS && !(rdlane(f, kTS - 1) & k7_FIN)) ? rdlane(v, kTS - 1) : 0u;
		const uint64_t pm = __ballot(fin && (f & k7_PEND));
		if (pm) {  // the wave's last buffer continues in the next wave: shift its part to the buffer's end
			const int k = __builtin_ctzll(pm);
			const uint32_t vv = mul_xpow(v7_kargs()->tabs, rdlane(v, k), p_shift);
			v = lane == k ? vv : v;
		}
		// windowed buffers' out[] words are zeroed by the prep kernel; the part
		// holding window 0 carries the final inversion
		KV7* kp = v7_kargs();
		const uint64_t wd = (uint64_t)blockIdx.x * kV7RangesPerBlock + rdfirst(threadIdx.x >> 6);  // (w, not held)
		atomicXor(fin ? kp->out + bi_w + X.oi : kp->dummy + wd * 64 + lane, fin ? ((f & k7_INV) ? ~v : v) : 0u);
	};
	// Two blocks in ping-pong (a register copy would wait for the loads in
	// flight): pass p computes from one while pass p + 1 loads into the other.
	// Full tables have 16 passes, so the next table's pass 0 lands in ba.
	static_assert(kTS == 64, "16 passes per table");
	Block ba, bb;
	// all passes of table X (its pass 0 already issued into ba); V holds the
	// previous table (phase 1 done) and is rebuilt as the next table
	auto run_table = [&](Tab7& X, Tab7& V, uint32_t sbX, uint32_t fX) -> uint32_t {
		const uint32_t npass = (fX + 3) >> 2;
		uint32_t fY = 0;
		uint32_t p = 0;
		if (npass >= 3) {  // first pair: the previous table's phase 2
			load(bb, X, 1);
			__builtin_amdgcn_sched_barrier(0);
			phase2(V);
			__builtin_amdgcn_sched_barrier(0);
			compute(ba, X, 0);
			__builtin_amdgcn_sched_barrier(0);
			load(ba, X, 2);
			__builtin_amdgcn_sched_barrier(0);
			compute(bb, X, 1);
			__builtin_amdgcn_sched_barrier(0);
			p = 2;
		} else {
			phase2(V);
		}
		// steady state: only the data loads touch vector memory.  The explicit
		// wait (a no-op at run time) pins the loop's entry state for the
		// compiler's wait-count pass.
		kWaitVm6();
		for (; p + 2 < npass; p += 2) {
			load(bb, X, p + 1);
			__builtin_amdgcn_sched_barrier(0);
			compute(ba, X, p);
			__builtin_amdgcn_sched_barrier(0);
			load(ba, X, p + 2);
			__builtin_amdgcn_sched_barrier(0);
			compute(bb, X, p + 1);
			__builtin_amdgcn_sched_barrier(0);
			kWaitVm6();
		}
		if (p + 1 < npass) {  // last pair: the next table's pass 0 goes to ba
			load(bb, X, p + 1);
			__builtin_amdgcn_sched_barrier(0);
			compute(ba, X, p);
			__builtin_amdgcn_sched_barrier(0);
			fY = fX == kTS ? build_table(V, sbX + kTS) : 0u;
			if (fY) load(ba, V, 0);
			__builtin_amdgcn_sched_barrier(0);
			compute(bb, X, p + 1);
			__builtin_amdgcn_sched_barrier(0);
		} else {  // a single pass left (odd pass count: the wave's last table)
			compute(ba, X, p);
			__builtin_amdgcn_sched_barrier(0);
		}
		phase1(X, fX);
		return fY;
	};

	Tab7 t0, t1;
	t1.wa = 0;
	t1.f = 1024u;  // empty: the first table's "previous table" finishes nothing
	t1.oi = 0;
	t1.S = 0;
	t1.em = ~0ull;
	phase1(t1, 0);
	prefetch(nb_bi0);
	build();
	uint32_t sb = 0;
	uint32_t f0 = build_table(t0, 0);
	if (f0) load(ba, t0, 0);
	while (f0) {
		const uint32_t f1 = run_table(t0, t1, sb, f0);
		sb += kTS;
		if (!f1) {
			phase2(t0);
			break;
		}
		f0 = run_table(t1, t0, sb, f1);
		sb += kTS;
		if (!f0) phase2(t1);
	}
	(void)wpb;
}

#ifndef FDBCRC_BIGMIN
#define FDBCRC_BIGMIN 4096  // smallest span (bytes) sent to the block route; 0 disables it
#endif
static_assert(FDBCRC_BIGMIN == 0 || FDBCRC_BIGMIN >= 4096, "the route's edge terms assume distinct lead and tail chunks");

static uint64_t al16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

uint64_t varlen7_workspace_bytes(uint64_t count, uint64_t nwave) {
	nwave = nwave > 16 * 1024 ? nwave : 16 * 1024;  // covers any launch geometry up to 1024 CUs
	const uint64_t ntile = (count + kTileW - 1) / kTileW;
	return 64 + 32 * (ntile + 1) + al16(4 * nwave + 8 * count) + 256 * nwave + 4 * nwave + 64  // window route
	       + 16 * (ntile + 1) + 8 * count + 4 * al16(4 * count)                                    // block route
	       + 4 * nwave;                                                                            // its counters
}

int launch_varlen7(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t stride,
                   uint64_t length, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                   const DevTables* tabs, int num_cus, void* ws, hipStream_t stream, int route, uint64_t* hstat,
                   uint32_t* err, const XState* xs, uint32_t* bacc, uint32_t* pctr) {
	const uint64_t grid = (uint64_t)num_cus;
	const uint64_t nwave = grid * kV7RangesPerBlock;  // one slot range per wave
	const uint64_t ntile = (count + kTileW - 1) / kTileW;
	uint8_t* wp = static_cast<uint8_t*>(ws);
	V7Params P{};
	P.base = base; P.offsets = offsets; P.lengths = lengths; P.stride = stride; P.length = length; P.count = count;
	P.seed = seed; P.seeds = seeds; P.out = out; P.tabs = tabs;
	P.ntile = ntile; P.nwave = nwave; P.qalign = 4;
	// block route: output indices are 32-bit there.  FDBCRC_BIGMIN in the
	// environment (development: route threshold experiments) overrides the
	// built-in threshold; values below 4096 are raised to it, 0 disables.
	static const uint64_t bigmin_env = [] {
		const char* e = getenv("FDBCRC_BIGMIN");
		if (!e) return (uint64_t)FDBCRC_BIGMIN;
		const uint64_t v = strtoull(e, nullptr, 0);
		return v == 0 ? 0 : (v < 4096 ? 4096 : v);
	}();
	// kRouteBoth: spans from bigmin up go to the blocks, the rest to windows;
	// kRouteWindows: no block launch; kRouteBlocks: every windowed span goes to
	// the blocks and the window kernel is not launched
	P.bigmin = count >= 0xFFFFFFFFull || route == kRouteWindows || route == kRouteExtent ? 0
	           : route == kRouteBlocks                          ? kSmallSpan + 1
	                                                            : bigmin_env;
	if (route == kRouteBlocks && P.bigmin == 0) route = kRouteWindows;
	P.hstat = hstat;
	P.err = err;
	const bool extent = route == kRouteExtent && xs != nullptr && count < (1ull << 31);  // (point ids 2i + end: 32 bits)
	if (route == kRouteExtent) route = kRouteWindows;  // the fallback: windows
	if (extent) {
		P.xhdr = xs->xhdr;
		P.epoch = xs->epoch;
		if (xs->ctr) {
			P.xwq = xs->wq;
			P.xcapg = xs->capg;
		}
	}
	P.hdr = reinterpret_cast<uint64_t*>(wp);      // [0..3] totals and quantum, [kHdrRefused] refusal flag
	P.tsum = reinterpret_cast<uint64_t*>(wp + 64);
	P.incl = P.tsum + ntile + 1;
	P.bsum = P.incl + ntile + 1;
	P.nsum = P.bsum + ntile + 1;
	uint32_t* wave_tile = reinterpret_cast<uint32_t*>(P.nsum + ntile + 1);  // k_scan output (unused here)
	P.gs = wave_tile + nwave;
	P.cl = P.gs + count;
	P.dummy = P.cl + count;
	uint8_t* rp = reinterpret_cast<uint8_t*>(P.dummy + 64 * nwave + nwave) + 64;
	rp = reinterpret_cast<uint8_t*>(al16(reinterpret_cast<uint64_t>(rp)));
	P.ent = reinterpret_cast<BigEnt*>(rp);
	rp += al16(sizeof(BigEnt) * count);
	P.bctr = reinterpret_cast<uint32_t*>(rp);
	P.nbctr = (uint32_t)(kPageCtrWords * grid);
	// tile prefixes: each prep block sums its predecessors (up to kScanTiles tiles);
	// larger batches scan the tile sums first; batches of at most
	// kSelfSumTiles tiles skip the count kernel (a prep block counts its
	// predecessors' windows itself: one launch less, which is most of a small
	// batch's latency; 32 tiles: chunks 0.202 -> 0.198 ms, 8 Ki x 16 KiB +-0)
	// (summing the predecessors costs each prep block O(tile) loads: past
	// kScanTiles tiles one scan block is cheaper)
	P.scanned = ntile > kScanTiles;
	P.selfsum = ntile <= kSelfSumTiles;
	if (extent) {
		k_xcount<<<(unsigned)ntile, 256, 0, stream>>>(P);  // the packing check and the grab map
		launch_extent(base, offsets, lengths, stride, length, count, seed, seeds, out, tabs, num_cus, *xs, hstat, stream,
		              0);
		launch_extent(base, offsets, lengths, stride, length, count, seed, seeds, out, tabs, num_cus, *xs, hstat, stream,
		              1);
		return 0;
	}
	// The block route alone over a list batch of at most kNPMax buffers, with
	// the stream's part accumulators: no prep, one kernel (k_bigblocks<U, true>
	// plans its own blocks).  FDBCRC_NP=0 (development) keeps the prep.
	static const bool np_env = [] {
		const char* e = getenv("FDBCRC_NP");
		return !(e && atoi(e) == 0);
	}();
	if (np_env && route == kRouteBlocks && P.bigmin && bacc && pctr && offsets && lengths && count <= kNPMax &&
	    (uint64_t)num_cus <= 1024) {
		BigParams B{};
		B.out = out;
		B.ctr = pctr;
		B.tabs = tabs;
		B.base = base;
		B.offsets = offsets;
		B.lengths = lengths;
		B.nbuf = count;
		B.seed = seed;
		B.seeds = seeds;
		B.acc = bacc;
		B.priv = reinterpret_cast<BigEnt*>(al16(reinterpret_cast<uint64_t>(P.gs)));  // (the window route's area)
		B.hstat = hstat;
		B.err = err;
		return launch_bigblocks_np(B, num_cus, stream);
	}
	if (!P.selfsum) k_v7count<<<(unsigned)ntile, 256, 0, stream>>>(P);
	if (P.scanned)
		k_scan<<<1, 1024, 0, stream>>>(P.tsum, ntile, wave_tile, nwave, P.hdr, 4, 4, P.bigmin ? P.bsum : nullptr,
		                               P.bigmin ? P.nsum : nullptr);
	if (P.bigmin)
		k_v7prep_b<<<(unsigned)ntile, 256, 0, stream>>>(P);
	else
		k_v7prep_w<<<(unsigned)ntile, 256, 0, stream>>>(P);
	if (P.bigmin) {
		BigParams B{};
		B.hdr = P.hdr; B.ent = P.ent;
		B.out = out; B.ctr = P.bctr; B.tabs = tabs;
		launch_bigblocks(B, num_cus, stream);
	}
	if (route != kRouteBlocks) k_varlen7<<<(unsigned)grid, FDBCRC_V7_THREADS, 0, stream>>>(P);
	return 0;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
uint64_t varlen_workspace_bytes(uint64_t count, uint64_t nwave) { return varlen7_workspace_bytes(count, nwave); }

int launch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count, uint32_t seed,
                  const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, void* ws,
                  hipStream_t stream, int route, uint64_t* hstat, uint32_t* err, const XState* xs, uint32_t* bacc,
                  uint32_t* pctr) {
	return launch_varlen7(base, offsets, lengths, 0, 0, count, seed, seeds, out, tabs, num_cus, ws, stream, route,
	                      hstat, err, xs, bacc, pctr);
}

// Fixed stride, any length and alignment: the same engine with metadata
// computed on the fly.  The length is known here, so is the route: 16 KiB
// or more (blocks waste at most 20 %) goes to the blocks, the rest to windows.
int launch_fixed_general(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                         const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, void* ws,
                         hipStream_t stream) {
	return launch_varlen7(base, nullptr, nullptr, stride, length, count, seed, seeds, out, tabs, num_cus, ws, stream,
	                      length >= 16384 ? kRouteBlocks : kRouteWindows, nullptr);
}

#ifdef FDBCRC_DEBUG
__global__ void k_dbg_set(unsigned long long lo, unsigned long long hi) {
	g_dbg[0] = lo; g_dbg[1] = hi;
	for (int k = 2; k < 8; ++k) g_dbg[k] = 0;
}
__global__ void k_dbg_get(unsigned long long* out) {
	for (int k = 0; k < 8; ++k) out[k] = g_dbg[k];
}
#endif

}  // namespace fdbcrc

#ifdef FDBCRC_DEBUG
// Debug builds only (make debug): allowed window for the data loads of the
// varlen engine and the block route (lo = hi = 0: no checking), and readback
// of [lo, hi, violations, first bad address, site, ...] over both.
namespace fdbcrc {
void dbg_set_pages(uint64_t lo, uint64_t hi);
void dbg_get_pages(uint64_t* d_out8);
}
extern "C" int crc32c_debug_bounds(uint64_t lo, uint64_t hi) {
	fdbcrc::k_dbg_set<<<1, 1>>>(lo, hi);
	fdbcrc::dbg_set_pages(lo, hi);
	return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
extern "C" int crc32c_debug_read(uint64_t* d_out8) {
	uint64_t a[8], b[8];
	fdbcrc::k_dbg_get<<<1, 1>>>(reinterpret_cast<unsigned long long*>(d_out8));
	if (hipMemcpy(a, d_out8, 64, hipMemcpyDeviceToHost) != hipSuccess) return -3;
	fdbcrc::dbg_get_pages(d_out8);
	if (hipMemcpy(b, d_out8, 64, hipMemcpyDeviceToHost) != hipSuccess) return -3;
	if (!a[2]) {
		a[3] = b[3];
		a[4] = b[4];
	}
	a[2] += b[2];
	return hipMemcpy(d_out8, a, 64, hipMemcpyHostToDevice) == hipSuccess ? 0 : -3;
}
#endif

#ifdef FDBCRC_PTIMES
extern "C" int fdbcrc_debug_ptimes(void* host, uint64_t ntile) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbcrc::g_pt), ntile * 32, 0, hipMemcpyDeviceToHost);
}
#endif
