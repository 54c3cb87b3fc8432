// Extent route of the variable-length engine (gfx950): batches whose buffers
// are PACKED -- ascending, no overlaps, small gaps: packets back to back in a
// receive buffer (fdbrpc/FlowTransport.cpp:1260-1364 scans them out of one),
// chunks of a file (fdbrpc/FileTransfer.cpp:29-37).  Reference semantics:
// crc32c_append (contrib/crc32/crc32c.cpp:346-356) per buffer.
//
// The whole covering byte range -- the EXTENT [S, Eend), S = the first
// buffer's start rounded down to 16 -- is streamed as 4 KiB blocks exactly
// like 4 KiB pages (k_pages4k's loads, permlane swizzle, register chains), so
// no byte is padded and nothing is masked.  Every buffer's CRC comes from two
// PREFIX registers of that stream (CRC linearity; tests/extent_model.py is
// the byte-exact CPU model, extent_crcs_ranges the form implemented here):
//     raw(bytes [s, e)) = R(e) ^ R(s) * x^(8(e - s))
// so the gap bytes between buffers cancel.  Wave w streams the blocks
// [k0, k1) = [w*per, (w+1)*per) of its RANGE and keeps R relative to the
// range's start: X_k (0 at k0), Z[k] = X_k * M (M = x^(8*4096)), stored per
// block, X_{k+1} = Z[k] ^ B[k] (B: the block register), the range's end value
// A[w] = X_{k1}.  A point p in block k = (p-1) >> 12 with cnt = (p - 4096k) >> 6
// whole lane spans before it has, positioned at block k's end,
//     G(p) = Z[k] ^ H_k[cnt-1]
// (H_k: the block's lane registers weighted to the block end -- the page
// kernel's fold -- XOR-prefixed over the lanes; the stream kernel captures
// H_k[cnt-1] for every point of its blocks), and
//     R(p64) = G(p) * x^(-8*64*(64-cnt)),   R(p) = R(p64) fed the p - p64 < 64 bytes after p64.
// A buffer whose two points lie in one range needs nothing else (the range's
// global start register cancels); one spanning ranges ws < we adds
// D = (A[ws] M^per ^ A[ws+1]) M^per ... ^ A[we-1] to its end point's prefix,
// positioned there: G(e) ^= D * M^(ke - k0(we) + 1).  Then
//     crc32c_append(seed, buffer) = ~(R(e) ^ (R(s) ^ ~seed) * x^(8 len)).
//
//   k_v7count (crc32c_varlen.hip)  the packing and capacity checks (epoch-tagged
//                                  flags) and the stream's route statistics
//   k_xstream   static block ranges per wave; per block: chains, lane weights,
//               prefix XOR (DPP), the block register; the points of the block
//               from a window of 64 buffers in the lanes (ds_bpermute)
//   k_xz        per range: the block registers turned into the range-local
//               prefixes Z (a lane-parallel weighted scan, LDS tables)
//   k_xfin      per buffer: R(s), R(e) (the < 64-byte remainders re-read),
//               the range aggregates between them, x^(8 len), the inversion;
//               a batch that failed the checks: every buffer directly, one
//               lane each (x_fallback)
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "crc32c_common.h"

namespace fdbcrc {

namespace {

typedef __attribute__((address_space(1))) const uint32_t xg_u32;
typedef __attribute__((address_space(1))) const uint64_t xg_u64;
__device__ __forceinline__ uint32_t xld32(const uint32_t* p) { return *((xg_u32*)reinterpret_cast<uintptr_t>(p)); }
__device__ __forceinline__ uint64_t xld64(const uint64_t* p) { return *((xg_u64*)reinterpret_cast<uintptr_t>(p)); }
// A uniform word through the constant address space: s_load (lgkmcnt), so
// waiting for it never waits for the block loads in flight (in-order vmcnt);
// only for words no kernel of the launch writes (the grab map).
__device__ __forceinline__ uint32_t sld32(const uint32_t* p) {
	typedef __attribute__((address_space(4))) const uint32_t c_u32;
	return *((const c_u32*)reinterpret_cast<uintptr_t>(p));
}

// Lane-parallel multiply by a constant whose nibble tables are in global
// memory (8 gathers, L2-resident).
__device__ __forceinline__ uint32_t xmul(const uint32_t (*tab)[16], uint32_t v) {
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= xld32(&tab[n][(v >> (4 * n)) & 15u]);
	return r;
}

struct XParams {
	const uint8_t* base;
	const uint64_t* offsets;   // nullptr: fixed stride
	const uint64_t* lengths;   // nullptr: fixed length
	uint64_t stride, length, count;
	uint32_t seed;
	const uint32_t* seeds;
	uint32_t* out;
	XState x;
	const DevTables* tabs;
	uint64_t* hstat;
	uint64_t nwave;  // waves of k_xstream (its static ranges)
	uint32_t* ctr;   // k_xgrab: the stream's per-workgroup grab counters (page_counters)
	bool grabs;      // k_xgrab streamed the batch (else k_xstream's static ranges)
	uint64_t ngrid;  // workgroups of the grab stream (k_xgrab / k_xgf): one per CU
};

__device__ __forceinline__ void x_buffer(const XParams& P, uint64_t i, uint64_t& P0, uint64_t& P1) {
	const uint64_t off = P.offsets ? xld64(P.offsets + i) : i * P.stride;
	const uint64_t len = P.lengths ? xld64(P.lengths + i) : P.length;
	P0 = reinterpret_cast<uint64_t>(P.base) + off;
	P1 = P0 + len;
}

// Wave-uniform: the batch passed the packing and capacity checks of this
// launch (k_v7count stored the launch's epoch where it failed one).
__device__ __forceinline__ bool x_packed(const XParams& P) {
	const uint32_t a = rdfirst(xld32(P.x.xhdr)), b = rdfirst(xld32(P.x.xhdr + 1));
	return a != P.x.epoch && b != P.x.epoch;
}
__device__ __forceinline__ bool x_unordered(const XParams& P) { return rdfirst(xld32(P.x.xhdr)) == P.x.epoch; }

struct XGeo {
	uint64_t S, Eend, nblk;
};
// The extent of a packed batch: its first buffer's start rounded down to 16,
// its last buffer's end rounded up to 16.
__device__ __forceinline__ XGeo x_geo(const XParams& P) {
	uint64_t a0, a1, b0, b1;
	x_buffer(P, 0, a0, a1);
	x_buffer(P, P.count - 1, b0, b1);
	XGeo g;
	g.S = rdfirst64(a0 & ~uint64_t(15));
	g.Eend = rdfirst64((b1 + 15) & ~uint64_t(15));
	g.nblk = (g.Eend - g.S + 4095) >> 12;
	return g;
}

// The launch's checks and the extent with every load issued at once (at the
// start of k_xgrab): x_packed, then x_geo behind x_buffer's
// stride / list branches, were four dependent scalar round trips before any
// wave could load a block.  Unconditional: a fixed-stride or fixed-length
// batch reads xhdr instead and discards it.
struct XStart {
	bool packed, unordered;
	XGeo G;
};
__device__ __forceinline__ XStart x_start(const XParams& P) {
	const uint64_t* const dflt = reinterpret_cast<const uint64_t*>(P.x.xhdr);
	const uint64_t* const po = P.offsets ? P.offsets : dflt;
	const uint64_t* const pl = P.lengths ? P.lengths : dflt;
	const uint64_t il = P.count - 1;
	const uint64_t o0 = xld64(po), o1 = xld64(po + (P.offsets ? il : 0)), l1 = xld64(pl + (P.lengths ? il : 0));
	const uint32_t a = rdfirst(xld32(P.x.xhdr)), b = rdfirst(xld32(P.x.xhdr + 1));
	XStart x;
	x.packed = a != P.x.epoch && b != P.x.epoch;
	x.unordered = a == P.x.epoch;
	const uint64_t base = reinterpret_cast<uint64_t>(P.base);
	const uint64_t a0 = base + (P.offsets ? o0 : 0);
	const uint64_t b0 = base + (P.offsets ? o1 : il * P.stride);
	const uint64_t b1 = b0 + (P.lengths ? l1 : P.length);
	x.G.S = rdfirst64(a0 & ~uint64_t(15));
	x.G.Eend = rdfirst64((b1 + 15) & ~uint64_t(15));
	x.G.nblk = (x.G.Eend - x.G.S + 4095) >> 12;
	return x;
}

// Blocks per wave of k_xstream's static ranges: whole units of 2U blocks.
__device__ __forceinline__ uint64_t x_per(uint64_t nblk, uint64_t nwave) {
	return (((nblk + nwave - 1) / nwave) + 3) / 4 * 4;
}

// Point p (bytes from S): its block and the whole lane spans before it in
// that block (0..64).  p = 0 maps to block 0 with no span before it: the
// register captured there is 0, as R(0) is.
__device__ __forceinline__ uint32_t x_blk(uint64_t p) { return p ? (uint32_t)((p - 1) >> 12) : 0u; }
__device__ __forceinline__ uint32_t x_cnt(uint64_t p, uint32_t k) {
	return p ? (uint32_t)((p - 4096ull * k) >> 6) : 0u;
}

}  // namespace

// ---------------------------------------------------------------------------
// k_xstream: the extent as 4 KiB blocks, static block ranges per wave
// ---------------------------------------------------------------------------
constexpr uint32_t kXU = 2;  // blocks per unit (register chains interleaved)

__global__ __launch_bounds__(1024) void k_xstream(XParams P) {
	if (!x_packed(P)) return;  // k_xfin checksums this batch buffer by buffer
	if (x_geo(P).nblk == 0) return;  // every buffer empty at one 16-byte-aligned address: k_xfin alone
	FillRegs fill;
	fill_issue_1024(fill, P.tabs);  // table loads in flight while the ranges are found
	__shared__ uint32_t lds[kLdsBytesB / 4];
	const XGeo G = x_geo(P);
	const LaneCtx c = make_ctx();
	const uint32_t lane = (uint32_t)c.lane;
	const uint32_t col4 = (lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (lane >> 5) * 0x4000) | col4;
	const uint32_t wi = rdfirst(threadIdx.x >> 6);
	const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
	const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wi;
	// static ranges of whole units (the extent's blocks are consecutive)
	static_assert(2 * kXU == 4, "x_per: ranges of whole units");
	const uint64_t per = x_per(G.nblk, nwave);
	const uint64_t k0 = w * per < G.nblk ? w * per : G.nblk;
	const uint64_t k1 = k0 + per < G.nblk ? k0 + per : G.nblk;
	// The extent's last block may run past its end: it is left out of the main
	// loop (whose loads then need no clamping, and no branch: a branch around
	// a load makes the compiler wait for every load in flight) and done at
	// the end by its wave with clamped loads.
	const uint64_t km = k1 < G.nblk ? k1 : G.nblk - 1;  // main-loop blocks [k0, km)
	const uint64_t ksafe = km > k0 ? km - 1 : 0;        // (only used when km > k0)
	auto load_blk = [&](Block& b, uint64_t k) {
		const uint64_t kk = k < km ? k : ksafe;  // past the range: duplicates, discarded
		load_block(b, reinterpret_cast<const uint8_t*>(G.S + 4096ull * kk), c.ld_off);
	};
	Block u0[kXU], u1[kXU];
	if (km > k0) {  // (a wave without main-loop blocks loads nothing here: its block may be the last)
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) load_blk(u0[j], k0 + j);
	}

	// ---- window of 64 buffers (lane j <-> buffer q + j): its points -------
	// the first buffer whose end lies past this range's start (64-ary narrowing)
	const uint64_t T0 = G.S + 4096ull * k0;
	uint64_t qa = 0, qm = P.count;
	while (qm > 64) {
		const uint64_t stp = (qm + 63) >> 6;
		const uint64_t kk = (uint64_t)lane * stp;
		bool le = false;
		if (kk < qm) {
			uint64_t a, b;
			x_buffer(P, qa + (kk + stp - 1 < qm ? kk + stp - 1 : qm - 1), a, b);
			le = b <= T0;
		}
		const uint64_t cnt = __builtin_popcountll(__ballot(le));
		qa += cnt * stp;
		qm = cnt * stp + stp <= qm ? stp : qm - cnt * stp;
	}
	uint64_t q;
	{
		bool le = false;
		if (lane < qm) {
			uint64_t a, b;
			x_buffer(P, qa + lane, a, b);
			le = b <= T0;
		}
		q = qa + __builtin_popcountll(__ballot(le));
	}
	// per lane: start / end blocks, whole lane spans before each point and the
	// 16-byte chunk of its span it lies in; uniform: the window's last end block
	uint32_t wbs, wbe, wcs, wce, wqs, wqe, wlast;
	uint32_t Vs = 0, Ve = 0, Ys = 0, Ye = 0;  // captured: G(p) and the span's register at p's chunk
	uint64_t pf0 = 0, pf1 = 0;  // the next window's buffer (prefetched one window ahead)
	auto prefetch = [&](uint64_t q0) {
		const uint64_t j = q0 + lane < P.count ? q0 + lane : P.count - 1;
		x_buffer(P, j, pf0, pf1);
	};
	auto make_window = [&](uint64_t q0) {
		const bool ok = q0 + lane < P.count;
		const uint64_t s = pf0 - G.S, e = pf1 - G.S;
		wbs = ok ? x_blk(s) : 0xFFFFFFFEu;
		wbe = ok ? x_blk(e) : 0xFFFFFFFEu;
		wcs = x_cnt(s, wbs);
		wce = x_cnt(e, wbe);
		wqs = ((uint32_t)s >> 4) & 3u;  // (p - 4096k - 64 cnt) >> 4: S is 16-byte aligned
		wqe = ((uint32_t)e >> 4) & 3u;
		wlast = q0 + 64 <= P.count ? rdlane(wbe, 63) : 0xFFFFFFFFu;  // the batch's last window never retires
		Vs = Ve = Ys = Ye = 0;
	};
	uint32_t* const dmy = P.x.dummy + 128 * w;
	// the window's points that lie in this wave's blocks leave (the others
	// belong to the neighbouring ranges); unconditional stores
	auto flush = [&](uint64_t q0) {
		const bool ok = q0 + lane < P.count;
		const bool os = ok && wbs >= k0 && wbs < k1, oe = ok && wbe >= k0 && wbe < k1;
		typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
		*reinterpret_cast<u32x2*>(os ? P.x.ps + 2 * (q0 + lane) : dmy + 2 * lane) = u32x2{Vs, Ys};
		*reinterpret_cast<u32x2*>(oe ? P.x.pe + 2 * (q0 + lane) : dmy + 2 * lane) = u32x2{Ve, Ye};
	};
	prefetch(q);
	make_window(q);
	prefetch(q + 64);

	fill_commit_1024(fill, lds);
	if (k0 >= k1) return;

	// ---- blocks -------------------------------------------------------------
	// X: the range-local prefix register at the start of the next block (0 at
	// k0).  Per block: Z = X * M (M = x^(8*4096)), X = Z ^ B.  The uniform
	// multiply by M chains two of the lane tables already in LDS -- lane 0's
	// x^(8*64*63) and lane 62's x^(8*64) -- eight lanes per table (lane n:
	// nibble n; all 64 lanes run it, lanes n and n + 8k read the same word).
	uint32_t X = 0;
	auto mulM = [&](uint32_t v) -> uint32_t {
		const uint32_t n = lane & 7;
		uint32_t t = lds_rd(lds, kS4LaneOff + ((n * 16 + ((v >> (4 * n)) & 15u)) << 7));
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0x124, 0xF, 0xF, false);  // row_ror:4 (n ^ 4)
		t = rdfirst(t);
		uint32_t u = lds_rd(lds, kS4LaneOff + 4 * (4096 + (n * 16 + ((t >> (4 * n)) & 15u)) * 32 + 30));
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0xB1, 0xF, 0xF, false);
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0x4E, 0xF, 0xF, false);
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0x124, 0xF, 0xF, false);
		return rdfirst(u);
	};
	// chains, lane weights and the prefix XOR over the lanes of one unit; Y:
	// each lane's register after 16, 32 and 48 bytes of its span
	auto unit_h = [&](Block (&u)[kXU], uint32_t (&H)[kXU], uint32_t (&Y)[kXU][3]) {
		uint32_t x[kXU];
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) {
			unswizzle(u[j]);
			x[j] = u[j].r[0][0];
		}
#pragma unroll
		for (int wd = 0; wd < 16; ++wd)
#pragma unroll
			for (uint32_t j = 0; j < kXU; ++j) {
				const uint32_t nx = wd < 15 ? u[j].r[(wd + 1) >> 2][(wd + 1) & 3] : 0u;
				x[j] = word_step4_next(lds, x[j], nx, c4);
				// after step wd, x = y_(wd+1) ^ word (wd+1): y_4, y_8, y_12
				if (wd == 3 || wd == 7 || wd == 11) Y[j][(wd >> 2)] = x[j] ^ nx;
			}
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) H[j] = wave_scanx(mul_nibbles(lds, x[j], c_lane));
	};
	// the window's points in block kb (two permutes per block for G; the span
	// registers only for points past a span's first chunk -- uniform skip)
	auto capture = [&](uint32_t H, const uint32_t (&Yb)[3], uint32_t Zb, uint32_t kb, bool valid) {
		const bool hs = valid && wbs == kb, he = valid && wbe == kb;
		const uint32_t ts = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((wcs ? wcs - 1 : 0) << 2), (int)H);
		const uint32_t te = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((wce ? wce - 1 : 0) << 2), (int)H);
		Vs = hs ? Zb ^ (wcs ? ts : 0u) : Vs;
		Ve = he ? Zb ^ (wce ? te : 0u) : Ve;
		auto pull = [&](uint32_t cnt, uint32_t qd) -> uint32_t {
			const int a = (int)((cnt & 63u) << 2);
			const uint32_t y1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[0]);
			const uint32_t y2 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[1]);
			const uint32_t y3 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[2]);
			return qd == 1 ? y1 : qd == 2 ? y2 : qd == 3 ? y3 : 0u;
		};
		if (__ballot(hs && wqs)) {
			const uint32_t y = pull(wcs, wqs);
			Ys = hs ? y : Ys;
		}
		if (__ballot(he && wqe)) {
			const uint32_t y = pull(wce, wqe);
			Ye = he ? y : Ye;
		}
	};
	// the registers and points of blocks k .. k + 2U - 1 (those before kend)
	auto finish = [&](const uint32_t (&H)[2 * kXU], const uint32_t (&Y)[2 * kXU][3], uint64_t k, uint64_t kend) {
		uint32_t Z[2 * kXU];
#pragma unroll
		for (uint32_t j = 0; j < 2 * kXU; ++j) {
			Z[j] = mulM(X);
			if (k + j < kend) X = Z[j] ^ rdlane(H[j], 63);
		}
#pragma unroll
		for (uint32_t j = 0; j < 2 * kXU; ++j) capture(H[j], Y[j], Z[j], (uint32_t)(k + j), k + j < kend);
		const uint64_t kn = k + 2 * kXU < kend ? k + 2 * kXU : kend;
		// every buffer of the window ends in the blocks done so far: the next 64
		// (rare for packets of KiBs; these blocks' prefixes are still in
		// registers).  Not past kend: a point in a later block is still to come.
		while ((uint64_t)wlast < kn) {
			flush(q);
			q += 64;
			make_window(q);
			prefetch(q + 64);
#pragma unroll
			for (uint32_t j = 0; j < 2 * kXU; ++j) capture(H[j], Y[j], Z[j], (uint32_t)(k + j), k + j < kend);
		}
	};
	// two units in ping-pong: one computes while the other's loads are in
	// flight (a register copy of a block in flight would wait for its loads)
	for (uint64_t k = k0; k < km; k += 2 * kXU) {
		uint32_t H[2 * kXU], Y[2 * kXU][3];
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) load_blk(u1[j], k + kXU + j);
		__builtin_amdgcn_sched_barrier(0);
		unit_h(u0, reinterpret_cast<uint32_t(&)[kXU]>(H[0]), reinterpret_cast<uint32_t(&)[kXU][3]>(Y[0]));
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) load_blk(u0[j], k + 2 * kXU + j);
		__builtin_amdgcn_sched_barrier(0);
		unit_h(u1, reinterpret_cast<uint32_t(&)[kXU]>(H[kXU]), reinterpret_cast<uint32_t(&)[kXU][3]>(Y[kXU]));
		__builtin_amdgcn_sched_barrier(0);
		finish(H, Y, k, km);
	}
	if (km < k1) {  // the extent's last block: chunks past its end re-read its last chunk (never used)
		const uint64_t last_chunk = G.Eend - 16;
		const uint64_t a = G.S + 4096ull * km + c.ld_off;
#pragma unroll
		for (int q2 = 0; q2 < 4; ++q2) {
			const uint64_t o = a + 2048u * (q2 & 1) + 1024u * (q2 >> 1);
			u0[0].r[q2] = ld16(reinterpret_cast<const uint8_t*>(o <= last_chunk ? o : last_chunk));
		}
		u0[1] = u0[0];
		uint32_t H[2 * kXU], Y[2 * kXU][3];
		unit_h(u0, reinterpret_cast<uint32_t(&)[kXU]>(H[0]), reinterpret_cast<uint32_t(&)[kXU][3]>(Y[0]));
		H[2] = H[3] = 0;
#pragma unroll
		for (uint32_t j = 0; j < 3; ++j) Y[2][j] = Y[3][j] = 0;
		finish(H, Y, km, k1);
	}
	flush(q);
	if (lane == 0) P.x.ragg[w] = X;  // A[w]: the range-local prefix at the range's end
}

// ---------------------------------------------------------------------------
// k_xgrab: the extent as 4 KiB blocks in GRABS of gsz blocks (x_gsz: 8 or
// more), taken dynamically by the waves of a workgroup -- the page kernel's
// load balance (a static share per wave finishes unevenly: the SIMD's issue
// arbitration favours some waves).  A grab is self-contained: its prefix X
// starts at 0 at its first block, its points are captured grab-local from a
// window of buffers starting at wq[g] (the first buffer ending past the
// grab's start, written by k_v7count), and its aggregate X at its end is
// gagg[g]; k_xfin chains the grabs a buffer spans (the range form of
// tests/extent_model.py with per = gsz).
// The grabs [0, ngrab - 1) are full blocks and stream without clamping; the
// last grab, which holds the extent's partial last block, goes first to
// wave 0 of workgroup 0 with clamped chunk addresses.
// ---------------------------------------------------------------------------
#ifdef FDBX_TIMES
// development: per-wave start / end timestamps of k_xgrab (s_memrealtime, 100 MHz)
__device__ uint64_t g_xt[16384][4];
// ... per workgroup of k_xgf: start, stream done, finishing set up, own buffers done, end
__device__ uint64_t g_xft[1024][8];
#endif
// The grab streaming of one workgroup (k_xgrab, and the first phase of
// k_xgf): every grab of its range and, in workgroup 0, the last grab; the
// points and aggregates stored; returns after a barrier once every wave's
// stores have completed and the workgroup's grab counter is back at zero.
// fill: the table loads issued by the caller (in flight while it ran the
// launch checks); lds: the 160 KiB image.
__device__ __forceinline__ void xgrab_stream(const XParams& P, const XGeo G, FillRegs& fill, uint32_t* lds) {
#ifdef FDBX_TIMES
	const uint64_t xt0 = __builtin_amdgcn_s_memrealtime();
	uint32_t xt_grabs = 0;
#endif
	const LaneCtx c = make_ctx();
	const uint32_t lane = (uint32_t)c.lane;
	const uint32_t col4 = (lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (lane >> 5) * 0x4000) | col4;
	const uint32_t wpb = blockDim.x >> 6;
	const uint32_t wi = rdfirst(threadIdx.x >> 6);
	// (32-bit block, grab and buffer numbers: the extent is below 2^40 bytes,
	// the grabs at most kXGrabCap, the route takes batches of < 2^32 buffers)
	const uint32_t nblk = (uint32_t)G.nblk;
	const uint32_t gsz = (uint32_t)x_gsz(nblk, P.x.capg);  // blocks per grab
	const uint32_t ngrab = (nblk + gsz - 1) / gsz;
	const uint32_t spg = gsz / 4;                          // steps of 4 blocks per grab
	const uint32_t nd = ngrab - 1;                         // dynamic grabs [0, nd)
	const uint32_t gper = (nd + gridDim.x - 1) / gridDim.x;
	const uint32_t g0 = blockIdx.x * gper < nd ? blockIdx.x * gper : nd;
	const uint32_t g1 = g0 + gper < nd ? g0 + gper : nd;
	const uint32_t cnt32 = (uint32_t)P.count;
	uint32_t* const my_ctr = P.ctr + kPageCtrWords * blockIdx.x;
	auto clampg = [&](uint32_t g) { return g < g1 ? g : nd; };  // nd: nothing left
	auto request = [&]() -> uint32_t {
		uint32_t r = 0;
		if (lane == 0) r = atomicAdd(my_ctr, 1u);
		return r;
	};
	auto blk_ptr = [&](uint32_t k) { return reinterpret_cast<const uint8_t*>(G.S + 4096ull * k); };
	// a dynamic step's blocks (a step past the wave's grabs re-reads block 0: discarded)
	auto load_step_unit = [&](Block (&u)[kXU], uint32_t g, uint32_t s, uint32_t half) {
		const uint32_t k = g < nd ? g * gsz + 4 * s + 2 * half : 0;
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) load_block(u[j], blk_ptr(k + j), c.ld_off);
	};
	// grab A static (g0 + wi), then one request per grab, issued at its start
	// and read in its first step (k_pages4k: a wave holds at most its grab and
	// the next when the range runs out)
	uint32_t gA = clampg(g0 + wi), gB = nd;
	Block u0[kXU], u1[kXU];
	// wave 0 of workgroup 0 streams the last grab first (below): its first
	// dynamic unit is loaded after that
	const bool lastg = blockIdx.x == 0 && wi == 0;
	if (!lastg && gA < nd) load_step_unit(u0, gA, 0, 0);  // (nd > 0: block 0 is a full block)

	// ---- window of 64 buffers (lane j <-> buffer q + j) ---------------------
	uint32_t q = 0;
	uint32_t wbs, wbe, wcs, wce, wqs, wqe, wlast;
	uint32_t Vs = 0, Ve = 0, Ys = 0, Ye = 0;
	// The next window's buffer, prefetched as the raw offset and length: any
	// arithmetic on them here would wait on the loads at once -- and, the
	// counter being in order, on every block load issued before them.
	uint64_t pf0 = 0, pf1 = 0;
	const uint64_t bS = reinterpret_cast<uint64_t>(P.base) - G.S;
	// (unconditional loads, a strided batch's from the extent start: a load
	// under a branch leaves the wait counter unknown where the paths join)
	auto prefetch = [&](uint32_t q0) {
		const uint32_t j = q0 + lane < cnt32 ? q0 + lane : cnt32 - 1;
		const uint64_t* const dflt = reinterpret_cast<const uint64_t*>(G.S);
		pf0 = xld64(P.offsets ? P.offsets + j : dflt);
		pf1 = xld64(P.lengths ? P.lengths + j : dflt);
	};
	auto make_window = [&](uint32_t q0) {
		const bool ok = q0 + lane < cnt32;
		const uint32_t j = ok ? q0 + lane : cnt32 - 1;
		const uint64_t s = bS + (P.offsets ? pf0 : (uint64_t)j * P.stride), e = s + (P.lengths ? pf1 : P.length);
		wbs = ok ? x_blk(s) : 0xFFFFFFFEu;
		wbe = ok ? x_blk(e) : 0xFFFFFFFEu;
		wcs = x_cnt(s, wbs);
		wce = x_cnt(e, wbe);
		wqs = ((uint32_t)s >> 4) & 3u;
		wqe = ((uint32_t)e >> 4) & 3u;
		wlast = (uint64_t)q0 + 64 <= cnt32 ? rdlane(wbe, 63) : 0xFFFFFFFFu;  // the batch's last window never retires
		Vs = Ve = Ys = Ye = 0;
	};
	// The window's points in blocks [kb0, kb1) leave through a QUEUE of 64
	// point values in the wave's lanes (lane p: point id 2i + end, G, Y),
	// stored only when it fills: a store in the stream loop holds up every
	// later wait on the loads issued behind it (in-order vmcnt), and one store
	// per grab cost ~9 % of the stream (zipf, same-box A/B).  Points move into
	// the queue with ds_permute: the window lanes with a point go to the next
	// free slots in lane order, the others to the remaining lanes (a bijection,
	// so every destination is written once).
	// A second bank holds the previous 64 (a full bank moves there; a store
	// only when both are full): one store per ~128 points.
	uint32_t qid = 0, qv = 0, qy = 0, qn = 0;
	uint32_t bid = 0, bv = 0, by = 0;
	bool bfull = false;
	auto store_bank = [&](uint32_t id, uint32_t v, uint32_t y, uint32_t n) {
		typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
		if (lane < n) *reinterpret_cast<u32x2*>((id & 1 ? P.x.pe : P.x.ps) + 2ull * (id >> 1)) = u32x2{v, y};
	};
	auto store_queue = [&]() {  // bank A is full (or the wave is done)
		if (bfull) store_bank(bid, bv, by, 64);
		bid = qid;
		bv = qv;
		by = qy;
		bfull = qn == 64;
		if (!bfull) store_bank(qid, qv, qy, qn);
		qn = 0;
	};
	auto push = [&](bool on, uint32_t pid, uint32_t v, uint32_t y) {
		const uint64_t m = __ballot(on);
		const uint32_t n = (uint32_t)__builtin_popcountll(m);
		if (n == 0) return;
		const uint32_t below = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
		const uint32_t dst = on ? qn + below : (qn + n + (lane - below)) & 63u;
		const int a = (int)(dst << 2);
		const uint32_t rp = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)pid);
		const uint32_t rv = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)v);
		const uint32_t ry = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)y);
		const bool mine = lane - qn < n;  // (unsigned: lanes qn .. qn + n - 1)
		qid = mine ? rp : qid;
		qv = mine ? rv : qv;
		qy = mine ? ry : qy;
		qn += n;
	};
	auto flush = [&](uint32_t q0, uint32_t kb0, uint32_t kb1) {
		const bool ok = q0 + lane < cnt32;
		const bool os = ok && wbs >= kb0 && wbs < kb1, oe = ok && wbe >= kb0 && wbe < kb1;
		if (qn + (uint32_t)__builtin_popcountll(__ballot(os)) > 64) store_queue();
		push(os, 2 * (q0 + lane), Vs, Ys);
		if (qn + (uint32_t)__builtin_popcountll(__ballot(oe)) > 64) store_queue();
		push(oe, 2 * (q0 + lane) + 1, Ve, Ye);
	};
	auto wq_of = [&](uint32_t g) -> uint32_t { return sld32(P.x.wq + g); };
	if (gA < nd) {
		q = wq_of(gA);
		prefetch(q);
	}

	fill_commit_1024(fill, lds);

	uint32_t X = 0;  // the grab-local prefix at the next block
	auto mulM = [&](uint32_t v) -> uint32_t {  // v * x^(8*4096), uniform (lane tables of lanes 0 and 62)
		const uint32_t n = lane & 7;
		uint32_t t = lds_rd(lds, kS4LaneOff + ((n * 16 + ((v >> (4 * n)) & 15u)) << 7));
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0xB1, 0xF, 0xF, false);
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0x4E, 0xF, 0xF, false);
		t ^= __builtin_amdgcn_update_dpp(0u, t, 0x124, 0xF, 0xF, false);
		t = rdfirst(t);
		uint32_t u = lds_rd(lds, kS4LaneOff + 4 * (4096 + (n * 16 + ((t >> (4 * n)) & 15u)) * 32 + 30));
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0xB1, 0xF, 0xF, false);
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0x4E, 0xF, 0xF, false);
		u ^= __builtin_amdgcn_update_dpp(0u, u, 0x124, 0xF, 0xF, false);
		return rdfirst(u);
	};
	auto unit_h = [&](Block (&u)[kXU], uint32_t (&H)[kXU], uint32_t (&Y)[kXU][3]) {
		uint32_t x[kXU];
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) {
			unswizzle(u[j]);
			x[j] = u[j].r[0][0];
		}
#pragma unroll
		for (int wd = 0; wd < 16; ++wd)
#pragma unroll
			for (uint32_t j = 0; j < kXU; ++j) {
				const uint32_t nx = wd < 15 ? u[j].r[(wd + 1) >> 2][(wd + 1) & 3] : 0u;
				x[j] = word_step4_next(lds, x[j], nx, c4);
				if (wd == 3 || wd == 7 || wd == 11) Y[j][(wd >> 2)] = x[j] ^ nx;
			}
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) H[j] = wave_scanx(mul_nibbles(lds, x[j], c_lane));
	};
	auto capture = [&](uint32_t H, const uint32_t (&Yb)[3], uint32_t Zb, uint32_t kb, bool valid) {
		const bool hs = valid && wbs == kb, he = valid && wbe == kb;
		const uint32_t ts = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((wcs ? wcs - 1 : 0) << 2), (int)H);
		const uint32_t te = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((wce ? wce - 1 : 0) << 2), (int)H);
		Vs = hs ? Zb ^ (wcs ? ts : 0u) : Vs;
		Ve = he ? Zb ^ (wce ? te : 0u) : Ve;
		auto pull = [&](uint32_t cnt, uint32_t qd) -> uint32_t {
			const int a = (int)((cnt & 63u) << 2);
			const uint32_t y1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[0]);
			const uint32_t y2 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[1]);
			const uint32_t y3 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)Yb[2]);
			return qd == 1 ? y1 : qd == 2 ? y2 : qd == 3 ? y3 : 0u;
		};
		if (__ballot(hs && wqs)) {
			const uint32_t y = pull(wcs, wqs);
			Ys = hs ? y : Ys;
		}
		if (__ballot(he && wqe)) {
			const uint32_t y = pull(wce, wqe);
			Ye = he ? y : Ye;
		}
	};
	// the unit of blocks k, k + 1 of grab [gb0, gb1) (those before kend): the
	// prefix chain, the points, windows retired inside the grab.  Per unit, so
	// only one unit's H and Y are live: a window retired here can only hold
	// points in this unit's blocks or later (its buffers start after the
	// previous window's last end, which lies in this unit or later).
	auto finish = [&](const uint32_t (&H)[kXU], const uint32_t (&Y)[kXU][3], uint32_t k, uint32_t kend, uint32_t gb0,
	                  uint32_t gb1) {
		uint32_t Z[kXU];
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) {
			Z[j] = mulM(X);
			if (k + j < kend) X = Z[j] ^ rdlane(H[j], 63);
		}
#pragma unroll
		for (uint32_t j = 0; j < kXU; ++j) capture(H[j], Y[j], Z[j], k + j, k + j < kend);
		const uint32_t kn = k + kXU < kend ? k + kXU : kend;
		auto retire = [&]() {  // every buffer of the window ends in the blocks so far: the next 64
			flush(q, gb0, gb1);
			q += 64;
			make_window(q);
			prefetch(q + 64);
#pragma unroll
			for (uint32_t j = 0; j < kXU; ++j) capture(H[j], Y[j], Z[j], k + j, k + j < kend);
		};
		// (the first retirement peeled: a loop's wait on the window loads would
		// assume they were just issued, and drain the next unit's block loads)
		if (wlast < kn) {
			retire();
			while (wlast < kn) retire();
		}
	};

	// ---- the last grab (partial last block): clamped loads, no pipelining ----
	if (lastg) {
		const uint32_t gb0 = nd * gsz, gb1 = nblk;
		const uint64_t last_chunk = G.Eend - 16;
		const uint32_t ql = wq_of(nd);
		prefetch(ql);
		make_window(ql);
		q = ql;
		prefetch(q + 64);
		X = 0;
		for (uint32_t s = 0; s < spg && gb0 + 4 * s < nblk; ++s) {
#pragma unroll
			for (uint32_t h = 0; h < 2; ++h) {
				uint32_t H[kXU], Y[kXU][3];
#pragma unroll
				for (uint32_t j = 0; j < kXU; ++j) {
					const uint64_t a = G.S + 4096ull * (gb0 + 4 * s + 2 * h + j) + c.ld_off;
#pragma unroll
					for (int q2 = 0; q2 < 4; ++q2) {
						const uint64_t o = a + 2048u * (q2 & 1) + 1024u * (q2 >> 1);
						u1[j].r[q2] = ld16(reinterpret_cast<const uint8_t*>(o <= last_chunk ? o : last_chunk));
					}
				}
				unit_h(u1, H, Y);
				finish(H, Y, gb0 + 4 * s + 2 * h, gb1, gb0, gb1);
			}
		}
		flush(q, gb0, gb1);
		if (lane == 0) P.x.gagg[nd] = X;
		// back to this wave's first dynamic grab
		if (gA < nd) {
			q = wq_of(gA);
			prefetch(q);
			load_step_unit(u0, gA, 0, 0);
		}
	}

	// ---- dynamic grabs: steps of 4 blocks, two units in ping-pong ----------
	uint32_t s = 0;
	uint32_t wqv = 0;
	while (gA < nd) {
		const uint32_t gb0 = gA * gsz, gb1 = gb0 + gsz;
		const uint32_t k = gb0 + 4 * s;
		uint32_t qnx = 0;
		uint32_t req = 0;
		if (s == 0) {
			X = 0;
			req = request();
		}
		load_step_unit(u1, gA, s, 1);
		__builtin_amdgcn_sched_barrier(0);
		{
			uint32_t H[kXU], Y[kXU][3];
			unit_h(u0, H, Y);
			__builtin_amdgcn_sched_barrier(0);
			const bool last_step = s + 1 == spg;  // (not step 0: a grab has at least two)
			qnx = last_step ? wqv : 0u;
			// the grab's window (its metadata prefetched a grab ahead; the next
			// window's loads issued ahead of the next unit's, so that a window
			// retired in this unit waits only for them); the next grab and its
			// window start (read at this grab's end)
			if (s == 0) {
				make_window(q);
				prefetch(q + 64);
				gB = clampg(g0 + wpb + rdlane(req, 0));
				wqv = sld32(P.x.wq + (gB < nd ? gB : 0u));
			}
			// the next unit's loads go out before this unit's points are captured
			load_step_unit(u0, last_step ? gB : gA, last_step ? 0u : s + 1, 0);
			__builtin_amdgcn_sched_barrier(0);
			finish(H, Y, k, gb1, gb0, gb1);
		}
		const bool last_step = s + 1 == spg;
		__builtin_amdgcn_sched_barrier(0);
		{
			uint32_t H[kXU], Y[kXU][3];
			unit_h(u1, H, Y);
			__builtin_amdgcn_sched_barrier(0);
			finish(H, Y, k + kXU, gb1, gb0, gb1);
		}
		if (last_step) {
#ifdef FDBX_TIMES
			++xt_grabs;
#endif
			flush(q, gb0, gb1);
			if (lane == 0) P.x.gagg[gA] = X;
			q = qnx;
			if (gB < nd) prefetch(q);  // the next grab's window, consumed a step later
			gA = gB;
			s = 0;
		} else {
			++s;
		}
	}
	if (bfull) store_bank(bid, bv, by, 64);
	store_bank(qid, qv, qy, qn);
#ifdef FDBX_TIMES
	if (lane == 0) {
		const uint32_t w = blockIdx.x * wpb + wi;
		g_xt[w][0] = xt0;
		g_xt[w][1] = __builtin_amdgcn_s_memrealtime();
		g_xt[w][2] = xt_grabs;
		g_xt[w][3] = g1 - g0;
	}
#endif
	// every request of every wave has returned: the counter goes back to zero
	__builtin_amdgcn_s_waitcnt(0);
	__syncthreads();
	if (threadIdx.x == 0) *my_ctr = 0;
}

__global__ __launch_bounds__(1024) void k_xgrab(XParams P) {
	// (the table loads first: vector loads, in flight while the checks' scalar
	// loads return)
	FillRegs fill;
	fill_issue_1024(fill, P.tabs);
	const XStart X0 = x_start(P);
	if (!X0.packed) return;  // k_xfin checksums this batch buffer by buffer
	if (X0.G.nblk == 0) return;  // every buffer empty at one 16-byte-aligned address: k_xfin alone
	__shared__ uint32_t lds[kLdsBytesB / 4];
	xgrab_stream(P, X0.G, fill, lds);
}

// ---------------------------------------------------------------------------
// v * M^m for 0 <= m < 2^32 blocks (bpow: x^(8*4096*j*256^i)); the levels no
// lane needs are skipped.
__device__ __forceinline__ uint32_t xmul_blocks(const DevTables* T, uint32_t v, uint32_t m) {
	v = xmul(T->bpow[0][m & 255u], v);
	if (__ballot(m >> 8)) v = xmul(T->bpow[1][(m >> 8) & 255u], v);
	if (__ballot(m >> 16)) v = xmul(T->bpow[2][(m >> 16) & 255u], v);
	if (__ballot(m >> 24)) v = xmul(T->bpow[3][m >> 24], v);
	return v;
}

// ---------------------------------------------------------------------------
// k_xfin: one buffer per thread, persistent (one 1024-thread workgroup per
// CU).  The constant multiplies run from LDS copies of the nibble tables the
// finishing math uses (x^(-8*64j), x^(8d), x^(8*64c), M^j for j < 64, and the
// slicing tables): two dependent global round trips per buffer (metadata,
// then the point registers and remainder bytes) instead of one per multiply.
// ---------------------------------------------------------------------------
constexpr uint32_t kFinThreads = 1024;
constexpr uint32_t kFinXinv = 0;                        // xinv64[65]  } in DevTables' order: one
constexpr uint32_t kFinPow64 = kFinXinv + 65 * 128;     // pow64[64]   } contiguous copy
constexpr uint32_t kFinPow1 = kFinPow64 + 64 * 128;     // pow1[64]    }
constexpr uint32_t kFinBp0 = kFinPow1 + 64 * 128;       // bpow[0][0..63]
constexpr uint32_t kFinS4 = kFinBp0 + 64 * 128;         // slice4[4][256]
constexpr uint32_t kFinC = kFinS4 + 4 * 256;            // M^per (built per launch)
constexpr uint32_t kFinWords = kFinC + 128;             // 34048 words = 133 KiB
static_assert(offsetof(DevTables, pow64) == offsetof(DevTables, xinv64) + sizeof(uint32_t) * 65 * 128 &&
                  offsetof(DevTables, pow1) == offsetof(DevTables, pow64) + sizeof(uint32_t) * 64 * 128,
              "xinv64, pow64, pow1 are contiguous");

__device__ __forceinline__ uint32_t lmul(const uint32_t* lds, uint32_t tab, uint32_t v) {
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= lds[tab + 16 * n + ((v >> (4 * n)) & 15u)];
	return r;
}

// The finishing kernel's LDS tables: every 16-byte load of the three copies
// issued before any LDS write (clamped addresses, so no load sits behind a
// branch), one L2 round trip instead of one per copy-loop iteration.
__device__ __forceinline__ void fin_fill(uint32_t* lds, const DevTables* T) {
	typedef __attribute__((address_space(1))) const u32x4 gq;
	constexpr uint32_t NA = 193 * 32, NB = 64 * 32, NC = 256;  // quads: xinv64..pow1, bpow[0][0..63], slice4
	constexpr uint32_t IA = (NA + kFinThreads - 1) / kFinThreads, IB = NB / kFinThreads;
	static_assert(NB % kFinThreads == 0 && NC <= kFinThreads, "copy shapes");
	const gq* sa = (const gq*)reinterpret_cast<uintptr_t>(&T->xinv64[0][0][0]);
	const gq* sb = (const gq*)reinterpret_cast<uintptr_t>(&T->bpow[0][0][0][0]);
	const gq* sc = (const gq*)reinterpret_cast<uintptr_t>(&T->slice4[0][0]);
	const uint32_t t = threadIdx.x;
	u32x4 a[IA], b[IB], c;
#pragma unroll
	for (uint32_t i = 0; i < IA; ++i) {
		const uint32_t q = t + kFinThreads * i;
		a[i] = sa[q < NA ? q : NA - 1];
	}
#pragma unroll
	for (uint32_t i = 0; i < IB; ++i) b[i] = sb[t + kFinThreads * i];
	c = sc[t < NC ? t : NC - 1];
	u32x4* d = reinterpret_cast<u32x4*>(lds);
#pragma unroll
	for (uint32_t i = 0; i < IA; ++i)
		if (t + kFinThreads * i < NA) d[kFinXinv / 4 + t + kFinThreads * i] = a[i];
#pragma unroll
	for (uint32_t i = 0; i < IB; ++i) d[kFinBp0 / 4 + t + kFinThreads * i] = b[i];
	if (t < NC) d[kFinS4 / 4 + t] = c;
}

// GF(2) product of two registers (reflected CRC-32C polynomial), bit by bit.
__device__ __forceinline__ uint32_t gf2mul(uint32_t a, uint32_t b) {
	uint32_t r = 0;
	for (int q = 0; q < 32; ++q) {
		r ^= (a & 0x80000000u) ? b : 0u;
		a <<= 1;
		b = (b & 1u) ? (b >> 1) ^ 0x82f63b78u : (b >> 1);
	}
	return r;
}
// x^(8n) for any n < 2^64 (pow2 nibble tables: x^(8*2^m)).
__device__ __forceinline__ uint32_t xpow8_any(const DevTables* T, uint64_t n) {
	uint32_t v = 0x80000000u;
	for (int m = 0; n; ++m, n >>= 1)
		if (n & 1) v = xmul(T->pow2[m], v);
	return v;
}

// The batch failed the packing check (k_v7count): every buffer is
// checksummed directly -- crc32c_append's register loop
// (contrib/crc32/crc32c.cpp:346-356) with 4-byte slicing from LDS, 16-byte
// loads -- and the stream's next kXfailBackoff (16) batches take the window
// engine (kHstatXfail counts them down; then the extent route is tried again).  Buffers under 4 KiB: one lane each.  Longer ones: one wave
// each, the 64 lanes on 64 equal parts aligned to the buffer's END (parts
// before the buffer's start are empty -- leading zeros are free -- and the
// lane whose part holds P0 starts from ~seed there), joined by a 6-level tree
// where a left group takes x^(8 * d * part) (uniform per level, squared from
// level to level): a 200 MiB buffer takes ~10 ms instead of ~0.2 s.
__device__ void x_fallback(const XParams& P, const uint32_t* s4) {
	auto word = [&](uint32_t& r, uint32_t w) {
		r ^= w;
		r = s4[r & 255u] ^ s4[256 + ((r >> 8) & 255u)] ^ s4[512 + ((r >> 16) & 255u)] ^ s4[768 + (r >> 24)];
	};
	auto byte = [&](uint32_t& r, uint64_t a) {
		r = (r >> 8) ^ s4[768 + ((r ^ ld1(reinterpret_cast<const uint8_t*>(a))) & 255u)];
	};
	// raw register of bytes [a, b) fed into r
	auto run = [&](uint32_t r, uint64_t a, uint64_t b) -> uint32_t {
		for (; a < b && (a & 15); ++a) byte(r, a);
		for (; a + 16 <= b; a += 16) {
			const u32x4 v = ld16(reinterpret_cast<const uint8_t*>(a));
			word(r, v[0]);
			word(r, v[1]);
			word(r, v[2]);
			word(r, v[3]);
		}
		for (; a < b; ++a) byte(r, a);
		return r;
	};
	constexpr uint64_t kWaveMin = 4096;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P.count;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t P0, P1;
		x_buffer(P, i, P0, P1);
		if (P1 - P0 >= kWaveMin) continue;
		const uint32_t sd = P.seeds ? xld32(P.seeds + i) : P.seed;
		P.out[i] = ~run(~sd, P0, P1);
	}
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rdfirst(threadIdx.x >> 6); i < P.count; i += nw) {
		uint64_t P0, P1;
		x_buffer(P, i, P0, P1);
		P0 = rdfirst64(P0);
		P1 = rdfirst64(P1);
		if (P1 - P0 < kWaveMin) continue;
		const uint32_t sd = rdfirst(P.seeds ? xld32(P.seeds + i) : P.seed);
		const uint64_t part = ((P1 - P0) + 63) / 64;
		const uint64_t hi = P1 - (63 - lane) * part;               // this lane's part: [hi - part, hi)
		const uint64_t lo = hi - part;
		const uint64_t a = lo > P0 ? lo : P0;  // parts before P0 are empty; the one holding P0 starts there
		uint32_t r = hi > P0 ? run(a == P0 ? ~sd : 0u, a, hi) : 0u;
		uint32_t S = xpow8_any(P.tabs, part);  // x^(8 * d * part) at level d
		for (uint32_t d = 1; d < 64; d <<= 1) {
			const uint32_t right = (uint32_t)__shfl_down((int)r, d);
			r = (lane % (2 * d) == 0) ? gf2mul(r, S) ^ right : r;
			S = gf2mul(S, S);
		}
		if (lane == 0) P.out[i] = ~r;
	}
}

// A buffer spanning more than kFinLongChain units (grabs) is not chained by
// its own lane (one dependent table multiply per unit: a 300 MiB buffer on
// 8-block grabs is 9600 of them, ~1 ms of one lane) but by its whole wave,
// inside the pass (a uniform loop over the wave's long buffers): lane j
// chains a 64th of the aggregates, weights its part by C^(units after it) =
// M^(per * units), and the parts XOR-reduce (the aggregate chain is linear).
constexpr uint32_t kFinLongChain = 64;
// The aggregates of units [ws, we) chained by the wave (D = sum of agg[v] *
// C^(we - 1 - v)): lane j Horner-combines units [ws + j*sl, ws + (j+1)*sl)
// and carries its part past the units after it, * C^(we - its end) =
// M^(per * units); the parts XOR-reduce.
__device__ __forceinline__ uint32_t wave_chain(const uint32_t* agg, const uint32_t* lds, uint32_t cbase,
                                                        const DevTables* T, uint64_t per, uint64_t ws, uint64_t we,
                                                        uint32_t lane) {
	const uint64_t n = we - ws, sl = (n + 63) / 64;
	const uint64_t v0 = ws + lane * sl < we ? ws + lane * sl : we;
	const uint64_t v1 = v0 + sl < we ? v0 + sl : we;
	uint32_t part = 0;
	for (uint64_t v = v0; v < v1; v += 4) {  // four aggregates per round trip (eight: an SGPR spill)
		uint32_t a[4];
#pragma unroll
		for (uint32_t t = 0; t < 4; ++t) a[t] = xld32(agg + (v + t < v1 ? v + t : v1 - 1));
#pragma unroll
		for (uint32_t t = 0; t < 4; ++t)
			if (v + t < v1) part = lmul(lds, cbase, part) ^ a[t];
	}
	const uint64_t after = we - v1;
	if (after && v1 > v0) part = xmul_blocks(T, part, (uint32_t)(per * after));
#pragma unroll
	for (int d = 32; d >= 1; d >>= 1) part ^= (uint32_t)__shfl_xor((int)part, d);
	return part;
}

// The finishing pass's setup (k_xfin, and the second phase of k_xgf): its
// LDS tables and the chained units' geometry.  Ends with a barrier.
struct XFin {
	uint64_t per;         // blocks per chained unit (grab or static range)
	uint32_t lgp;         // log2(per) for grabs (a power of two), else 64
	uint32_t cbase;       // LDS nibble tables of C = M^per
	const uint32_t* agg;  // the units' aggregates
};
__device__ __forceinline__ XFin xfin_setup(const XParams& P, uint32_t* lds, const XGeo& G) {
	const DevTables* T = P.tabs;
	XFin F;
	// the chained units: k_xgrab's grabs or k_xstream's static ranges
	F.per = P.grabs ? x_gsz(G.nblk, P.x.capg) : x_per(G.nblk, P.nwave);
	F.lgp = P.grabs ? x_log2(F.per) : 64u;  // grabs: a power of two
	F.agg = P.grabs ? P.x.gagg : P.x.ragg;
	fin_fill(lds, T);
	// nibble tables of C = M^per (the unit stride), for the straddling
	// buffers' aggregate chains: entry [n][v] = (v x^4n) * C, bit by bit --
	// except for grabs of fewer than 64 blocks, whose M^gsz is one of the
	// block-power tables already copied (no build, no barrier wait on it)
	F.cbase = F.per < 64 ? kFinBp0 + 128 * (uint32_t)F.per : kFinC;
	if (F.per >= 64 && threadIdx.x < 128) {
		const uint32_t C = xmul_blocks(T, 0x80000000u, (uint32_t)F.per);
		uint32_t a = (threadIdx.x & 15u) << (4 * (threadIdx.x >> 4)), b = C, r = 0;
		for (int q = 0; q < 32; ++q) {
			r ^= (a & 0x80000000u) ? b : 0u;
			a <<= 1;
			b = (b & 1u) ? (b >> 1) ^ 0x82f63b78u : (b >> 1);
		}
		lds[kFinC + threadIdx.x] = r;
	}
	__syncthreads();
	return F;
}

// Finish the buffers idx(j), j in [0, n): thread t takes j = start + t +
// 2*stride*k and j + stride (two buffers per pass, their loads issued
// together).  k_xfin: the whole batch over the grid; k_xgf: a workgroup's own
// buffers, then its share of the buffers spanning several workgroups' grabs.
template <class Idx>
__device__ __forceinline__ void xfin_buffers(const XParams& P, const uint32_t* lds, const XGeo& G, const XFin& F,
                                             uint64_t n, uint64_t start, uint64_t stride, Idx idx) {
	const DevTables* T = P.tabs;
	const uint64_t per = F.per;
	const uint32_t lgp = F.lgp, cbase = F.cbase;
	const uint32_t* const agg = F.agg;
	const uint32_t* s4 = lds + kFinS4;
	typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
	typedef __attribute__((address_space(1))) const u32x2 xg_u2;
	// Two buffers per thread per pass, their loads issued together: the pass
	// is a chain of dependent round trips (metadata and point values, then the
	// points' chunks), so two in flight halve the passes (zipf: 17.9 -> 16.7 us).
	struct In {
		u32x2 cs, ce;
		uint64_t P0, P1;
		uint64_t ws, we;  // the units holding its start and end (set by units())
		uint64_t i;       // the buffer
		uint32_t sd;
		bool ok;
	};
	auto load_in = [&](In& I, uint64_t j) {
		// (idx may return ~0: no buffer at j -- k_xshared's empty candidates)
		const uint64_t ix = j < n ? idx(j) : ~0ull;
		I.ok = ix < P.count;
		const uint64_t ic = I.ok ? ix : 0;
		I.i = ic;
		// the captured point values do not depend on the metadata
		I.cs = *((xg_u2*)reinterpret_cast<uintptr_t>(P.x.ps + 2 * ic));
		I.ce = *((xg_u2*)reinterpret_cast<uintptr_t>(P.x.pe + 2 * ic));
		x_buffer(P, ic, I.P0, I.P1);
		I.sd = P.seeds ? xld32(P.seeds + ic) : P.seed;
	};
	// R(p): the prefix register at point p (0 at p = 0).  p = 4096k + 64 cnt
	// + 16 cq + r: G(p) back to p64, on by 16 cq bytes plus Y (the span's
	// register after its first cq chunks), then the r < 16 bytes of the
	// chunk at p - r.
	auto R = [&](uint64_t p, uint32_t g, uint32_t y) -> uint32_t {
		const uint32_t k = x_blk(p);
		const uint32_t cnt = x_cnt(p, k);
		const uint32_t rem = (uint32_t)(p - 4096ull * k) & 63u;  // (cnt = 64: rem 0)
		const uint32_t cq = rem >> 4, r16 = rem & 15u;
		uint32_t r = lmul(lds, kFinXinv + 128 * (64 - cnt), g);
		r = cq ? lmul(lds, kFinPow1 + 128 * (16 * cq), r) ^ y : r;
		r = p ? r : 0u;
		if (r16) {  // (a divergent load: unconditional chunk loads for every point cost ~10 us on zipf)
			const u32x4 ch = ld16(reinterpret_cast<const uint8_t*>(G.S + p - r16));
#pragma unroll
			for (uint32_t t = 0; t < 3; ++t) {
				if (4 * t + 4 <= r16) {
					r ^= ch[t];
					r = s4[r & 255u] ^ s4[256 + ((r >> 8) & 255u)] ^ s4[512 + ((r >> 16) & 255u)] ^ s4[768 + (r >> 24)];
				}
			}
			const uint32_t wd = r16 >> 2, nb = r16 & 3u;
			const uint32_t word = wd == 0 ? ch[0] : wd == 1 ? ch[1] : wd == 2 ? ch[2] : ch[3];
			for (uint32_t b = 0; b < nb; ++b) r = (r >> 8) ^ s4[768 + ((r ^ (word >> (8 * b))) & 255u)];
		}
		return r;
	};
	// A buffer spanning units ws < we: the end point takes the aggregates of
	// the units from ws to we - 1 (the start point's unit start is the origin)
	// (a lane past the list holds a clamped copy of its last buffer: it chains
	// nothing -- its result is discarded, and a huge last buffer's chain run by
	// every idle lane of the grid took 14 ms for one 1.1 GB buffer)
	auto units = [&](In& I) {
		const uint32_t ks = x_blk(I.P0 - G.S), ke = x_blk(I.P1 - G.S);
		I.ws = lgp < 64 ? ks >> lgp : ks / per;
		I.we = !I.ok ? I.ws : (lgp < 64 ? ke >> lgp : ke / per);
	};
	// Dq (long chains): the aggregate chain, computed by the wave
	auto finish = [&](const In& I, bool queued, uint32_t Dq) -> uint32_t {
		const uint64_t sp = I.P0 - G.S, ep = I.P1 - G.S;
		const uint32_t ke = x_blk(ep);
		// G(p): the unit-local prefix at p64, positioned at its block's end
		uint32_t ge = I.ce[0];
		const uint64_t ws = I.ws, we = I.we;
		if (ws != we) {
			uint32_t D = Dq;
			for (uint64_t v = ws; !queued && v < we; v += 8) {  // eight aggregates in flight per round trip
				uint32_t a[8];
#pragma unroll
				for (uint32_t t = 0; t < 8; ++t) a[t] = xld32(agg + (v + t < we ? v + t : we - 1));
#pragma unroll
				for (uint32_t t = 0; t < 8; ++t)
					if (v + t < we) D = lmul(lds, cbase, D) ^ a[t];
			}
			const uint32_t j = (uint32_t)(ke - we * per + 1);
			ge ^= j < 64 ? lmul(lds, kFinBp0 + 128 * j, D) : xmul_blocks(T, D, j);
		}
		const uint32_t re = R(ep, ge, I.ce[1]);
		uint32_t rs = R(sp, I.cs[0], I.cs[1]) ^ ~I.sd;
		// rs * x^(8 len), len = 4096a + 64c + d
		const uint64_t len = I.P1 - I.P0;
		rs = lmul(lds, kFinPow1 + 128 * (uint32_t)(len & 63u), rs);
		rs = lmul(lds, kFinPow64 + 128 * (uint32_t)((len >> 6) & 63u), rs);
		const uint64_t nbk = len >> 12;
		if (nbk >= 64)
			rs = xmul_blocks(T, rs, (uint32_t)nbk);
		else if (nbk)
			rs = lmul(lds, kFinBp0 + 128 * (uint32_t)nbk, rs);
		return ~(re ^ rs);
	};
	// Long chains (more than kFinLongChain units) are chained by the whole
	// wave, one buffer at a time (uniform loop over the ballot), and the
	// owning lane finishes with that D.
	auto long_chains = [&](In& I, uint32_t& D) -> bool {
		units(I);
		const bool lg = I.ok && I.we - I.ws > kFinLongChain;
		uint64_t m = __ballot(lg);
		D = 0;
		while (m) {
			const int j = __builtin_ctzll(m);
			m &= m - 1;
			const uint64_t ws = rdlane64(I.ws, j), we = rdlane64(I.we, j);
			const uint32_t d = wave_chain(agg, lds, cbase, T, per, ws, we, threadIdx.x & 63);
			D = (int)(threadIdx.x & 63) == j ? d : D;
		}
		return lg;
	};
	for (uint64_t j0 = start; j0 < n; j0 += 2 * stride) {
		In A, B;
		load_in(A, j0 + threadIdx.x);
		load_in(B, j0 + stride + threadIdx.x);
		uint32_t Da, Db;
		const bool la = long_chains(A, Da), lb = long_chains(B, Db);
		const uint32_t ra = finish(A, la, Da);
		const uint32_t rb = finish(B, lb, Db);
		if (A.ok) P.out[A.i] = ra;
		if (B.ok) P.out[B.i] = rb;
	}
}

// The stream's next route choice: the count kernel's statistics (staged in
// xhdr, kXStage) and this batch's back-off word (one thread).
__device__ __forceinline__ void x_publish_stats(const XParams& P) {
	const uint64_t* st = reinterpret_cast<const uint64_t*>(P.x.xhdr) + kXStage;
	uint64_t v[kHstatPacked + 1];
#pragma unroll
	for (int k = 0; k <= kHstatPacked; ++k) v[k] = st[k];
#pragma unroll
	for (int k = 0; k <= kHstatPacked; ++k) P.hstat[k] = v[k];
	P.hstat[kHstatXfail] = x_unordered(P) ? kXfailBackoff : 0;
}

// A batch that failed the packing check (x_fallback, slicing tables in LDS),
// or whose buffers are all empty at one 16-byte-aligned address
// (crc32c_append(seed, p, 0) == seed).
__device__ __forceinline__ void x_unpacked(const XParams& P, uint32_t* lds) {
	for (uint32_t k = threadIdx.x; k < 1024; k += blockDim.x) lds[kFinS4 + k] = xld32(&P.tabs->slice4[0][0] + k);
	__syncthreads();
	x_fallback(P, lds + kFinS4);
}
__device__ __forceinline__ void x_all_empty(const XParams& P) {
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P.count; i += (uint64_t)gridDim.x * blockDim.x)
		P.out[i] = P.seeds ? xld32(P.seeds + i) : P.seed;
}

__global__ __launch_bounds__(kFinThreads) void k_xfin(XParams P) {
	__shared__ uint32_t lds[kFinWords];
	const bool packed = x_packed(P);
	if (blockIdx.x == 0 && threadIdx.x == 0 && P.hstat) x_publish_stats(P);
	if (!packed) {
		x_unpacked(P, lds);
		return;
	}
	// (x_start's one-round-trip form here holds the kernel's arguments in
	// SGPRs across the pass: 5 SGPR spills)
	const XGeo G = x_geo(P);
	if (G.nblk == 0) {
		x_all_empty(P);
		return;
	}
	const XFin F = xfin_setup(P, lds, G);
	xfin_buffers(P, lds, G, F, P.count, (uint64_t)blockIdx.x * blockDim.x, (uint64_t)gridDim.x * blockDim.x,
	             [](uint64_t j) { return j; });
}

// ---------------------------------------------------------------------------
// k_xgf: the grab stream and the finishing pass in one kernel.  Grid: one
// 1024-thread workgroup per CU, as k_xgrab.  A workgroup that has streamed
// its grabs (all its waves' points and aggregates stored) reloads its LDS with
// the finishing tables and finishes the buffers whose END lies in its grabs
// and whose start lies in them too -- those need nothing any other workgroup
// wrote -- while other workgroups are still streaming (their stream ends
// spread over ~30-50 us).  A buffer whose grabs belong to several workgroups
// (the first buffer of a range when it starts in the range before, and the
// first buffer of the extent's last grab, which workgroup 0 streams, when it
// starts before that grab: at most one per workgroup) is left to k_xshared,
// launched next, which finds the same buffers from the grab map and finishes
// them after the kernel boundary has made every workgroup's stores visible.
// (Finishing them in k_xgf behind per-workgroup flags measured ~60 us slower:
// the agent-scope release / acquire each workgroup needs writes back and
// invalidates its XCD's whole L2 while the other workgroups stream; by the
// last workgroup to arrive, after a release per workgroup, ~5-15 us slower.
// tools/probe_xftimes.py.)  Not the default: the own pass (~2.5 us of table
// fill, ~7.5 us of finishing) lands on every workgroup's stream end, the
// latest included, and k_xshared's chain of round trips costs ~13 us, so the
// pair measured 0.2459-0.2470 ms per zipf step against k_xgrab + k_xfin's
// 0.2326-0.2336 ms (same box).
// ---------------------------------------------------------------------------
static_assert(kFinWords + 16 <= kLdsBytesB / 4, "the finishing tables fit in the stream's LDS image");

// The grab partition of k_xgf's grid (xgrab_stream's): grabs [g0, g1) of
// workgroup b, the last grab nd streamed by workgroup 0.
struct XParts {
	uint32_t lgp, nd, gper;
	__device__ __forceinline__ XParts(const XParams& P, const XGeo& G) {
		const uint32_t nblk = (uint32_t)G.nblk;
		const uint32_t gsz = (uint32_t)x_gsz(nblk, P.x.capg);
		lgp = x_log2(gsz);
		nd = (nblk + gsz - 1) / gsz - 1;
		gper = (nd + (uint32_t)P.ngrid - 1) / (uint32_t)P.ngrid;
	}
	__device__ __forceinline__ void range(uint32_t b, uint32_t& g0, uint32_t& g1) const {
		g0 = b * gper < nd ? b * gper : nd;
		g1 = g0 + gper < nd ? g0 + gper : nd;
	}
	__device__ __forceinline__ uint32_t grab(uint64_t p) const { return x_blk(p) >> lgp; }  // p: bytes from S
	__device__ __forceinline__ uint32_t owner(uint32_t g) const { return g >= nd ? 0u : g / gper; }
};
__device__ __forceinline__ uint32_t x_start_grab(const XParams& P, const XGeo& G, const XParts& X, uint32_t i) {
	uint64_t a, b;
	x_buffer(P, i, a, b);
	return X.grab(a - G.S);
}
// The shared buffer of workgroup b (b < ngrid: the first buffer of its range
// when it starts in an earlier workgroup's grabs) or of the last grab (b ==
// ngrid: its first buffer when it starts before it), else ~0.  k_xgf's own
// passes leave exactly these out.
__device__ __forceinline__ uint64_t x_shared_of(const XParams& P, const XGeo& G, const XParts& X, uint32_t b) {
	const uint32_t cnt32 = (uint32_t)P.count;
	if (b < (uint32_t)P.ngrid) {
		uint32_t g0, g1;
		X.range(b, g0, g1);
		if (g0 == 0 || g0 >= g1) return ~0ull;
		const uint32_t lo = xld32(P.x.wq + g0), hi = xld32(P.x.wq + g1);
		return lo < hi && X.owner(x_start_grab(P, G, X, lo)) != b ? lo : ~0ull;
	}
	if (X.nd == 0) return ~0ull;
	const uint32_t c = xld32(P.x.wq + X.nd);
	return c < cnt32 && x_start_grab(P, G, X, c) < X.nd ? c : ~0ull;
}

// The finishing phase of k_xgf (below): this workgroup's own buffers.
__device__ __forceinline__ void xgf_finish(const XParams& P, const XGeo& G, uint32_t* lds) {
	const XParts X(P, G);
	uint32_t g0, g1;
	X.range(blockIdx.x, g0, g1);
	const uint32_t cnt32 = (uint32_t)P.count;
#ifdef FDBX_TIMES
	if (threadIdx.x == 0) g_xft[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
	// the buffers whose end lies in this workgroup's grabs, [lo, hi) (wq[g]:
	// the first buffer ending past grab g's start; buffer 0 may end at the
	// extent's start), less the first when it starts in an earlier
	// workgroup's grabs; in workgroup 0 also the last grab's [wq[nd], count),
	// less its first when it starts before that grab
	const uint32_t lo = g0 == 0 ? 0u : rdfirst(xld32(P.x.wq + g0));
	const uint32_t hi = g0 < g1 ? rdfirst(xld32(P.x.wq + g1)) : lo;
	const bool sh1 = lo < hi && g0 != 0 && X.owner(x_start_grab(P, G, X, lo)) != blockIdx.x;
	const uint32_t a0 = lo + (sh1 ? 1u : 0u);
	uint32_t b0 = cnt32;
	if (blockIdx.x == 0) {
		const uint32_t c = X.nd == 0 ? 0u : rdfirst(xld32(P.x.wq + X.nd));
		b0 = c + (c < cnt32 && X.nd != 0 && x_start_grab(P, G, X, c) < X.nd ? 1u : 0u);
	}
	const XFin F = xfin_setup(P, lds, G);
#ifdef FDBX_TIMES
	if (threadIdx.x == 0) g_xft[blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
#endif
	xfin_buffers(P, lds, G, F, hi > a0 ? hi - a0 : 0u, 0, blockDim.x, [&](uint64_t j) { return a0 + j; });
	if (blockIdx.x == 0)
		xfin_buffers(P, lds, G, F, cnt32 > b0 ? cnt32 - b0 : 0u, 0, blockDim.x, [&](uint64_t j) { return b0 + j; });
#ifdef FDBX_TIMES
	if (threadIdx.x == 0) g_xft[blockIdx.x][3] = g_xft[blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();
#endif
}

__global__ __launch_bounds__(1024) void k_xgf(XParams P) {
#ifdef FDBX_TIMES
	if (threadIdx.x == 0) g_xft[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
#endif
	__shared__ uint32_t lds[kLdsBytesB / 4];  // the stream's image, then the finishing tables
	FillRegs fill;
	fill_issue_1024(fill, P.tabs);
	const XStart X0 = x_start(P);
	if (blockIdx.x == 0 && threadIdx.x == 0 && P.hstat) x_publish_stats(P);
	if (!X0.packed) {
		x_unpacked(P, lds);
		return;
	}
	if (X0.G.nblk == 0) {
		x_all_empty(P);
		return;
	}
	xgrab_stream(P, X0.G, fill, lds);
	// The finishing phase reads its arguments again from the kernarg segment
	// through an opaque pointer, so nothing it needs but the stream's own
	// values is held in registers across the stream (held, they spilled: 85
	// SGPRs into VGPR lanes, and a VGPR to scratch inside the grab loop).
#if defined(__HIP_DEVICE_COMPILE__)
	typedef __attribute__((address_space(4))) const XParams KParams;
	KParams* kp = (KParams*)(__builtin_amdgcn_kernarg_segment_ptr());
	asm volatile("" : "+s"(kp));
	XParams P2;
	__builtin_memcpy(&P2, (const XParams*)kp, sizeof(XParams));
	xgf_finish(P2, X0.G, lds);
#endif
}

// The buffers k_xgf left out: those whose grabs belong to several
// workgroups, one per workgroup at most (x_shared_of), finished after the
// kernel boundary by one workgroup.
__global__ __launch_bounds__(kFinThreads) void k_xshared(XParams P) {
	__shared__ uint32_t lds[kFinWords];
	if (!x_packed(P)) return;  // (k_xgf checksummed the batch buffer by buffer)
	const XGeo G = x_geo(P);
	if (G.nblk == 0) return;
	const XParts X(P, G);
	const uint32_t nb = (uint32_t)P.ngrid + 1;
	// (the grid has fewer than kFinThreads workgroups: one candidate per thread)
	const uint64_t mine = threadIdx.x < nb ? x_shared_of(P, G, X, threadIdx.x) : ~0ull;
	if (!__syncthreads_or(mine != ~0ull)) return;
	const XFin F = xfin_setup(P, lds, G);
	xfin_buffers(P, lds, G, F, nb, 0, blockDim.x, [&](uint64_t j) { return j == threadIdx.x ? mine : ~0ull; });
}

// ---------------------------------------------------------------------------
// state and launch
// ---------------------------------------------------------------------------
static uint64_t xal(uint64_t x) { return (x + 255) & ~uint64_t(255); }

uint64_t extent_state_bytes(uint64_t count, uint64_t capg, int num_cus) {
	const uint64_t nwave = (uint64_t)num_cus * 16;
	return 256 + 2 * xal(8 * count) + xal(512 * nwave) + xal(4 * nwave) + 2 * xal(4 * capg);
}

void extent_state_carve(void* mem, uint64_t count, uint64_t capg, int num_cus, XState* x) {
	uint8_t* p = static_cast<uint8_t*>(mem);
	const uint64_t nwave = (uint64_t)num_cus * 16;
	x->xhdr = reinterpret_cast<uint32_t*>(p);
	p += 256;
	x->ps = reinterpret_cast<uint32_t*>(p);
	p += xal(8 * count);
	x->pe = reinterpret_cast<uint32_t*>(p);
	p += xal(8 * count);
	x->dummy = reinterpret_cast<uint32_t*>(p);
	p += xal(512 * nwave);
	x->ragg = reinterpret_cast<uint32_t*>(p);
	p += xal(4 * nwave);
	x->wq = reinterpret_cast<uint32_t*>(p);
	p += xal(4 * capg);
	x->gagg = reinterpret_cast<uint32_t*>(p);
	x->capg = capg;
}

// The grab stream and the finishing pass in one kernel (k_xgf + k_xshared):
// correct, measured slower than k_xgrab + k_xfin,
// so off unless FDBX_FUSED=1 or fdbx_set_fused(1) (tests) turns it on.
static int g_fused = -1;
static bool extent_fused() {
	if (__atomic_load_n(&g_fused, __ATOMIC_RELAXED) < 0) {
		const char* e = getenv("FDBX_FUSED");
		int expect = -1;
		__atomic_compare_exchange_n(&g_fused, &expect, e && atoi(e) == 1 ? 1 : 0, false, __ATOMIC_RELAXED,
		                            __ATOMIC_RELAXED);
	}
	return __atomic_load_n(&g_fused, __ATOMIC_RELAXED) == 1;
}

// phase 0: the streaming kernel; phase 1: the finishing kernel.  Both return
// at once when the packing check failed.
int launch_extent(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t stride,
                  uint64_t length, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                  const DevTables* tabs, int num_cus, const XState& xs, uint64_t* hstat, hipStream_t stream,
                  int phase) {
	if (count == 0) return 0;
	XParams P{};
	P.base = base; P.offsets = offsets; P.lengths = lengths; P.stride = stride; P.length = length; P.count = count;
	P.seed = seed; P.seeds = seeds; P.out = out; P.x = xs; P.tabs = tabs; P.hstat = hstat;
	P.nwave = (uint64_t)num_cus * 16;  // k_xstream: one 1024-thread workgroup per CU
	P.ctr = xs.ctr;
	P.grabs = xs.ctr != nullptr && xs.wq != nullptr;
	P.ngrid = (uint64_t)num_cus;
	if (num_cus + 1 > (int)kFinThreads) return -1;  // (k_xshared: one candidate per thread)
	if (P.grabs && extent_fused()) {
		if (phase == 0)
			k_xgf<<<(unsigned)num_cus, 1024, 0, stream>>>(P);
		else
			k_xshared<<<1, kFinThreads, 0, stream>>>(P);
		return 0;
	}
	if (phase == 0) {
		if (P.grabs)
			k_xgrab<<<(unsigned)num_cus, 1024, 0, stream>>>(P);
		else
			k_xstream<<<(unsigned)num_cus, 1024, 0, stream>>>(P);
	} else {
		// persistent, but no more workgroups than the buffers fill (each fills 133 KiB of LDS)
		const uint64_t g = (count + 2 * kFinThreads - 1) / (2 * kFinThreads);  // (two buffers per thread per pass)
		k_xfin<<<(unsigned)(g < (uint64_t)num_cus ? g : (uint64_t)num_cus), kFinThreads, 0, stream>>>(P);
	}
	return 0;
}

}  // namespace fdbcrc

// Development / tests: select the extent route's fused kernels (1) or the
// default pair (0) for later launches; returns the previous setting.
extern "C" int fdbx_set_fused(int on) {
	const int prev = fdbcrc::extent_fused() ? 1 : 0;
	__atomic_store_n(&fdbcrc::g_fused, on ? 1 : 0, __ATOMIC_RELAXED);
	return prev;
}

#ifdef FDBX_TIMES
extern "C" int fdbx_debug_times(void* host, uint64_t nwave) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbcrc::g_xt), nwave * 32, 0, hipMemcpyDeviceToHost);
}
extern "C" int fdbx_debug_ftimes(void* host, uint64_t nwg) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbcrc::g_xft), nwg * 64, 0, hipMemcpyDeviceToHost);
}
#endif
