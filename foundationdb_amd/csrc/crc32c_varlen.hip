// Variable-length / unaligned batched CRC-32C (gfx950).
//
// Serves every batch the 4 KiB page kernel does not: any alignment, any
// length (0 .. 2^64), offsets in any order (overlaps allowed), per-buffer
// seeds.  Reference semantics: crc32c_append (contrib/crc32/crc32c.cpp:346-356)
// per buffer; the chained/streaming callers (fdbrpc/FileTransfer.cpp:29-37)
// reduce to the same thing through crc32c_combine.
//
// Work decomposition -- balanced by BYTES, not by buffers:
//   k_plan   one workgroup per tile of 256 buffers: tile byte sums; zeroes out[]
//   k_scan   one workgroup: exclusive prefix over tiles, total bytes, quantum
//            Q = ceil(total / waves), and for each wave the tile holding its
//            first byte (w*Q)
//   k_varlen every wave owns the byte range [w*Q, (w+1)*Q) of the buffers laid
//            end to end in index order.  It walks the 4 KiB blocks of the
//            buffer pieces inside its range as ONE stream, with the next
//            block's loads always in flight (also across buffer boundaries),
//            and the per-buffer metadata fetched 64 buffers at a time.
// A buffer cut by a range boundary is checksummed in pieces: each piece's raw
// register is multiplied by x^(8*(bytes after the piece)) and XORed into
// out[] with atomicXor (linearity of CRC, the same identity as
// crc32c_combine); whole buffers are stored directly.
//
// Inside a piece [P0, P1): the 16-byte aligned chunks covering it are read as
// blocks aligned to the piece's aligned END (front padding of the first block
// reads as zero and costs nothing, see crc32c_kernels.hip); bytes outside
// [P0, P1) in the boundary chunks are masked to zero.  The seed enters as the
// register value at P0 -- XORed into the four message bytes at P0 -- and the
// z = (16 - P1 % 16) % 16 zero bytes masked after P1 are removed by a final
// multiply with x^(-8z).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_common.h"

namespace fdbcrc {

constexpr uint32_t kTile = 256;               // buffers per planning tile
constexpr uint64_t kSmall = 1024;             // pieces whose aligned span fits one 1 KiB quarter

struct VarlenParams {
	const uint8_t* base;
	const uint64_t* offsets;   // nullptr: fixed mode, buffer i at base + i*stride
	const uint64_t* lengths;   // nullptr: fixed mode, every buffer `length` bytes
	uint64_t stride, length, count;
	uint32_t seed;
	const uint32_t* seeds;
	uint32_t* out;
	const uint64_t* prefix;      // varlen: exclusive tile prefix [T+1]
	const uint32_t* wave_tile;   // varlen: tile of each wave's first byte
	const uint64_t* hdr;         // varlen: [0] total bytes, [1] quantum
	uint64_t total, quantum;     // fixed mode (host-computed)
	const DevTables* tabs;
};

// ---------------------------------------------------------------------------
// planning
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_plan(const uint64_t* __restrict__ lengths, uint64_t count,
                                              uint64_t* __restrict__ tile_sum, uint32_t* __restrict__ out) {
	__shared__ uint64_t part[4];
	const uint64_t i = (uint64_t)blockIdx.x * kTile + threadIdx.x;
	uint64_t v = 0;
	if (i < count) {
		v = lengths[i];
		out[i] = 0u;  // split buffers accumulate with atomicXor
	}
	// wave reduction (64 lanes) then across the 4 waves
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
	__syncthreads();
	if (threadIdx.x == 0) tile_sum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// Single workgroup.  ntile tiles, nwave waves in the main grid.
__global__ __launch_bounds__(1024) void k_scan(uint64_t* __restrict__ prefix, uint64_t ntile,
                                               uint32_t* __restrict__ wave_tile, uint64_t nwave,
                                               uint64_t* __restrict__ hdr) {
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
	q = q < 4096 ? 4096 : (q + 63) & ~uint64_t(63);
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
}

// ---------------------------------------------------------------------------
// main kernel helpers
// ---------------------------------------------------------------------------
// Uniform (wave-wide) multiply through nibble tables in global memory: the
// value is uniform, so these are scalar-cache loads, off the LDS path.
__device__ __forceinline__ uint32_t umul(const uint32_t (*tab)[16], uint32_t v) {
	v = rdfirst(v);
	uint32_t r = 0;
#pragma unroll
	for (int n = 0; n < 8; ++n) r ^= tab[n][(v >> (4 * n)) & 15u];
	return r;
}

// Uniform value times x^(8d), d >= 0: one table multiply per set bit of d.
__device__ uint32_t mul_xpow(const DevTables* __restrict__ t, uint32_t v, uint64_t d) {
	for (int m = 0; d; ++m, d >>= 1)
		if (d & 1) v = umul(t->pow2[m], v);
	return v;
}

// One piece of one buffer: bytes [P0, P1) of buffer `buf`.
struct Piece {
	uint64_t buf;
	uint64_t P0, P1;
	uint64_t after;     // bytes of the buffer after P1
	uint32_t seed;
	uint32_t flags;     // bit0: piece starts the buffer, bit1: buffer is split
};

__device__ __forceinline__ uint64_t span_aligned(const Piece& p) {
	return ((p.P1 + 15) & ~uint64_t(15)) - (p.P0 & ~uint64_t(15));
}

// Edge fix-ups of a piece, precomputed once (uniform):
//   lead chunk  (P0 & ~15): keep bytes >= P0%16, XOR the register value ~seed
//                           into the four message bytes at P0 (first piece)
//   spill chunk (lead+16):  the seed bytes that cross into the next chunk
//   tail chunk ((P1-1)&~15): keep bytes < P1 - tail
struct Edges {
	uint64_t lead, tail;
	uint32_t lm[4], inj[4], tm[4], spill;
	bool any_lead, any_tail, any_spill;
};

__device__ __forceinline__ Edges make_edges(const Piece& p) {
	Edges e;
	const int k0 = (int)(p.P0 & 15);
	const int k1 = (int)((p.P1 - 1) & 15) + 1;
	const uint32_t s0 = (p.flags & 1) ? ~p.seed : 0u;
	e.lead = p.P0 & ~uint64_t(15);
	e.tail = (p.P1 - 1) & ~uint64_t(15);
#pragma unroll
	for (int d = 0; d < 4; ++d) {
		const int lo = k0 - 4 * d, hi = k1 - 4 * d;  // kept byte range of dword d: [lo, hi)
		e.lm[d] = lo <= 0 ? ~0u : (lo >= 4 ? 0u : ~0u << (8 * lo));
		e.tm[d] = hi >= 4 ? ~0u : (hi <= 0 ? 0u : ~0u >> (8 * (4 - hi)));
		e.inj[d] = (lo >= 0 && lo < 4) ? s0 << (8 * lo) : ((lo < 0 && lo > -4) ? s0 >> (-8 * lo) : 0u);
	}
	e.spill = k0 > 12 ? s0 >> (8 * (16 - k0)) : 0u;
	e.any_lead = k0 != 0 || (p.flags & 1);
	e.any_tail = k1 != 16;
	e.any_spill = e.spill != 0;
	return e;
}

// Apply the edge fix-ups to the chunk this lane loaded at `ca` for one load
// whose 1 KiB window starts at `w` (uniform early-out when the window has no edge).
__device__ __forceinline__ void fix_edges(u32x4& r, uint64_t w, uint64_t ca, const Edges& e) {
	const bool wl = e.any_lead && e.lead >= w && e.lead < w + 1024;
	const bool wt = e.any_tail && e.tail >= w && e.tail < w + 1024;
	const bool ws = e.any_spill && e.lead + 16 >= w && e.lead + 16 < w + 1024;
	if (!(wl || wt || ws)) return;
	const bool il = ca == e.lead, it = ca == e.tail, is = ca == e.lead + 16;
#pragma unroll
	for (int d = 0; d < 4; ++d) {
		uint32_t m = (il ? e.lm[d] : ~0u) & (it ? e.tm[d] : ~0u);
		uint32_t inj = il ? e.inj[d] : ((is && d == 0) ? e.spill : 0u);
		r[d] = (r[d] & m) ^ inj;
	}
}

__device__ __forceinline__ u32x4 load_chunk_if(uint64_t ca, const Piece& p) {
	const bool ok = ca + 16 > p.P0 && ca < p.P1;
	return ok ? ld16(reinterpret_cast<const uint8_t*>(ca)) : u32x4{0u, 0u, 0u, 0u};
}

// Register chain over the lane's 64 contiguous bytes (layout B, 4-byte slicing).
__device__ __forceinline__ uint32_t chain64_b(const uint32_t* lds, uint32_t s, const Block& b, uint32_t c4) {
	s = feed16_b(lds, s, b.r[0], c4);
	s = feed16_b(lds, s, b.r[1], c4);
	s = feed16_b(lds, s, b.r[2], c4);
	s = feed16_b(lds, s, b.r[3], c4);
	return s;
}

__global__ __launch_bounds__(1024) void k_varlen(VarlenParams P, const DevTables* __restrict__ T) {
	__shared__ uint32_t lds[kLdsBytesB / 4];
	const LaneCtx c = make_ctx();
	const uint32_t col4 = (c.lane & 31) * 4;
	const uint32_t c4 = col4 | 0x10000u;
	const uint32_t c_lane = (kS4LaneOff + (c.lane >> 5) * 0x4000) | col4;
	fill_lds_b(lds, T);
	const uint64_t wpb = blockDim.x >> 6;
	const uint64_t nwave = (uint64_t)gridDim.x * wpb;
	const uint64_t w = (uint64_t)blockIdx.x * wpb + rdfirst(threadIdx.x >> 6);
	const bool fixed = P.offsets == nullptr;
	uint64_t total = P.total, Q = P.quantum;
	if (!fixed) {  // planner output (global address space)
		typedef __attribute__((address_space(1))) const uint64_t g_u64;
		const g_u64* h = (const g_u64*)reinterpret_cast<uintptr_t>(P.hdr);
		total = rdfirst64(h[0]);
		Q = rdfirst64(h[1]);
	}
	const uint64_t lo = w * Q;
	const uint64_t hi = w + 1 == nwave ? ~uint64_t(0) : lo + Q;
	if (lo > total || P.count == 0) return;

	auto rd64 = [](uint64_t v, int k) -> uint64_t { return rdlane64(v, k); };

	// ---- locate the first buffer touching [lo, hi)
	uint64_t i0, start0;
	if (fixed) {
		i0 = P.length ? lo / P.length : 0;
		start0 = i0 * P.length;
	} else {
		const uint64_t t = P.wave_tile[w];
		i0 = t * kTile;
		start0 = P.prefix[t];
		bool found = false;
		while (!found && i0 < P.count) {
			const uint64_t mylen = i0 + c.lane < P.count ? P.lengths[i0 + c.lane] : 0;
			for (int k = 0; k < 64 && i0 < P.count; ++k) {
				const uint64_t len = rd64(mylen, k);
				if (start0 + len > lo || (len == 0 && start0 >= lo)) { found = true; break; }
				start0 += len;
				++i0;
			}
		}
	}

	// ---- piece generator over [lo, hi); metadata 64 buffers per batch
	struct Gen {
		uint64_t i, start, bi0;
		uint64_t m_off, m_len, n_off, n_len;
		uint32_t m_sd, n_sd;
	};
	auto fetch = [&](uint64_t b0, uint64_t& off, uint64_t& len, uint32_t& sd) {
		const uint64_t j = b0 + c.lane;
		const bool ok = j < P.count;
		off = fixed ? j * P.stride : (ok ? P.offsets[j] : 0);
		len = fixed ? P.length : (ok ? P.lengths[j] : 0);
		sd = P.seeds ? (ok ? P.seeds[j] : 0) : P.seed;
	};
	auto gen_init = [&](Gen& g) {
		g.i = i0; g.start = start0; g.bi0 = i0;
		fetch(g.bi0, g.m_off, g.m_len, g.m_sd);
		fetch(g.bi0 + 64, g.n_off, g.n_len, g.n_sd);
	};
	// final register contribution r of a piece (already aligned to the piece end)
	auto store = [&](const Piece& p, uint32_t r) {
		if (p.after) r = mul_xpow(T, r, p.after);
#ifdef FDBCRC_DEBUG
		if (p.buf >= P.count) {
			if (c.lane == 0 && atomicAdd(&g_dbg[2], 1ull) == 0) { g_dbg[3] = p.buf; g_dbg[4] = 3; }
			return;
		}
#endif
		if (c.lane == 0) {
			if (!(p.flags & 2)) P.out[p.buf] = ~r;
			else atomicXor(P.out + p.buf, (p.flags & 1) ? ~r : r);
		}
	};
	// next piece whose smallness == want_small; zero-length buffers and tiny
	// (< 16 B) pieces are finished on the spot by the small sweep.
	auto gen_next = [&](Gen& g, Piece& p, bool want_small) -> bool {
		for (;;) {
			if (g.i >= P.count || g.start >= hi) return false;
			if (g.i - g.bi0 == 64) {
				g.bi0 += 64;
				g.m_off = g.n_off; g.m_len = g.n_len; g.m_sd = g.n_sd;
				fetch(g.bi0 + 64, g.n_off, g.n_len, g.n_sd);
			}
			const int k = (int)(g.i - g.bi0);
			const uint64_t off = rd64(g.m_off, k), len = rd64(g.m_len, k);
			const uint32_t sd = rdlane(g.m_sd, k);
			const uint64_t a = lo > g.start ? lo - g.start : 0;
			const uint64_t b = hi - g.start < len ? hi - g.start : len;
			p.buf = g.i;
			++g.i;
			g.start += len;
			if (len == 0) {
				if (want_small && c.lane == 0) P.out[p.buf] = sd;
				continue;
			}
			const uint64_t q = reinterpret_cast<uint64_t>(P.base) + off;
			p.P0 = q + a;
			p.P1 = q + b;
			p.after = len - b;
			p.seed = sd;
			p.flags = (a == 0 ? 1u : 0u) | ((a != 0 || b != len) ? 2u : 0u);
			if (b - a < 16) {  // tiny piece: byte-serial, wave-uniform, layout-B T0
				if (want_small) {
					uint32_t s = (p.flags & 1) ? ~sd : 0u;
					for (uint64_t q2 = p.P0; q2 < p.P1; ++q2) {
						const uint32_t x = s ^ ld1(reinterpret_cast<const uint8_t*>(q2));
						s = (s >> 8) ^ lds_rd(lds, __builtin_amdgcn_perm(x, c4, 0x0c020400u) + 128);
					}
					store(p, s);
				}
				continue;
			}
			if ((span_aligned(p) <= kSmall) == want_small) return true;
		}
	};

	// ======================= sweep 1: small pieces, four per pass ==========
	// Load k (k = 0..3) fetches quarter qk = {0,2,1,3}[k] = 16-lane team qk
	// after unswizzle; team t checksums piece t inside the 1 KiB window ending
	// at its aligned end.  Lane tables multiply lane l by x^(8*64*(63-l)), so
	// team t's row sum carries an extra x^(8*1024*(3-t)), removed together
	// with the z trailing zeros by one uniform multiply (corr tables).
	// The four piece descriptors live in lanes 0..3 of a few VGPRs.
	{
		struct Quad {
			uint64_t P0, P1, buf, after;
			uint32_t seed, flags;
			int n;
		};
		auto wl64 = [&](uint64_t old, uint64_t v, int k) -> uint64_t { return c.lane == k ? v : old; };
		auto wl32 = [&](uint32_t old, uint32_t v, int k) -> uint32_t { return c.lane == k ? v : old; };
		auto piece_of = [&](const Quad& q, int t) -> Piece {
			Piece p;
			p.P0 = rd64(q.P0, t);
			p.P1 = rd64(q.P1, t);
			p.buf = rd64(q.buf, t);
			p.after = rd64(q.after, t);
			p.seed = rdlane(q.seed, t);
			p.flags = rdlane(q.flags, t);
			return p;
		};
		Gen g;
		gen_init(g);
		auto gather = [&](Quad& q) {
			q.n = 0;
			Piece p;
			while (q.n < 4 && gen_next(g, p, true)) {
				q.P0 = wl64(q.P0, p.P0, q.n);
				q.P1 = wl64(q.P1, p.P1, q.n);
				q.buf = wl64(q.buf, p.buf, q.n);
				q.after = wl64(q.after, p.after, q.n);
				q.seed = wl32(q.seed, p.seed, q.n);
				q.flags = wl32(q.flags, p.flags, q.n);
				++q.n;
			}
		};
		auto win = [](const Piece& p) -> uint64_t { return ((p.P1 + 15) & ~uint64_t(15)) - 1024; };
		const int quarter[4] = {0, 2, 1, 3};
		auto load_quad = [&](Block& b, const Quad& q) {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const int t = quarter[k];
				b.r[k] = u32x4{0u, 0u, 0u, 0u};
				if (t < q.n) {
					const Piece p = piece_of(q, t);
					b.r[k] = load_chunk_if(win(p) + c.ld_off, p);
				}
			}
		};
		Quad cur{}, nxt{};
		gather(cur);
		Block b, nb;
		if (cur.n) load_quad(b, cur);
		while (cur.n) {
			gather(nxt);
			if (nxt.n) load_quad(nb, nxt);
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const int t = quarter[k];
				if (t < cur.n) {
					const Piece p = piece_of(cur, t);
					const Edges e = make_edges(p);
					fix_edges(b.r[k], win(p), win(p) + c.ld_off, e);
				}
			}
			unswizzle(b);
			const uint32_t x = row_xor(mul_nibbles(lds, chain64_b(lds, 0u, b, c4), c_lane));
			for (int t = 0; t < cur.n; ++t) {
				const Piece p = piece_of(cur, t);
				const uint32_t z = (uint32_t)(-p.P1 & 15);
				store(p, umul(T->corr[t][z], rdlane(x, 16 * t)));
			}
			__builtin_amdgcn_sched_barrier(0);
			cur = nxt;
			b = nb;
		}
	}

	// ======================= sweep 2: large pieces, 4 KiB blocks ===========
	// Blocks aligned to the piece's aligned end; each block's register sum is
	// reduced to a uniform value and folded Horner-style with x^(8*4096).
	{
		Gen g;
		gen_init(g);
		Piece cur, nxt;
		if (!gen_next(g, cur, false)) return;
		auto nblk_of = [](const Piece& p) -> uint64_t { return (span_aligned(p) + 4095) >> 12; };
		auto vbase_of = [&](const Piece& p) -> uint64_t {
			return ((p.P1 + 15) & ~uint64_t(15)) - 4096 * nblk_of(p);
		};
		const uint32_t koff[4] = {0, 2048, 1024, 3072};
		auto load_blk = [&](Block& b, const Piece& p, uint64_t blk) {
			const uint64_t bb = vbase_of(p) + 4096 * blk;
			if (bb >= p.P0 && bb + 4096 <= p.P1) {
				load_block(b, reinterpret_cast<const uint8_t*>(bb), c.ld_off);
			} else {
#pragma unroll
				for (int k = 0; k < 4; ++k) b.r[k] = load_chunk_if(bb + koff[k] + c.ld_off, p);
			}
		};
		uint64_t blk = 0, cur_nblk = nblk_of(cur);
		Edges e = make_edges(cur);
		Block b, nb;
		load_blk(b, cur, 0);
		uint32_t acc = 0;
		for (;;) {
			bool more;
			uint64_t nblk_idx = 0;
			if (blk + 1 < cur_nblk) {
				nxt = cur;
				nblk_idx = blk + 1;
				more = true;
			} else {
				more = gen_next(g, nxt, false);
			}
			if (more) load_blk(nb, nxt, nblk_idx);
			__builtin_amdgcn_sched_barrier(0);
			const uint64_t bb = vbase_of(cur) + 4096 * blk;
			// edges live in the first block, the last block, and (seed bytes
			// spilling over a chunk boundary) possibly the second: fix_edges'
			// uniform per-window test decides
#pragma unroll
			for (int k = 0; k < 4; ++k) fix_edges(b.r[k], bb + koff[k], bb + koff[k] + c.ld_off, e);
			unswizzle(b);
			const uint32_t v = wave_xor(mul_nibbles(lds, chain64_b(lds, 0u, b, c4), c_lane));
			acc = blk ? umul(T->block, acc) ^ v : v;
			if (blk + 1 == cur_nblk) store(cur, umul(T->corr[3][(uint32_t)(-cur.P1 & 15)], acc));
			__builtin_amdgcn_sched_barrier(0);
			if (!more) break;
			if (nblk_idx == 0) {
				cur_nblk = nblk_of(nxt);
				e = make_edges(nxt);
			}
			cur = nxt;
			blk = nblk_idx;
			b = nb;
		}
	}
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
uint64_t varlen_workspace_bytes(uint64_t count, uint64_t nwave) {
	const uint64_t ntile = (count + kTile - 1) / kTile;
	return 16 + 8 * (ntile + 1) + 4 * nwave + 64;
}

int launch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count, uint32_t seed,
                  const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, void* ws,
                  hipStream_t stream) {
	const uint64_t grid = (uint64_t)num_cus;
	const uint64_t nwave = grid * 16;
	const uint64_t ntile = (count + kTile - 1) / kTile;
	uint8_t* w = static_cast<uint8_t*>(ws);
	uint64_t* hdr = reinterpret_cast<uint64_t*>(w);
	uint64_t* prefix = reinterpret_cast<uint64_t*>(w + 16);
	uint32_t* wave_tile = reinterpret_cast<uint32_t*>(w + 16 + 8 * (ntile + 1));
	k_plan<<<(unsigned)ntile, 256, 0, stream>>>(lengths, count, prefix, out);
	k_scan<<<1, 1024, 0, stream>>>(prefix, ntile, wave_tile, nwave, hdr);
	VarlenParams P{};
	P.base = base; P.offsets = offsets; P.lengths = lengths; P.count = count;
	P.seed = seed; P.seeds = seeds; P.out = out;
	P.prefix = prefix; P.wave_tile = wave_tile; P.hdr = hdr; P.tabs = tabs;
	k_varlen<<<(unsigned)grid, 1024, 0, stream>>>(P, tabs);
	return 0;
}

int launch_fixed_general(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                         const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus,
                         hipStream_t stream) {
	const uint64_t grid = (uint64_t)num_cus;
	const uint64_t nwave = grid * 16;
	VarlenParams P{};
	P.base = base; P.stride = stride; P.length = length; P.count = count;
	P.seed = seed; P.seeds = seeds; P.out = out; P.tabs = tabs;
	P.total = count * length;
	const uint64_t per = (P.total + nwave - 1) / nwave;
	if (length <= per) {
		// whole buffers per wave: no piece ever straddles two waves
		P.quantum = (per + length - 1) / length * length;
	} else {
		// long buffers: cut into 4 KiB-multiple pieces merged with atomicXor
		P.quantum = per < 4096 ? 4096 : (per + 4095) & ~uint64_t(4095);
		if (hipMemsetAsync(out, 0, 4 * count, stream) != hipSuccess) return -1;
	}
	k_varlen<<<(unsigned)grid, 1024, 0, stream>>>(P, tabs);
	return 0;
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
// Debug builds only (make debug): allowed window for varlen data loads, and
// readback of [lo, hi, violations, first bad address, site, ...].
extern "C" int crc32c_debug_bounds(uint64_t lo, uint64_t hi) {
	fdbcrc::k_dbg_set<<<1, 1>>>(lo, hi);
	return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
extern "C" int crc32c_debug_read(uint64_t* d_out8) {
	fdbcrc::k_dbg_get<<<1, 1>>>(reinterpret_cast<unsigned long long*>(d_out8));
	return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
#endif
