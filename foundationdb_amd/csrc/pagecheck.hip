// Batched page-format verifiers on top of the CRC-32C and XXH3-64 engines.
//
// SQLite (fdbserver/kvstore/KeyValueStoreSQLite.cpp:100-201,
// PageChecksumCodec::checksum with write == false): the 8-byte trailer
// SumType{part1, part2} at [pageLen-8, pageLen) covers [0, pageLen-8) and
// matches, in this order,
//   1. part1 == 0 && part2 == crc32c_append(0xfdbeefdb, data)            (:119-128)
//   2. part1 >> 24 == 0 && (part1, part2) == XXH3 split 24/32 bits        (:131-145)
//   3. (part1, part2) == hashlittle2(data, pc = pageNumber, pb = 0x5ca1ab1e) (:147-155)
// and the page is corrupt otherwise.  The status byte records which check
// matched (1, 2, 3) or 0.
//
// DiskQueue (fdbserver/kvstore/DiskQueue.cpp:1047-1120, Page::checkHash) by
// the header's implementationVersion (u16 at byte 10):
//   V0: UID hash == (hashlittle2(&seq, 4080, 0x12345678, 0xbeefabcd) as
//       (c << 32 | b), 0xFDB)
//   V1: hash32 == crc32c_append(0xfdbeefdb, page + 4, 4092)
//   V2: hash64 == XXH3_64bits(page + 8, 4088)
//   other versions: false.
//
// Pipeline (all on the caller's stream): ONE classify pass over the
// trailers/headers compacts the page numbers that need each algorithm into
// device lists, the list-mode page kernels (crc32c_kernels.hip,
// xxh3_kernels.hip) checksum only those pages, compare kernels write the
// status and append the pages a check rejected to the next algorithm's list
// (CRC -> XXH3 -> lookup3, the reference's order), and the lookup3 pages run
// densely, one lane each, their bytes staged through LDS with coalesced loads.  Every page is read by the algorithm its
// trailer/header selects and by no other, plus the later algorithms only
// after a rejection.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "pagecheck.h"
#include "xxh3_device.h"

namespace fdbpc {

typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint64_t g_u64;

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *((g_u32*)reinterpret_cast<uintptr_t>(p)); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) {
	return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
}

// Append page i to a device list: one atomic per wave (ballot + prefix).
__device__ __forceinline__ void push(bool want, uint32_t i, uint32_t* list, unsigned long long* n) {
	const uint64_t m = __ballot(want);
	if (!m) return;
	const int lane = threadIdx.x & 63;
	unsigned long long base = 0;
	if (lane == __builtin_ctzll(m)) base = atomicAdd(n, (unsigned long long)__builtin_popcountll(m));
	base = __shfl(base, __builtin_ctzll(m));
	if (want) list[base + __builtin_popcountll(m & ((1ull << lane) - 1))] = i;
}

// lookup3 hashlittle2 (flow/Hash3.c:566-700), one lane, 16-byte aligned data:
// four rounds (48 bytes) per step from three 16-byte loads, a quarter of the
// load instructions of a word-by-word walk (one lane walks one page, so every
// load touches its own cache line: the fall-through is load-issue bound, not
// HBM bound); the last 1..48 bytes word by word, the final 1..12 with the
// reference's tail mix (same values as its masked reads).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
// Wave-cooperative main loop (STAGED): the wave's 64 pages (one per lane, all
// of one length) are read in stages of kSt = 192 bytes (16 rounds) per page,
// coalesced -- load t of a stage covers chunks u = 64t + lane, i.e. chunk u % 12
// of lane u / 12's page: 12 lanes read one page's 192 contiguous bytes -- and
// the chunks reach the lane that owns the page through LDS (page stride 49
// words, so the 64 lanes' word reads hit distinct banks).  Lane-per-page
// loads touch a cache line per lane per instruction; these touch ~13 per 1 KiB.
constexpr uint32_t kSt = 192, kStW = 49;
// pages per wave in the lookup3 kernels (lanes past it duplicate pages and
// discard the result): fewer pages per wave, more waves per SIMD for the mix
// chains to interleave -- measured on the bench's mix (64 Ki fall-through
// pages): 64 -> 65.5 us, 32 -> 67.1 us, 16 -> 105 us (the duplicates' loads)
#ifndef FDBPC_L3_PER_WAVE
#define FDBPC_L3_PER_WAVE 64
#endif
constexpr uint32_t kL3PerWave = FDBPC_L3_PER_WAVE;
template <bool STAGED>
__device__ void hashlittle2_core(const uint8_t* k, uint64_t length, uint32_t* pc, uint32_t* pb, uint32_t* lw) {
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + (uint32_t)length + *pc;
	c += *pb;
#define ROT(x, r) (((x) << (r)) | ((x) >> (32 - (r))))
#define MIX()                                                                                                          \
	a -= c; a ^= ROT(c, 4);  c += b;                                                                                  \
	b -= a; b ^= ROT(a, 6);  a += c;                                                                                  \
	c -= b; c ^= ROT(b, 8);  b += a;                                                                                  \
	a -= c; a ^= ROT(c, 16); c += b;                                                                                  \
	b -= a; b ^= ROT(a, 19); a += c;                                                                                  \
	c -= b; c ^= ROT(b, 4);  b += a;
	if (STAGED) {
		// whole stages while more data follows them (the reference's
		// `while (length > 12)`, 16 rounds at a time); `length` is wave-uniform
		const uint64_t nst = length > kSt ? (length - 1) / kSt : 0;
		if (nst) {
			const int lane = threadIdx.x & 63;
			uint64_t ad[12];
			uint32_t wo[12];
			const uint64_t kp = reinterpret_cast<uint64_t>(k);
#pragma unroll
			for (int t = 0; t < 12; ++t) {
				const uint32_t u = 64u * t + (uint32_t)lane, pg = u / 12u, ck = u % 12u;
				const uint64_t base = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(kp >> 32), (int)pg) << 32) |
				                      (uint64_t)(uint32_t)__shfl((int)(uint32_t)kp, (int)pg);
				ad[t] = base + 16u * ck;
				wo[t] = pg * kStW + 4u * ck;
			}
			u32x4 st[12];
#pragma unroll
			for (int t = 0; t < 12; ++t) st[t] = *((g_u32x4*)ad[t]);
			const uint32_t* mine = lw + lane * kStW;
			// one stage in flight while one is mixed (two in flight measured the
			// same: the mix chain, one wave per SIMD, bounds the bench's mix)
			for (uint64_t sg = 0; sg < nst; ++sg) {
#pragma unroll
				for (int t = 0; t < 12; ++t)
#pragma unroll
					for (int e = 0; e < 4; ++e) lw[wo[t] + e] = st[t][e];
				// the next stage's loads (the last stage re-reads itself: discarded)
				const uint64_t nx = (sg + 1 < nst ? sg + 1 : sg) * kSt;
#pragma unroll
				for (int t = 0; t < 12; ++t) st[t] = *((g_u32x4*)(ad[t] + nx));
				__builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes are done
				__builtin_amdgcn_wave_barrier();
#pragma unroll
				for (int r = 0; r < 16; ++r) {
					a += mine[3 * r];
					b += mine[3 * r + 1];
					c += mine[3 * r + 2];
					MIX();
				}
				__builtin_amdgcn_wave_barrier();
			}
			length -= kSt * nst;
			k += kSt * nst;
		}
	}
#undef MIX
#define MIX()                                                                                                          \
	a -= c; a ^= ROT(c, 4);  c += b;                                                                                  \
	b -= a; b ^= ROT(a, 6);  a += c;                                                                                  \
	c -= b; c ^= ROT(b, 8);  b += a;                                                                                  \
	a -= c; a ^= ROT(c, 16); c += b;                                                                                  \
	b -= a; b ^= ROT(a, 19); a += c;                                                                                  \
	c -= b; c ^= ROT(b, 4);  b += a;
	// groups of 48 bytes (four whole rounds) while more data follows them: the
	// reference's `while (length > 12)` taken four rounds at a time.  One lane
	// walks one page and the lanes are few (only the pages no other check
	// accepted), so each group's loads go out kPre groups ahead (clamped to the
	// last group: duplicates are never used) -- the mix chain never waits for
	// memory once the pipeline is full.
	constexpr int kPre = 8;
	const uint64_t m = length > 48 ? (length - 1) / 48 : 0;
	if (m) {
		u32x4 q[kPre][3];
		auto ld = [&](int s, uint64_t g) {
			const uint8_t* p = k + 48 * (g < m ? g : m - 1);
			q[s][0] = *((g_u32x4*)reinterpret_cast<uintptr_t>(p));
			q[s][1] = *((g_u32x4*)reinterpret_cast<uintptr_t>(p + 16));
			q[s][2] = *((g_u32x4*)reinterpret_cast<uintptr_t>(p + 32));
		};
#pragma unroll
		for (int s = 0; s < kPre; ++s) ld(s, s);
		for (uint64_t g0 = 0; g0 < m; g0 += kPre) {
#pragma unroll
			for (int s = 0; s < kPre; ++s) {
				if (g0 + s < m) {
					const u32x4 x = q[s][0], y = q[s][1], z = q[s][2];
					a += x[0]; b += x[1]; c += x[2]; MIX();
					a += x[3]; b += y[0]; c += y[1]; MIX();
					a += y[2]; b += y[3]; c += z[0]; MIX();
					a += z[1]; b += z[2]; c += z[3]; MIX();
				}
				ld(s, g0 + s + kPre);
			}
		}
		length -= 48 * m;
		k += 48 * m;
	}
#undef MIX
#undef ROT
	uint32_t c2 = c, b2 = b;
	// the last 1..48 bytes: the word-by-word form, continuing from (a, b, c)
	uint32_t aa = a;
	{
#define ROT(x, r) (((x) << (r)) | ((x) >> (32 - (r))))
		while (length > 12) {
			aa += ld32(k);
			b2 += ld32(k + 4);
			c2 += ld32(k + 8);
			aa -= c2; aa ^= ROT(c2, 4);  c2 += b2;
			b2 -= aa; b2 ^= ROT(aa, 6);  aa += c2;
			c2 -= b2; c2 ^= ROT(b2, 8);  b2 += aa;
			aa -= c2; aa ^= ROT(c2, 16); c2 += b2;
			b2 -= aa; b2 ^= ROT(aa, 19); aa += c2;
			c2 -= b2; c2 ^= ROT(b2, 4);  b2 += aa;
			length -= 12;
			k += 12;
		}
		if (length == 0) {
			*pc = c2;
			*pb = b2;
			return;
		}
		uint32_t w[3] = {0, 0, 0};
		for (uint64_t i = 0; i < length; ++i) w[i >> 2] |= (uint32_t)k[i] << (8 * (i & 3));
		aa += w[0];
		b2 += w[1];
		c2 += w[2];
		c2 ^= b2; c2 -= ROT(b2, 14);
		aa ^= c2; aa -= ROT(c2, 11);
		b2 ^= aa; b2 -= ROT(aa, 25);
		c2 ^= b2; c2 -= ROT(b2, 16);
		aa ^= c2; aa -= ROT(c2, 4);
		b2 ^= aa; b2 -= ROT(aa, 14);
		c2 ^= b2; c2 -= ROT(b2, 24);
#undef ROT
	}
	*pc = c2;
	*pb = b2;
}

// ---------------------------------------------------------------------------
// Device lists, appended per workgroup
// ---------------------------------------------------------------------------
// A workgroup of kCB threads handles kCB * kPer consecutive entries; each
// list's appends collect in LDS (one LDS atomic per wave) and leave with ONE
// global atomic per list per workgroup.  (One global counter takes ~12 ns per
// atomic: a wave-aggregated append over 1 Mi pages -- 16 Ki atomics on one
// word -- cost ~200 us per pass, more than the pass's reads.)
constexpr uint32_t kCB = 1024, kPer = 4, kSpan = kCB * kPer;

template <int NL>
struct Stage {
	uint32_t cnt[NL];
	unsigned long long base[NL];
	uint32_t item[NL][kSpan];
};

template <int NL>
__device__ __forceinline__ void stage_init(Stage<NL>& S) {
	if (threadIdx.x < NL) S.cnt[threadIdx.x] = 0;
	__syncthreads();
}

template <int NL>
__device__ __forceinline__ void stage_push(Stage<NL>& S, int L, bool want, uint32_t v) {
	const uint64_t m = __ballot(want);
	if (!m) return;
	const int lane = threadIdx.x & 63, lead = __builtin_ctzll(m);
	uint32_t pos = 0;
	if (lane == lead) pos = atomicAdd(&S.cnt[L], (uint32_t)__builtin_popcountll(m));
	pos = (uint32_t)__shfl((int)pos, lead);
	if (want) S.item[L][pos + __builtin_popcountll(m & ((1ull << lane) - 1))] = v;
}

template <int NL>
__device__ __forceinline__ void stage_flush(Stage<NL>& S, uint32_t* const (&lists)[NL], unsigned long long* ctr) {
	__syncthreads();
	if (threadIdx.x < NL) S.base[threadIdx.x] = S.cnt[threadIdx.x] ? atomicAdd(&ctr[threadIdx.x], (unsigned long long)S.cnt[threadIdx.x]) : 0;
	__syncthreads();
#pragma unroll
	for (int L = 0; L < NL; ++L)
		for (uint32_t k = threadIdx.x; k < S.cnt[L]; k += kCB) lists[L][S.base[L] + k] = S.item[L][k];
}

// failure count: one global atomic per workgroup
__device__ __forceinline__ void count_bad(bool bad, uint32_t* s_bad, unsigned long long* ctr_bad) {
	const uint64_t m = __ballot(bad);
	if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(s_bad, (uint32_t)__builtin_popcountll(m));
	__syncthreads();
	if (threadIdx.x == 0 && *s_bad) atomicAdd(ctr_bad, (unsigned long long)*s_bad);
}

// ---------------------------------------------------------------------------
// SQLite
// ---------------------------------------------------------------------------
// ctr[0] CRC list, ctr[1] XXH3 list, ctr[2] lookup3 list, ctr[3] corrupt pages.
constexpr uint8_t kPending = 0xFF;
enum { L_CRC = 0, L_XXH = 1, L_L3 = 2 };

// One pass over the trailers: part1 == 0 -> CRC list; else top byte zero ->
// XXH3 list; else lookup3 list.
// The trailers are saved in trl[] (8 B per page, coalesced): the compare
// passes read them there instead of each page's last line again from HBM.
__global__ __launch_bounds__(kCB) void k_sq_classify(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                                                     uint8_t* __restrict__ status, uint32_t* crc_l, uint32_t* xxh_l,
                                                     uint32_t* l3_l, unsigned long long* __restrict__ ctr,
                                                     uint64_t* __restrict__ trl) {
	__shared__ Stage<3> S;
	stage_init(S);
	const uint64_t i0 = (uint64_t)blockIdx.x * kSpan;
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t i = i0 + k * kCB + threadIdx.x;
		const bool in = i < count;
		const uint64_t t = in ? ld64(pages + i * ps + ps - 8) : 1u;
		const uint32_t part1 = (uint32_t)t;
		if (in) {
			status[i] = kPending;
			trl[i] = t;
		}
		stage_push(S, L_CRC, in && part1 == 0, (uint32_t)i);
		stage_push(S, L_XXH, in && part1 != 0 && (part1 >> 24) == 0, (uint32_t)i);
		stage_push(S, L_L3, in && (part1 >> 24) != 0, (uint32_t)i);
	}
	uint32_t* const lists[3] = {crc_l, xxh_l, l3_l};
	stage_flush(S, lists, ctr);
}

// CRC results -> status 1; a failed CRC page (part1 == 0, so a zero top
// byte) is offered to XXH3 next, as the reference does (:131).
// by_page: the results are indexed by page (page sizes other than 4 KiB run
// the general engine over every page) instead of by list position.
__global__ __launch_bounds__(kCB) void k_sq_after_crc(const uint8_t* __restrict__ pages, uint64_t ps,
                                                      const uint32_t* __restrict__ crc_l, const uint32_t* __restrict__ crc_out,
                                                      bool by_page, uint8_t* __restrict__ status, uint32_t* xxh_l,
                                                      unsigned long long* __restrict__ ctr,
                                                      const uint64_t* __restrict__ trl) {
	const uint64_t n = ctr[L_CRC];
	const uint64_t j0 = (uint64_t)blockIdx.x * kSpan;
	if (j0 >= n) return;  // uniform: the whole workgroup leaves
	__shared__ Stage<1> S;
	stage_init(S);
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t j = j0 + k * kCB + threadIdx.x;
		bool fail = false;
		uint32_t i = 0;
		if (j < n) {
			i = crc_l[j];
			const bool ok = (by_page ? crc_out[i] : crc_out[j]) == (uint32_t)(trl[i] >> 32);
			if (ok) status[i] = 1;
			fail = !ok;
		}
		stage_push(S, 0, fail, i);
	}
	uint32_t* const lists[1] = {xxh_l};
	stage_flush(S, lists, ctr + L_XXH);
}

__global__ __launch_bounds__(kCB) void k_sq_after_xxh(const uint8_t* __restrict__ pages, uint64_t ps,
                                                      const uint32_t* __restrict__ xxh_l, const uint64_t* __restrict__ xxh_out,
                                                      uint8_t* __restrict__ status, uint32_t* l3_l,
                                                      unsigned long long* __restrict__ ctr,
                                                      const uint64_t* __restrict__ trl) {
	const uint64_t n = ctr[L_XXH];
	const uint64_t j0 = (uint64_t)blockIdx.x * kSpan;
	if (j0 >= n) return;
	__shared__ Stage<1> S;
	stage_init(S);
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t j = j0 + k * kCB + threadIdx.x;
		bool fail = false;
		uint32_t i = 0;
		if (j < n) {
			i = xxh_l[j];
			const uint64_t h = xxh_out[j];
			const uint64_t t = trl[i];
			const bool ok = (uint32_t)t == (uint32_t)((h >> 32) & 0x00ffffffu) && (uint32_t)(t >> 32) == (uint32_t)h;
			if (ok) status[i] = 2;
			fail = !ok;
		}
		stage_push(S, 0, fail, i);
	}
	uint32_t* const lists[1] = {l3_l};
	stage_flush(S, lists, ctr + L_L3);
}

// The pages no other check accepted, one per lane (dense list): hashlittle2
// with the page number (:147-155), then the final status and the corrupt count.
__global__ __launch_bounds__(256) void k_sq_final(const uint8_t* __restrict__ pages, uint64_t ps, uint32_t first_pgno,
                                                  const uint32_t* __restrict__ l3_l, uint8_t* __restrict__ status,
                                                  unsigned long long* __restrict__ ctr,
                                                  const uint64_t* __restrict__ trl) {
	const uint64_t n = ctr[L_L3];
	if ((uint64_t)blockIdx.x * 4 * kL3PerWave >= n) return;
	__shared__ uint32_t s_bad;
	__shared__ uint32_t lw[4][64 * kStW];  // per wave: one stage of its 64 lanes' pages
	if (threadIdx.x == 0) s_bad = 0;
	__syncthreads();
	bool bad = false;
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t j0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kL3PerWave;  // the wave's first entry
	const uint64_t j = j0 + lane % kL3PerWave;
	if (j0 < n) {  // wave-uniform: the whole wave reads cooperatively, lanes past the list re-read the last page
		const uint32_t i = l3_l[j < n ? j : n - 1];
		const uint8_t* p = pages + (uint64_t)i * ps;
		uint32_t c = first_pgno + i, b = 0x5ca1ab1eu;
		hashlittle2_core<true>(p, ps - 8, &c, &b, lw[threadIdx.x >> 6]);  // pages 16-byte aligned (the contract)
		const uint64_t t = trl[i];
		const bool ok = c == (uint32_t)t && b == (uint32_t)(t >> 32);
		if (j < n && lane < kL3PerWave) {
			status[i] = ok ? 3 : 0;
			bad = !ok;
		}
	}
	count_bad(bad, &s_bad, &ctr[3]);
}

// The last kernel of a verify or seal call: the failure count out, and the
// stream's counters (crc32c_capi.cpp: stream_aux) back to zero for the next
// call -- no memset ahead of any call.
__global__ void k_pc_done(unsigned long long* __restrict__ ctr, uint64_t* __restrict__ d_bad) {
	const unsigned long long bad = ctr[3];
	__syncthreads();
	if (threadIdx.x == 0 && d_bad) *d_bad = bad;
	if (threadIdx.x < 8) ctr[threadIdx.x] = 0;
}

// ---------------------------------------------------------------------------
// DiskQueue (4096-byte pages)
// ---------------------------------------------------------------------------
// ctr[0] V1 list, ctr[1] V2 list, ctr[2] V0 (lookup3) list, ctr[3] failures.
// The first 8 bytes of each page (V1's hash32, V2's hash64) are saved in
// hs[] for the compare pass, from the line the version is read from.
__global__ __launch_bounds__(kCB) void k_dq_classify(const uint8_t* __restrict__ pages, uint64_t count,
                                                     uint8_t* __restrict__ ok, uint32_t* v1_l, uint32_t* v2_l,
                                                     uint32_t* v0_l, unsigned long long* __restrict__ ctr,
                                                     uint64_t* __restrict__ hs) {
	__shared__ Stage<3> S;
	__shared__ uint32_t s_bad;
	if (threadIdx.x == 0) s_bad = 0;
	stage_init(S);
	const uint64_t i0 = (uint64_t)blockIdx.x * kSpan;
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t i = i0 + k * kCB + threadIdx.x;
		const bool in = i < count;
		// the page's first 16 bytes in one load (pages are 16-byte aligned): the
		// stored hash (bytes 0..7) and implementationVersion (bytes 10..11)
		typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
		typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
		const u32x4 h = in ? *((g_u32x4*)reinterpret_cast<uintptr_t>(pages + i * 4096)) : u32x4{0u, 0u, 0u, 0u};
		const uint32_t ver = in ? (h[2] >> 16) : 0xFFFFu;
		if (in) {
			ok[i] = ver <= 2 ? kPending : 0;
			hs[i] = (uint64_t)h[0] | ((uint64_t)h[1] << 32);
		}
		stage_push(S, 0, in && ver == 1, (uint32_t)i);
		stage_push(S, 1, in && ver == 2, (uint32_t)i);
		stage_push(S, 2, in && ver == 0, (uint32_t)i);
		const uint64_t m = __ballot(in && ver > 2);  // unknown versions fail (:1119)
		if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(&s_bad, (uint32_t)__builtin_popcountll(m));
	}
	uint32_t* const lists[3] = {v1_l, v2_l, v0_l};
	stage_flush(S, lists, ctr);
	if (threadIdx.x == 0 && s_bad) atomicAdd(&ctr[3], (unsigned long long)s_bad);
}

// The two lists' results against the saved hashes.  kSpan entries per
// workgroup (kPer per thread), so the failure count takes one global atomic
// per 4096 entries: with 256-entry workgroups and a failure in nearly every
// one (1/16 of the bench's pages), the 4096 atomics on one word serialised
// to ~45 us (~12 ns each).
__global__ __launch_bounds__(kCB) void k_dq_compare(const uint8_t* __restrict__ pages, const uint32_t* __restrict__ v1_l,
                                                    const uint32_t* __restrict__ v2_l, const unsigned long long* __restrict__ ctr,
                                                    const uint32_t* __restrict__ crc_out, const uint64_t* __restrict__ xxh_out,
                                                    uint8_t* __restrict__ ok, unsigned long long* __restrict__ ctr_bad,
                                                    const uint64_t* __restrict__ hs) {
	const uint64_t n1 = ctr[0], n2 = ctr[1];
	const uint64_t j0 = (uint64_t)blockIdx.x * kSpan;
	if (j0 >= (n1 > n2 ? n1 : n2)) return;  // uniform: the whole workgroup leaves
	__shared__ uint32_t s_bad;
	if (threadIdx.x == 0) s_bad = 0;
	__syncthreads();
	uint32_t nbad = 0;
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t j = j0 + k * kCB + threadIdx.x;
		if (j < n1) {
			const uint64_t i = v1_l[j];
			const bool g = crc_out[j] == (uint32_t)hs[i];
			ok[i] = g ? 1 : 0;
			nbad += g ? 0 : 1;
		}
		if (j < n2) {
			const uint64_t i = v2_l[j];
			const bool g = xxh_out[j] == hs[i];
			ok[i] = g ? 1 : 0;
			nbad += g ? 0 : 1;
		}
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) nbad += (uint32_t)__shfl_xor((int)nbad, o);
	if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(&s_bad, nbad);
	__syncthreads();
	if (threadIdx.x == 0 && s_bad) atomicAdd(ctr_bad, (unsigned long long)s_bad);
}

// V0 pages: hashlittle2 over [16, 4096) -> UID(c << 32 | b, 0xFDB)
__global__ __launch_bounds__(256) void k_dq_final(const uint8_t* __restrict__ pages, const uint32_t* __restrict__ v0_l,
                                                  uint8_t* __restrict__ ok, unsigned long long* __restrict__ ctr) {
	const uint64_t n = ctr[2];
	if ((uint64_t)blockIdx.x * 4 * kL3PerWave >= n) return;
	__shared__ uint32_t s_bad;
	__shared__ uint32_t lw[4][64 * kStW];  // per wave: one stage of its 64 lanes' pages
	if (threadIdx.x == 0) s_bad = 0;
	__syncthreads();
	bool bad = false;
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t j0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kL3PerWave;
	const uint64_t j = j0 + lane % kL3PerWave;
	if (j0 < n) {  // wave-uniform (see k_sq_final)
		const uint64_t i = v0_l[j < n ? j : n - 1];
		const uint8_t* p = pages + i * 4096;
		uint32_t c = 0x12345678u, b = 0xbeefabcdu;
		hashlittle2_core<true>(p + 16, 4080, &c, &b, lw[threadIdx.x >> 6]);
		const bool good = ld64(p) == (((uint64_t)c << 32) | b) && ld64(p + 8) == 0xFDBull;
		if (j < n && lane < kL3PerWave) {
			ok[i] = good ? 1 : 0;
			bad = !good;
		}
	}
	count_bad(bad, &s_bad, &ctr[3]);
}

// ---------------------------------------------------------------------------
// Write side: sealing pages in place
// ---------------------------------------------------------------------------
// SQLite checksum(write = true) (KeyValueStoreSQLite.cpp:107-116): the trailer
// of page i = XXH3 split part1 = (h >> 32) & 0xffffff, part2 = (uint32_t)h, as
// one little-endian u64 at [ps - 8, ps) (8-byte aligned: pages 16-byte aligned).
// The seal stores are nontemporal: a plain 8-byte store leaves a partially
// written line in the last-level cache that costs the NEXT pass over the pages
// ~120 us per 1 Mi 4 KiB pages (its read-modify-write on the way to HBM lands
// in that pass); rewriting the whole 64-byte line instead (read 56 B + write
// 64 B) recovered nothing, the nontemporal 8-byte store all of it (same box:
// sqlite-seal 0.830 -> 0.722 ms, its XXH3 pass 778 -> 667 us = the pass on
// untouched pages; diskqueue-seal 0.873 -> 0.802 ms; tools/seal_probe.py).
__device__ __forceinline__ uint64_t sq_trailer(uint64_t h) { return ((h >> 32) & 0x00ffffffull) | (h << 32); }
__global__ __launch_bounds__(256) void k_sq_seal(uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                                                 const uint64_t* __restrict__ xxh_out) {
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
		__builtin_nontemporal_store(sq_trailer(xxh_out[i]), reinterpret_cast<uint64_t*>(pages + i * ps + ps - 8));
}

// DiskQueue Page::updateHash (DiskQueue.cpp:1089-1105) by implementationVersion:
// V1 -> list a (CRC-32C of [4, 4096) into hash32), V0 -> list c (hashlittle2
// UID), V2 and every other version -> list b (the switch's default: XXH3 of
// [8, 4096) into hash64).
__global__ __launch_bounds__(kCB) void k_dq_seal_classify(const uint8_t* __restrict__ pages, uint64_t count,
                                                          uint32_t* v1_l, uint32_t* v2_l, uint32_t* v0_l,
                                                          unsigned long long* __restrict__ ctr) {
	__shared__ Stage<3> S;
	stage_init(S);
	const uint64_t i0 = (uint64_t)blockIdx.x * kSpan;
#pragma unroll
	for (uint32_t k = 0; k < kPer; ++k) {
		const uint64_t i = i0 + k * kCB + threadIdx.x;
		const bool in = i < count;
		const uint32_t ver = in ? (ld32(pages + i * 4096 + 8) >> 16) : 0xFFFFu;
		stage_push(S, 0, in && ver == 1, (uint32_t)i);
		stage_push(S, 1, in && ver != 0 && ver != 1, (uint32_t)i);
		stage_push(S, 2, in && ver == 0, (uint32_t)i);
	}
	uint32_t* const lists[3] = {v1_l, v2_l, v0_l};
	stage_flush(S, lists, ctr);
}

// The hash stores of V1 / V2 pages (nontemporal, see k_sq_seal).
__global__ __launch_bounds__(kCB) void k_dq_seal_write(uint8_t* __restrict__ pages, const uint32_t* __restrict__ v1_l,
                                                       const uint32_t* __restrict__ v2_l,
                                                       const unsigned long long* __restrict__ ctr,
                                                       const uint32_t* __restrict__ crc_out,
                                                       const uint64_t* __restrict__ xxh_out) {
	const uint64_t n1 = ctr[0], n2 = ctr[1];
	for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < (n1 > n2 ? n1 : n2);
	     t += (uint64_t)gridDim.x * blockDim.x) {
		if (t < n1) __builtin_nontemporal_store(crc_out[t], reinterpret_cast<uint32_t*>(pages + (uint64_t)v1_l[t] * 4096));
		if (t < n2) __builtin_nontemporal_store(xxh_out[t], reinterpret_cast<uint64_t*>(pages + (uint64_t)v2_l[t] * 4096));
	}
}

// V0 pages: hash = UID(c << 32 | b, 0xFDB) from hashlittle2 over [16, 4096)
// (checksum_hashlittle2, DiskQueue.cpp:1077-1082); bytes 8..15 become 0xFDB
// (magic 0x0FDB, implementationVersion 0: the UID overlays them).  One serial
// lookup3 chain per page: ~30 us for any number of V0 pages up to a few
// thousand, a latency the stores' launch cannot hide (run in the same launch,
// under the stores' memory traffic, the chain's 21 dependent load stages took
// the launch from 50 to 84 us; a grid capped at 64 workgroups with a stride
// loop ran 44 us against this form's 30).
__global__ __launch_bounds__(256) void k_dq_seal_v0(uint8_t* __restrict__ pages, const uint32_t* __restrict__ v0_l,
                                                    const unsigned long long* __restrict__ ctr) {
	const uint64_t n = ctr[2];
	if ((uint64_t)blockIdx.x * 4 * kL3PerWave >= n) return;
	__shared__ uint32_t lw[4][64 * kStW];
	const uint32_t lane = threadIdx.x & 63;
	const uint64_t j0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kL3PerWave;
	const uint64_t j = j0 + lane % kL3PerWave;
	if (j0 < n) {  // wave-uniform (see k_sq_final)
		const uint64_t i = v0_l[j < n ? j : n - 1];
		uint8_t* p = pages + i * 4096;
		uint32_t c = 0x12345678u, b = 0xbeefabcdu;
		hashlittle2_core<true>(p + 16, 4080, &c, &b, lw[threadIdx.x >> 6]);
		if (j < n && lane < kL3PerWave) *reinterpret_cast<u32x4*>(p) = u32x4{b, c, 0xFDBu, 0u};
	}
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
uint64_t workspace_bytes(uint64_t count) {
	// counters, three u32 lists, u32 CRC results, u64 XXH3 results, and the
	// general engine's workspace (page sizes other than 4 KiB)
	return 64 + 8 * count + 4 * count * 4 + 64 + fdbcrc::varlen7_workspace_bytes(count, 0) + 16 + 8 * count + 16;
}

struct Ws {
	unsigned long long* ctr;
	uint32_t *list_a, *list_b, *list_c, *crc_out;
	uint64_t* xxh_out;
	uint64_t* trl;  // every page's trailer (SQLite) or first 8 bytes (DiskQueue), saved by the classify pass
	void* eng;
};
static Ws carve(void* ws, uint64_t count) {
	uint8_t* p = static_cast<uint8_t*>(ws);
	Ws w;
	w.ctr = reinterpret_cast<unsigned long long*>(p);
	p += 64;
	w.xxh_out = reinterpret_cast<uint64_t*>(p);
	p += 8 * count;
	w.list_a = reinterpret_cast<uint32_t*>(p);
	p += 4 * count;
	w.list_b = reinterpret_cast<uint32_t*>(p);
	p += 4 * count;
	w.list_c = reinterpret_cast<uint32_t*>(p);
	p += 4 * count;
	w.crc_out = reinterpret_cast<uint32_t*>(p);
	p += 4 * count;
	p = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
	w.trl = reinterpret_cast<uint64_t*>(p);
	p += 8 * count;
	w.eng = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
	return w;
}

static unsigned blocks(uint64_t n, uint64_t per = 256) { return (unsigned)((n + per - 1) / per); }

// The setup a verify / seal call can fail in, done before its classify pass
// counts into the stream's counters: the page kernels' grab counters (first
// use of the stream allocates them) and the XXH3 list kernel's shape rule.
static int setup_lists(const uint8_t* xxh_base, uint64_t ps, bool crc_pages, int num_cus, hipStream_t s) {
	uint32_t* pctr = nullptr;
	if (crc_pages && fdbcrc::page_counters(s, num_cus, &pctr)) return -1;
	if (((reinterpret_cast<uint64_t>(xxh_base) | ps) & 7) != 0 || ps - 8 <= 240) return -1;
	return 0;
}
// An error after the classify pass: the counters still go back to zero (in
// stream order, behind what was enqueued), so the stream's next call starts
// clean.
static int bail(unsigned long long* ctr, hipStream_t s) {
	k_pc_done<<<1, 64, 0, s>>>(ctr, nullptr);
	return -1;
}

int sqlite_verify(const uint8_t* pages, uint64_t ps, uint64_t count, uint32_t first_pgno, uint8_t* status,
                  uint64_t* d_bad, const fdbcrc::DevTables* tabs, int num_cus, void* ws, unsigned long long* ctr,
                  hipStream_t s) {
	const Ws w = carve(ws, count);
	// every fallible setup step before the classify pass, which starts counting
	// into the stream's counters (only k_pc_done puts them back to zero)
	if (setup_lists(pages, ps, ps == 4096, num_cus, s)) return -1;
	k_sq_classify<<<blocks(count, kSpan), kCB, 0, s>>>(pages, ps, count, status, w.list_a, w.list_b, w.list_c, ctr,
	                                                  w.trl);
	const uint64_t* n_crc = reinterpret_cast<const uint64_t*>(&ctr[L_CRC]);
	const uint64_t* n_xxh = reinterpret_cast<const uint64_t*>(&ctr[L_XXH]);
	if (ps == 4096) {
		if (fdbcrc::launch_pages_window_list(pages, 4096, w.list_a, n_crc, count, 0, 8, 0xFDBEEFDBu, w.crc_out, tabs,
		                                     num_cus, s))
			return bail(ctr, s);
		k_sq_after_crc<<<blocks(count, kSpan), kCB, 0, s>>>(pages, ps, w.list_a, w.crc_out, false, status, w.list_b, ctr,
		                                                   w.trl);
	} else {
		// other page sizes: every page through the general fixed-stride engine
		fdbcrc::launch_fixed_general(pages, ps, ps - 8, count, 0xFDBEEFDBu, nullptr, w.crc_out, tabs, num_cus, w.eng, s);
		k_sq_after_crc<<<blocks(count, kSpan), kCB, 0, s>>>(pages, ps, w.list_a, w.crc_out, true, status, w.list_b, ctr,
		                                                   w.trl);
	}
	fdbxxh::XxhParams P{};
	P.base = pages;
	P.stride = ps;
	P.length = ps - 8;
	P.count = count;
	P.out = w.xxh_out;
	P.idx = w.list_b;
	P.d_count = n_xxh;
	if (fdbxxh::launch_xxh3_pages_list(P, num_cus, s)) return bail(ctr, s);
	k_sq_after_xxh<<<blocks(count, kSpan), kCB, 0, s>>>(pages, ps, w.list_b, w.xxh_out, status, w.list_c, ctr, w.trl);
	k_sq_final<<<blocks(count, 4 * kL3PerWave), 256, 0, s>>>(pages, ps, first_pgno, w.list_c, status, ctr, w.trl);
	k_pc_done<<<1, 64, 0, s>>>(ctr, d_bad);
	return 0;
}

int diskqueue_check(const uint8_t* pages, uint64_t count, uint8_t* ok, uint64_t* d_bad,
                    const fdbcrc::DevTables* tabs, int num_cus, void* ws, unsigned long long* ctr, hipStream_t s) {
	const Ws w = carve(ws, count);
	if (setup_lists(pages + 8, 4096, true, num_cus, s)) return -1;
	k_dq_classify<<<blocks(count, kSpan), kCB, 0, s>>>(pages, count, ok, w.list_a, w.list_b, w.list_c, ctr, w.trl);
	const uint64_t* n1 = reinterpret_cast<const uint64_t*>(&ctr[0]);
	const uint64_t* n2 = reinterpret_cast<const uint64_t*>(&ctr[1]);
	// V1: crc32c(0xfdbeefdb, bytes [4, 4096))
	if (fdbcrc::launch_pages_window_list(pages, 4096, w.list_a, n1, count, 4, 0, 0xFDBEEFDBu, w.crc_out, tabs, num_cus, s))
		return bail(ctr, s);
	// V2: XXH3_64bits(bytes [8, 4096))
	fdbxxh::XxhParams P{};
	P.base = pages + 8;
	P.stride = 4096;
	P.length = 4088;
	P.count = count;
	P.out = w.xxh_out;
	P.idx = w.list_b;
	P.d_count = n2;
	if (fdbxxh::launch_xxh3_pages_list(P, num_cus, s)) return bail(ctr, s);
	k_dq_compare<<<blocks(count, kSpan), kCB, 0, s>>>(pages, w.list_a, w.list_b, ctr, w.crc_out, w.xxh_out, ok, &ctr[3],
	                                           w.trl);
	k_dq_final<<<blocks(count, 4 * kL3PerWave), 256, 0, s>>>(pages, w.list_c, ok, ctr);
	k_pc_done<<<1, 64, 0, s>>>(ctr, d_bad);
	return 0;
}

// Seal every page of the batch in place (codec op 6 / 7, KeyValueStoreSQLite.cpp:203-244).
int sqlite_seal(uint8_t* pages, uint64_t ps, uint64_t count, uint32_t first_pgno, int num_cus, void* ws,
                hipStream_t s) {
	const Ws w = carve(ws, count);
	const unsigned g = blocks(count) < 4096 ? blocks(count) : 4096;
	// page 1 of a database with pages over SQLITE_DEFAULT_PAGE_SIZE is first
	// sealed as a 1024-byte page (:221-224); its trailer at [1016, 1024) lies in
	// the full page's hashed bytes, so this goes first (stream order)
	const uint64_t i1 = (uint32_t)(1u - first_pgno);
	if (i1 < count && ps > 1024) {
		uint64_t* h1 = w.trl;  // (scratch: the saved trailers are not used here)
		fdbxxh::XxhParams P{};
		P.base = pages + i1 * ps;
		P.stride = 1024;
		P.length = 1016;
		P.count = 1;
		P.out = h1;
		if (fdbxxh::launch_xxh3(P, num_cus, nullptr, s)) return -1;
		k_sq_seal<<<1, 64, 0, s>>>(pages + i1 * ps, 1024, 1, h1);
	}
	fdbxxh::XxhParams P{};
	P.base = pages;
	P.stride = ps;
	P.length = ps - 8;
	P.count = count;
	P.out = w.xxh_out;
	if (fdbxxh::launch_xxh3(P, num_cus, nullptr, s)) return -1;
	k_sq_seal<<<g, 256, 0, s>>>(pages, ps, count, w.xxh_out);
	return 0;
}

int diskqueue_seal(uint8_t* pages, uint64_t count, const fdbcrc::DevTables* tabs, int num_cus, void* ws,
                   unsigned long long* ctr, hipStream_t s) {
	const Ws w = carve(ws, count);
	if (setup_lists(pages + 8, 4096, true, num_cus, s)) return -1;
	k_dq_seal_classify<<<blocks(count, kSpan), kCB, 0, s>>>(pages, count, w.list_a, w.list_b, w.list_c, ctr);
	const uint64_t* n1 = reinterpret_cast<const uint64_t*>(&ctr[0]);
	const uint64_t* n2 = reinterpret_cast<const uint64_t*>(&ctr[1]);
	if (fdbcrc::launch_pages_window_list(pages, 4096, w.list_a, n1, count, 4, 0, 0xFDBEEFDBu, w.crc_out, tabs, num_cus, s))
		return bail(ctr, s);
	fdbxxh::XxhParams P{};
	P.base = pages + 8;
	P.stride = 4096;
	P.length = 4088;
	P.count = count;
	P.out = w.xxh_out;
	P.idx = w.list_b;
	P.d_count = n2;
	if (fdbxxh::launch_xxh3_pages_list(P, num_cus, s)) return bail(ctr, s);
	k_dq_seal_write<<<blocks(count, kSpan), kCB, 0, s>>>(pages, w.list_a, w.list_b, ctr, w.crc_out, w.xxh_out);
	k_dq_seal_v0<<<blocks(count, 4 * kL3PerWave), 256, 0, s>>>(pages, w.list_c, ctr);
	k_pc_done<<<1, 64, 0, s>>>(ctr, nullptr);
	return 0;
}

}  // namespace fdbpc
