// Long-buffer XXH3-64 route (gfx950): xxHash v0.8.0 XXH3_64bits[_withSeed]
// (flow/include/flow/xxhash.h:3641-3718, 3800-3837) of buffers longer than
// kXSplitMin, bit-identical, with the blocks of one buffer computed by many
// waves at once.
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
// k_xlong: one persistent 1024-thread workgroup per CU, D never leaves it.
// Four CHAIN waves each own a SLOT: a buffer taken from the batch's long
// buffers, largest first (the planner's size classes), and a ring of 64
// STEPS (4 blocks each) of stripe sums in LDS.  Twelve PRODUCER waves claim
// steps of the slots' buffers (LDS compare-and-swap, never past the ring's
// free room), stream the step's four blocks exactly like k_xxh3_rows (a
// 16-lane row per block: four coalesced 256-byte loads, 32x32->64 products,
// two DPP row rotates) and write D into the ring with the step's tag; the
// chain wave scrambles the steps in order as their tags appear and merges.
// A first version wrote D to HBM (64 B per KiB) for a second kernel of
// chains: the stores alone cost phase A a fifth of its time (they hold up the
// in-order vmcnt waits on the loads behind them) and the chains ran after
// the stream.
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
typedef __attribute__((address_space(1))) const uint64_t g_u64;

__device__ __forceinline__ uint64_t gld64(const uint64_t* p) { return *((g_u64*)reinterpret_cast<uintptr_t>(p)); }
}  // namespace

// ---------------------------------------------------------------------------
// k_xlong
// ---------------------------------------------------------------------------
// Four chain slots: with two (fourteen producers) the chains bound the
// launch (264 us against 193 us on the chunks batch), three ~ four.
constexpr uint32_t kLWaves = 16, kLChains = 4, kLProd = kLWaves - kLChains;
constexpr uint32_t kLRingSteps = 64;  // per slot: 64 steps x 4 blocks x 64 B = 16 KiB
constexpr uint32_t kLSpinMax = 1u << 24;  // bounded waits (a correct launch never reaches them)

struct LSlot {
	// {claimed, gbase} is the producers' 64-bit compare-and-swap word: gbase (the
	// slot's step number of its buffer's step 0) grows with every buffer the
	// slot takes, so a claim read before the slot changed buffers can never
	// succeed after it (no ABA on `claimed` alone)
	uint32_t claimed;         // steps claimed by producers (~0 while the slot changes buffers)
	uint32_t gbase;
	uint32_t lim;             // steps that may be claimed: min(nsteps, consumed + kLRingSteps)
	uint32_t nsteps;          // the buffer's steps
	uint64_t p, len, seed;
	uint32_t closed, pad;     // the slot takes no more buffers
};
typedef __attribute__((address_space(3))) volatile LSlot lds_vslot;
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
typedef __attribute__((address_space(3))) volatile uint64_t lds_vu64;
struct LShared {
	uint64_t ring[kLChains][kLRingSteps * 4][8];  // D of block row (gstep % 64) * 4 + r
	uint32_t tag[kLChains][kLRingSteps];          // gstep + 1 once the step's D is in the ring
	LSlot slot[kLChains];
};

#ifdef FDBXXH_TIMES
// development: per-wave {start, producers' first idle / chains' last dequeue, end, steps | buffers + spins << 20}
__device__ uint64_t g_lt[4096][4];
#endif

template <bool SEEDS>
__global__ __launch_bounds__(1024) void k_xlong(XLong S) {
	__shared__ LShared L;
	const uint64_t nlong = rdf64(gld64(S.sh + 0));
	if (nlong == 0) return;  // no long buffer this batch (uniform over the grid)
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#ifdef FDBXXH_TIMES
	const uint64_t lt0 = __builtin_amdgcn_s_memrealtime();
	uint64_t lt1 = 0, lcnt = 0;
	const uint32_t lw = blockIdx.x * 16 + wv;
#endif
	for (uint32_t q = threadIdx.x; q < kLChains * kLRingSteps; q += blockDim.x) (&L.tag[0][0])[q] = 0;
	if (threadIdx.x < kLChains) {
		LSlot& s = L.slot[threadIdx.x];
		s.nsteps = s.gbase = s.lim = 0;
		s.claimed = ~0u;
		s.closed = 0;
	}
	__syncthreads();
	// LDS-typed volatile pointers: address-space inference leaves volatile
	// accesses alone, and through a generic pointer every slot or tag read was
	// a FLAT load -- which waits vmcnt(0), i.e. for the producer's whole load
	// stream, at every claim (one step in flight per wave: 5.4 TB/s)
	lds_vslot* VS = (lds_vslot*)L.slot;
	lds_vu32* VT = (lds_vu32*)&L.tag[0][0];

	if (wv >= kLProd) {
		// ---------------- chain wave: slot c ----------------
		// Its scrambles are a dependent chain of a few instructions per block,
		// issued between the producers' streams on the same SIMD: at the default
		// priority the arbitration starved it (the rings filled and the producers
		// idled), so it takes the highest.
		__builtin_amdgcn_s_setprio(3);
		const uint32_t c = wv - kLProd;
		const uint32_t j = lane & 7;
		const uint64_t init = j == 0 ? P32_3 : j == 1 ? P64_1 : j == 2 ? P64_2 : j == 3 ? P64_3
		                    : j == 4 ? P64_4 : j == 5 ? P32_2 : j == 6 ? P64_5 : P32_1;
		uint32_t gseq = 0;
		for (;;) {
			uint64_t q = 0;
			if (lane == 0) q = atomicAdd((unsigned long long*)S.sh + 1, 1ull);
			q = rdf64(__shfl(q, 0));
			if (q >= nlong) break;
#ifdef FDBXXH_TIMES
			lt1 = __builtin_amdgcn_s_memrealtime();
			lcnt += 1;
#endif
			const XEnt E = S.ents[q];
			const uint64_t p = rdf64(E.p), len = rdf64(E.len), seed = rdf64(E.seed), idx = rdf64(E.idx);
			const uint64_t nfull = (len - 1) >> 10, nb = nfull + 1;
			const uint32_t nsteps = (uint32_t)((nb + 3) >> 2);
			// publish: claimed is the gate (~0 while the fields change: a producer
			// that reads it claims nothing; 0 opens the buffer's steps)
			if (lane == 0) {
				VS[c].p = p;
				VS[c].len = len;
				VS[c].seed = seed;
				VS[c].nsteps = nsteps;
				VS[c].gbase = gseq;
				VS[c].lim = nsteps < kLRingSteps ? nsteps : kLRingSteps;
				__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
				VS[c].claimed = 0;
			}
			const uint64_t ck = swd(16 + (int)j, seed);  // scramble key: secret + 128 + 8j
			const uint64_t gk = sat(1 + (int)j, 3, seed);  // merge key: secret + 11 + 8j
			const uint32_t cklo = (uint32_t)ck, ckhi = (uint32_t)(ck >> 32);
			// scrambleAcc (xxhash.h:3702-3718) in 32-bit halves: the high half's
			// product is off the low half's dependent path
			auto scr = [&](uint64_t a) __attribute__((always_inline)) -> uint64_t {
				const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
				const uint32_t lo2 = __builtin_amdgcn_bitop3_b32(lo, hi >> 15, cklo, 0x96);  // xor3
				const uint64_t m = (uint64_t)lo2 * (uint32_t)P32_1;
				return m + ((uint64_t)((hi ^ ckhi) * (uint32_t)P32_1) << 32);
			};
			uint64_t acc = init;
			for (uint32_t t = 0; t < nsteps; ++t) {
				const uint32_t gs = gseq + t, ri = gs % kLRingSteps;
				for (uint32_t spin = 0; VT[c * kLRingSteps + ri] != gs + 1; ++spin) {
					if (spin >= kLSpinMax) {
						// (never in a correct launch: a stalled ring).  The buffer's digest
						// is not written: the stall is reported through the workspace word
						// and the stream's status word (crc32c_gpu_stream_status).
						if (lane == 0) {
							*(volatile uint64_t*)(S.sh + 2) = 1;
							if (S.err) *(volatile uint32_t*)S.err = kErrXxhStall;
						}
						return;
					}
					__builtin_amdgcn_s_sleep(1);
#ifdef FDBXXH_TIMES
					lcnt += 1ull << 20;
#endif
				}
				__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
				const uint64_t b0 = 4ull * t;
				uint64_t x[4];
#pragma unroll
				for (uint32_t r = 0; r < 4; ++r) x[r] = L.ring[c][ri * 4 + r][j];
#pragma unroll
				for (uint32_t r = 0; r < 4; ++r)
					if (b0 + r < nb) acc = b0 + r < nfull ? scr(acc + x[r]) : acc + x[r];
				// the ring rows are read (in registers) before the step's room is handed back
				__builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
				if (lane == 0) VS[c].lim = t + 1 + kLRingSteps < nsteps ? t + 1 + kLRingSteps : nsteps;
			}
			if (lane == 0) {
				VS[c].claimed = ~0u;  // (every step was claimed: claimed == nsteps, no CAS in flight succeeds)
			}
			gseq += nsteps;
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
		}
		if (lane == 0) VS[c].closed = 1;
#ifdef FDBXXH_TIMES
		if (lane == 0 && lw < 4096) {
			g_lt[lw][0] = lt0;
			g_lt[lw][1] = lt1;
			g_lt[lw][2] = __builtin_amdgcn_s_memrealtime();
			g_lt[lw][3] = lcnt;
		}
#endif
		return;
	}

	// ---------------- producer wave ----------------
	// Lane (r, g, k) = (lane / 16, (lane % 16) / 4, lane % 4): row r takes block
	// 4t + r of a step, stripes g, g+4, g+8, g+12 for accumulator pair k.
	const int r = lane >> 4, l = lane & 15, k = l & 3, g = l >> 2;
	struct PStep {
		uint64_t v[4][2];
		uint64_t p, len, seed;
		uint32_t c, t, gs, nrows;  // slot, step, its tag - 1, rows in use (0: idle)
	};
	uint32_t pref = wv % kLChains;  // the slot tried first (rotates)
	// Claim a step (wave-uniform): one LDS read of the slot's {claimed, lim},
	// lane 0's compare-and-swap, then the buffer's fields (the buffer cannot
	// change while one of its steps is unwritten).
	auto claim = [&](PStep& St) __attribute__((always_inline)) {
		St.nrows = 0;
		// (a lost race moves on to the next slot: the winner's neighbours are
		// likely racing for this one too; two rounds over the slots)
		for (uint32_t u = 0; u < 2 * kLChains; ++u) {
			const uint32_t c = (pref + u) % kLChains;
			{
				const uint64_t cw = *(lds_vu64*)&VS[c].claimed;
				const uint32_t cl = (uint32_t)cw, gb = (uint32_t)(cw >> 32);
				// lim is read after {claimed, gbase}: if the slot changed buffers in
				// between, gbase differs and the swap below fails
				const uint32_t lim = VS[c].lim;
				if (cl >= lim) continue;  // (~0: between buffers)
				unsigned long long old = 0;
				if (lane == 0)
					old = atomicCAS((unsigned long long*)&L.slot[c].claimed, (unsigned long long)cw,
					                (unsigned long long)cw + 1ull);
				if (rdf64((uint64_t)__shfl((long long)old, 0)) != cw) continue;
				St.c = c;
				St.t = cl;
				St.gs = gb + cl;
				St.p = rdf64(VS[c].p);
				St.len = rdf64(VS[c].len);
				St.seed = rdf64(VS[c].seed);
				const uint64_t nb = ((St.len - 1) >> 10) + 1;
				St.nrows = 4ull * cl + 4 <= nb ? 4u : (uint32_t)(nb - 4ull * cl);
				pref = (c + 1) % kLChains;
				return;
			}
		}
	};
	// The loads are unconditional -- an idle step reads the first long buffer's
	// first KiB and discards it -- so the in-order vmcnt waits count exactly
	// one step's loads behind each step: skipped loads on one path made every
	// wait vmcnt(0) (one step in flight per wave).
	const uint64_t idle_p = rdf64(S.ents[0].p);
	auto load = [&](PStep& St) __attribute__((always_inline)) {
		const bool on = St.nrows != 0;
		const uint32_t rr = (uint32_t)r < St.nrows ? (uint32_t)r : 0u;  // rows past the buffer: row 0's block
		const uint64_t blk = on ? 4ull * St.t + rr : 0;
		const uint64_t len = on ? St.len : 1024;
		const uint64_t p = on ? St.p : idle_p;
		const uint64_t nfull = (len - 1) >> 10;
		const uint32_t ns = (uint32_t)(((len - 1) - (nfull << 10)) >> 6);
		const bool fin = blk == nfull;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool tail = fin && (s == 15 || s >= ns);
			const uint64_t a = tail ? p + len - 64 + 16 * k : p + (blk << 10) + 64 * s + 16 * k;
			const u64x2u x = __builtin_nontemporal_load((g_u64x2u*)a);
			St.v[i][0] = x[0];
			St.v[i][1] = x[1];
		}
	};
	// keys: stripe g + 4i (secret + 8s + 16k), last stripe (secret + 121 + 16k).
	// Seeded (SEEDS): the default secret's words are held and each key is
	// derived at use -- word j + seed for even j, - seed for odd j
	// (xxhash.h:3550-3566) -- instead of re-deriving a set of keys whenever the
	// seed changes (the two sets live across the branch spilled 10 VGPRs).
	uint64_t k0[4], k1[4], l0, l1, b15, b16, b17;
	{
		const uint64_t sd = SEEDS ? 0 : S.seed;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			k0[i] = swd(g + 4 * i + 2 * k, sd);
			k1[i] = swd(g + 4 * i + 2 * k + 1, sd);
		}
		l0 = sat(15 + 2 * k, 1, sd);
		l1 = sat(16 + 2 * k, 1, sd);
		b15 = kSecS[15 + 2 * k];
		b16 = kSecS[16 + 2 * k];
		b17 = kSecS[17 + 2 * k];
	}
	uint32_t tag_at = 0, tag_v = 0;  // the last computed step's tag, not yet published
	auto compute = [&](const PStep& St) __attribute__((always_inline)) {
		if (St.nrows == 0) return;
		// seeded keys: + seed on even secret words, - seed on odd ones (the
		// stripe keys' word parity is g's; the last stripe's straddle two words)
		const uint64_t sp = SEEDS ? ((g & 1) ? 0 - St.seed : St.seed) : 0;
		const uint64_t lk0 = SEEDS ? (((b15 - St.seed) >> 8) | ((b16 + St.seed) << 56)) : l0;
		const uint64_t lk1 = SEEDS ? (((b16 + St.seed) >> 8) | ((b17 - St.seed) << 56)) : l1;
		const uint64_t blk = 4ull * St.t + r;
		const uint64_t nfull = (St.len - 1) >> 10;
		const uint32_t ns = (uint32_t)(((St.len - 1) - (nfull << 10)) >> 6);
		const bool fin = blk == nfull;
		uint64_t d0 = 0, d1 = 0;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t s = g + 4 * i;
			const bool last = fin && s == 15;
			const bool on = !fin || s < ns || last;
			const uint64_t x0 = St.v[i][0] ^ (last ? lk0 : k0[i] + sp);
			const uint64_t x1 = St.v[i][1] ^ (last ? lk1 : k1[i] - sp);
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
		const uint32_t ri = St.gs % kLRingSteps;
		if (g == 0 && (uint32_t)r < St.nrows)
			*reinterpret_cast<u64x2*>(&L.ring[St.c][ri * 4 + r][2 * k]) =
			    u64x2{((uint64_t)hi0 << 32) | lo0, ((uint64_t)hi1 << 32) | lo1};
		tag_at = St.c * kLRingSteps + ri;
		tag_v = St.gs + 1;
	};
	// The step's tag, once its D is in LDS: issued after the next claim, whose
	// LDS round trips (in order with the D writes) already waited for them.
	auto publish = [&]() __attribute__((always_inline)) {
		if (tag_v == 0) return;
		__builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) (normally complete already)
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
		if (lane == 0) VT[tag_at] = tag_v;
		tag_v = 0;
	};
	auto all_closed = [&]() -> bool {
		bool cl = true;
#pragma unroll
		for (uint32_t c = 0; c < kLChains; ++c) cl = cl && VS[c].closed;
		return cl;
	};
	PStep A, B;
	claim(A);
	load(A);
	claim(B);
	load(B);
	uint32_t idle = 0;
	for (;;) {
		compute(A);
		claim(A);
		publish();
		load(A);
		compute(B);
		claim(B);
		publish();
		load(B);
#ifdef FDBXXH_TIMES
		lcnt += (A.nrows != 0) + (B.nrows != 0);
		if (A.nrows == 0 && B.nrows == 0 && lt1 == 0) lt1 = __builtin_amdgcn_s_memrealtime();
#endif
		if (A.nrows == 0 && B.nrows == 0) {
			if (all_closed()) break;
			if (++idle >= kLSpinMax) break;  // (never: see the chain's bound)
			__builtin_amdgcn_s_sleep(2);
		} else {
			idle = 0;
		}
	}
#ifdef FDBXXH_TIMES
	if (lane == 0 && lw < 4096) {
		g_lt[lw][0] = lt0;
		g_lt[lw][1] = lt1;
		g_lt[lw][2] = __builtin_amdgcn_s_memrealtime();
		g_lt[lw][3] = lcnt;
	}
#endif
}


int launch_xxh3_long(const XLong& S, int num_cus, bool seeds, hipStream_t stream) {
	if (seeds)
		k_xlong<true><<<(unsigned)num_cus, 1024, 0, stream>>>(S);
	else
		k_xlong<false><<<(unsigned)num_cus, 1024, 0, stream>>>(S);
	return 0;
}

}  // namespace fdbxxh

#ifdef FDBXXH_TIMES
extern "C" int fdbxxh_debug_ltimes(void* host, uint64_t nwave) {
	return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fdbxxh::g_lt), nwave * 32, 0, hipMemcpyDeviceToHost);
}
#endif
