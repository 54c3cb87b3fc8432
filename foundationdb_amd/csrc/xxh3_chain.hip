// One XXH3-64 per CHAIN of non-contiguous segments: a packet laid out over a
// PacketBuffer chain (fdbrpc/FlowTransport.cpp:2025-2068: XXH3_64bits over one
// buffer, or XXH3_64bits_reset/_update per buffer/_digest when the packet
// spans several).  XXH3's stripes and its per-block scramble are sequential
// over the message, so unlike CRC-32C (crc32c_chain.hip) the segment digests
// cannot be combined: the segments are gathered, in order, into one staging
// area on the device and the varlen engine hashes each chain's contiguous
// range there.
//
//   k_seg_bsum / k_seg_bscan / k_seg_scan   exclusive prefix of the segment
//                                           lengths (staging offsets)
//   k_chain_ranges                          chain c = staging range
//                                           [pre[starts[c]], pre[starts[c+1]])
//                                           -- or, for a chain of 2..16
//                                           segments and 241 B .. 1 MiB, a
//                                           flag: hashed in place
//   k_seg_gather                            the segments of the other chains
//                                           of two or more, to their staging
//                                           offsets
//   launch_xxh3                             the varlen engine over the ranges
//   launch_xxh3_lchain                      chains of 2..8 segments and at most
//                                           16 KiB (k_chain_ranges lists them
//                                           per XCD), one wave each, staged in
//                                           LDS: no staging area, each byte read
//                                           from HBM once (k_xxh3_lchain in
//                                           xxh3_kernels.hip), over the varlen
//                                           pass's empty digests
//   launch_xxh3_segrows                     the flagged chains where their
//                                           segments lie (xxh3_segrows.hip),
//                                           over the varlen pass's empty digests
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xxh3_device.h"

namespace fdbxxh {

constexpr unsigned kScanT = 1024, kScanPer = 4, kScanSpan = kScanT * kScanPer;

__device__ __forceinline__ uint64_t block_sum(uint64_t v, uint64_t* s_w) {
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
	if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
	__syncthreads();
	uint64_t t = 0;
	for (unsigned k = 0; k < blockDim.x / 64; ++k) t += s_w[k];
	__syncthreads();
	return t;
}

__global__ __launch_bounds__(kScanT) void k_seg_bsum(const uint64_t* __restrict__ len, uint64_t n,
                                                     uint64_t* __restrict__ bsum, uint64_t* __restrict__ lcount) {
	__shared__ uint64_t s_w[kScanT / 64];
	if (blockIdx.x == 0 && threadIdx.x < 8) lcount[16 * threadIdx.x] = 0;  // (k_chain_ranges appends after this launch)
	uint64_t v = 0;
	for (unsigned k = 0; k < kScanPer; ++k) {
		const uint64_t i = (uint64_t)blockIdx.x * kScanSpan + k * kScanT + threadIdx.x;
		v += i < n ? len[i] : 0;
	}
	const uint64_t t = block_sum(v, s_w);
	if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

// exclusive scan of the block sums in place (one workgroup, any count)
__global__ __launch_bounds__(kScanT) void k_seg_bscan(uint64_t* __restrict__ bsum, uint64_t nb) {
	__shared__ uint64_t s_w[kScanT / 64];
	__shared__ uint64_t s_carry;
	if (threadIdx.x == 0) s_carry = 0;
	__syncthreads();
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	for (uint64_t c0 = 0; c0 < nb; c0 += kScanT) {
		const uint64_t i = c0 + threadIdx.x;
		const uint64_t v = i < nb ? bsum[i] : 0;
		uint64_t inc = v;
		for (int d = 1; d < 64; d <<= 1) {
			const uint64_t y = __shfl_up(inc, d);
			if (lane >= d) inc += y;
		}
		if (lane == 63) s_w[w] = inc;
		__syncthreads();
		uint64_t wb = 0, tot = 0;
		for (int k = 0; k < (int)(kScanT / 64); ++k) {
			wb += k < w ? s_w[k] : 0;
			tot += s_w[k];
		}
		const uint64_t carry = s_carry;
		if (i < nb) bsum[i] = carry + wb + inc - v;
		__syncthreads();
		if (threadIdx.x == 0) s_carry = carry + tot;
		__syncthreads();
	}
}

// pre[i] = exclusive prefix of len; pre[n] = total
__global__ __launch_bounds__(kScanT) void k_seg_scan(const uint64_t* __restrict__ len, uint64_t n,
                                                     const uint64_t* __restrict__ bsum, uint64_t* __restrict__ pre) {
	__shared__ uint64_t s_w[kScanT / 64];
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	const uint64_t i0 = (uint64_t)blockIdx.x * kScanSpan + (uint64_t)threadIdx.x * kScanPer;  // 4 consecutive per thread
	uint64_t v[kScanPer], run = 0;
	for (unsigned k = 0; k < kScanPer; ++k) {
		v[k] = i0 + k < n ? len[i0 + k] : 0;
		run += v[k];
	}
	uint64_t inc = run;
	for (int d = 1; d < 64; d <<= 1) {
		const uint64_t y = __shfl_up(inc, d);
		if (lane >= d) inc += y;
	}
	if (lane == 63) s_w[w] = inc;
	__syncthreads();
	uint64_t wb = 0;
	for (int k = 0; k < w; ++k) wb += s_w[k];
	uint64_t x = bsum[blockIdx.x] + wb + inc - run;
	for (unsigned k = 0; k < kScanPer; ++k) {
		if (i0 + k <= n) pre[i0 + k] = x;  // i0 + k == n writes the total
		x += v[k];
	}
}

// Segment j -> staging[pre[j], pre[j] + len[j]), for the segments of chains
// of two or more (segflag[j] == 0; a one-segment chain is hashed where it
// lies).  Bytes past `cap` are dropped (the caller's total_bytes bound was
// wrong: results undefined, but no write leaves the staging area).  One wave
// per 64 consecutive segments: their metadata in the lanes (one load each),
// then segment after segment, the body in 16-byte pieces -- aligned in
// staging (the staging area is 16-byte aligned), loaded from the segment at
// whatever alignment it has, four pieces per lane in flight -- and the < 16
// bytes before and after it byte by byte.  (One workgroup per segment spent
// its time on the metadata round trip: 509 us for the bench's 900 MiB.)
// A wave takes 64 segments (their metadata in its lanes) and copies them four
// at a time, one per 16-lane quarter: a 4 KiB segment is sixteen 16-byte
// loads per lane, all in flight before the stores, and the head and tail
// bytes (the staging offset's misalignment) load with them.  One segment per
// wave at a time -- a load round trip and a store round trip per segment --
// took 422 us on the bench's 668 k segments.
__global__ __launch_bounds__(256) void k_seg_gather(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                    const uint64_t* __restrict__ len, const uint64_t* __restrict__ pre,
                                                    const uint8_t* __restrict__ segflag, uint64_t nsegs,
                                                    uint8_t* __restrict__ staging, uint64_t cap) {
	typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
	typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
	typedef __attribute__((address_space(1))) const u32x4u g_u32x4u;
	constexpr int kR = 16;  // 16-byte chunks per lane per round: 4 KiB per quarter
	const uint32_t lane = threadIdx.x & 63, sub = lane >> 4, sl = lane & 15;
	const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t j0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; j0 < nsegs; j0 += 64 * nw) {
		const uint64_t jl = j0 + lane < nsegs ? j0 + lane : nsegs - 1;
		const uint64_t m_off = off[jl], m_len = len[jl], m_pre = pre[jl];
		const bool m_on = j0 + lane < nsegs && segflag[jl] == 0;
		uint64_t todo = __ballot(m_on);
		while (todo) {
			// up to four segments: quarter q takes the q-th lowest left
			int kq = -1;
#pragma unroll
			for (uint32_t q = 0; q < 4; ++q) {
				const int k = todo ? __builtin_ctzll(todo) : -1;
				todo &= todo ? todo - 1 : 0;
				kq = sub == q ? k : kq;
			}
			const bool act = kq >= 0;
			const int ks = act ? kq : 0;
			const uint64_t so = __shfl(m_off, ks), n = __shfl(m_len, ks), d = __shfl(m_pre, ks);
			const uint8_t* src = base + so;
			uint8_t* dst = staging + d;
			const uint64_t lim = !act || d >= cap ? 0 : (cap - d < n ? cap - d : n);
			uint64_t head = (16 - (d & 15)) & 15;
			head = head < lim ? head : lim;
			const uint64_t body = (lim - head) & ~uint64_t(15);
			const uint64_t t0 = head + body, ntail = lim - t0;
			const uint8_t hb = sl < head ? src[sl] : 0;
			const uint8_t tb = sl < ntail ? src[t0 + sl] : 0;
			for (uint64_t q = 0; q < body; q += 256ull * kR) {
				u32x4u v[kR];
#pragma unroll
				for (int r = 0; r < kR; ++r) {
					const uint64_t o = head + q + 256ull * r + 16ull * sl;
					v[r] = __builtin_nontemporal_load((g_u32x4u*)reinterpret_cast<uintptr_t>(src + (o < t0 ? o : head)));
				}
#pragma unroll
				for (int r = 0; r < kR; ++r) {
					const uint64_t o = head + q + 256ull * r + 16ull * sl;
					if (o < t0) *reinterpret_cast<u32x4*>(dst + o) = u32x4{v[r][0], v[r][1], v[r][2], v[r][3]};
				}
			}
			if (sl < head) dst[sl] = hb;
			if (sl < ntail) dst[t0 + sl] = tb;
		}
	}
}

// Ranges are clamped into the staging area [0, cap) and the chain starts to
// [0, nsegs]: a wrong total_bytes (or chain start) gives undefined digests,
// never a read past the staging area or past pre[].  A chain of one segment
// is hashed in place: its offset is taken relative to the staging area
// (64-bit wrap-around: the kernels add it to the staging address), and its
// segment is flagged so that the gather skips it.
// With the segment rows on (rows_on), a chain of 2 .. kSegRowsMax segments
// and 241 B .. kSegRowsMaxLen bytes is hashed in place by them (chflag 2, its
// segments not gathered, its varlen range empty: that digest is overwritten);
// every other multi-segment chain is hashed from staging.
__global__ __launch_bounds__(256) void k_chain_ranges(const uint64_t* __restrict__ starts, uint64_t nchains,
                                                      uint64_t nsegs, const uint64_t* __restrict__ pre, uint64_t cap,
                                                      const uint8_t* __restrict__ base,
                                                      const uint64_t* __restrict__ seg_off,
                                                      const uint8_t* __restrict__ staging,
                                                      uint8_t* __restrict__ segflag, uint64_t* __restrict__ ch_off,
                                                      uint64_t* __restrict__ ch_len, uint8_t* __restrict__ chflag, int rows_on,
                                                      int lc_on, uint64_t* __restrict__ list, uint64_t* __restrict__ counts,
                                                      uint64_t lcap) {
	const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const bool in = c < nchains;
	const uint64_t cc = in ? c : 0;
	uint64_t s0 = starts[cc], s1 = starts[cc + 1];
	s0 = s0 < nsegs ? s0 : nsegs;
	s1 = s1 < nsegs ? s1 : nsegs;
	const uint64_t la = pre[s0], lb = pre[s1];  // (unclamped: the chain's true length)
	uint64_t a = la < cap ? la : cap, b = lb < cap ? lb : cap;
	const bool one = s1 == s0 + 1;
	const uint64_t L = lb > la ? lb - la : 0;
	// the LDS route (k_xxh3_lchain): 2 .. kLChainSegs segments, at most kLChainMax bytes
	const bool lc = in && lc_on && s1 >= s0 + 2 && s1 - s0 <= kLChainSegs && L <= kLChainMax;
	const bool rows = !lc && rows_on && !one && s1 > s0 && s1 - s0 <= kSegRowsMax && L > 240 && L <= kSegRowsMaxLen;
	// appended to the list of this workgroup's XCD (workgroup b runs on XCD
	// b % 8), one atomic per workgroup on that XCD's counter: one counter for
	// the batch, one atomic per wave, serialised the appends (81 us on the
	// bench's 406 k chains)
	{
		__shared__ uint32_t s_n[4];
		__shared__ uint64_t s_at;
		const uint64_t m = __ballot(lc);
		const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
		if (lane == 0) s_n[wv] = (uint32_t)__builtin_popcountll(m);
		__syncthreads();
		const uint32_t x = blockIdx.x & 7;
		if (threadIdx.x == 0) {
			const uint32_t tot = s_n[0] + s_n[1] + s_n[2] + s_n[3];
			s_at = tot ? atomicAdd((unsigned long long*)(counts + 16 * x), (unsigned long long)tot) : 0;
		}
		__syncthreads();
		if (lc) {
			uint64_t k = s_at + (uint64_t)__builtin_popcountll(m & ((1ull << lane) - 1));
			for (uint32_t u = 0; u < wv; ++u) k += s_n[u];
			uint64_t* const lx = list + 2 * lcap * x;
			lx[2 * k] = c;
			lx[2 * k + 1] = s0 | ((s1 - s0) << 56);
		}
	}
	if (!in) return;
	for (uint64_t j = s0; j < s1; ++j) segflag[j] = one || rows || lc ? 1 : 0;
	ch_off[c] = one ? reinterpret_cast<uint64_t>(base) + seg_off[s0] - reinterpret_cast<uint64_t>(staging) : a;
	ch_len[c] = rows || lc ? 0 : (b > a ? b - a : 0);
	chflag[c] = lc ? 3 : rows ? 2 : 0;
}

// The segment rows read each byte once where the gather route reads it
// three times, but measured slower on the bench's PacketBuffer-like chains
// (latency-bound at 2 waves per SIMD), so they are
// off unless FDBXXH_SEGROWS=1 or fdbxxh_set_segrows(1) (tests) turns them on.
static int g_segrows = -1;
static bool segrows_on() {
	if (__atomic_load_n(&g_segrows, __ATOMIC_RELAXED) < 0) {
		const char* e = getenv("FDBXXH_SEGROWS");
		int expect = -1;
		__atomic_compare_exchange_n(&g_segrows, &expect, e && atoi(e) == 1 ? 1 : 0, false, __ATOMIC_RELAXED,
		                            __ATOMIC_RELAXED);
	}
	return __atomic_load_n(&g_segrows, __ATOMIC_RELAXED) == 1;
}

// The LDS route for short chains (k_xxh3_lchain) is on unless FDBXXH_LCHAIN=0
// or fdbxxh_set_lchain(0) (tests: both routes against the reference).
static int g_lchain = -1;
static bool lchain_on() {
	if (__atomic_load_n(&g_lchain, __ATOMIC_RELAXED) < 0) {
		const char* e = getenv("FDBXXH_LCHAIN");
		int expect = -1;
		__atomic_compare_exchange_n(&g_lchain, &expect, e && atoi(e) == 0 ? 0 : 1, false, __ATOMIC_RELAXED,
		                            __ATOMIC_RELAXED);
	}
	return __atomic_load_n(&g_lchain, __ATOMIC_RELAXED) == 1;
}

static uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }
// entries per XCD list: the chains of every eighth 256-chain workgroup
static uint64_t lchain_cap(uint64_t nchains) { return 256 * (((nchains + 255) / 256 + 7) / 8); }

uint64_t xxh3_chain_workspace_bytes(uint64_t nsegs, uint64_t nchains, uint64_t total_bytes, uint64_t nwave) {
	const uint64_t nb = nsegs / kScanSpan + 1;  // the scan covers nsegs + 1 entries (pre[nsegs] = total)
	return al16(8 * (nb + 1)) + al16(8 * (nsegs + 1)) + 2 * al16(8 * nchains) + al16(nsegs + 1) + al16(nchains) +
	       8 * 128 + 8 * 16 * lchain_cap(nchains) + al16(total_bytes + 16) +
	       al16(xxh3_workspace_bytes_for(nchains ? nchains : 1, nwave, xxh3_long_blocks_bound(total_bytes)));
}

int launch_xxh3_chained(const uint8_t* base, const uint64_t* seg_off, const uint64_t* seg_len, uint64_t nsegs,
                        const uint64_t* starts, uint64_t nchains, uint64_t total_bytes, uint64_t seed,
                        const uint64_t* seeds, uint64_t* out, int num_cus, void* ws, hipStream_t s) {
	const uint64_t nb = nsegs / kScanSpan + 1;
	uint8_t* p = static_cast<uint8_t*>(ws);
	uint64_t* bsum = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * (nb + 1));
	uint64_t* pre = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * (nsegs + 1));
	uint64_t* ch_off = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * nchains);
	uint64_t* ch_len = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * nchains);
	uint8_t* segflag = p;
	p += al16(nsegs + 1);
	uint8_t* chflag = p;
	p += al16(nchains);
	// the LDS route's lists: per XCD a count (its own 128-byte line) and entries
	const uint64_t lcap = lchain_cap(nchains);
	uint64_t* counts = reinterpret_cast<uint64_t*>(p);
	p += 8 * 128;
	uint64_t* list = reinterpret_cast<uint64_t*>(p);
	p += 8 * 16 * lcap;
	uint8_t* staging = p;
	p += al16(total_bytes + 16);
	void* eng = p;
	if (nsegs) {
		k_seg_bsum<<<(unsigned)nb, kScanT, 0, s>>>(seg_len, nsegs, bsum, counts);
		k_seg_bscan<<<1, kScanT, 0, s>>>(bsum, nb);
		k_seg_scan<<<(unsigned)nb, kScanT, 0, s>>>(seg_len, nsegs, bsum, pre);
	} else if (hipMemsetAsync(pre, 0, 8, s) != hipSuccess) {
		return -1;
	}
	const bool rows_on = segrows_on();
	const bool lc_on = nsegs != 0 && lchain_on();  // (nsegs == 0: no chain of two segments)
	k_chain_ranges<<<(unsigned)((nchains + 255) / 256), 256, 0, s>>>(starts, nchains, nsegs, pre, total_bytes, base,
	                                                                   seg_off, staging, segflag, ch_off, ch_len, chflag,
	                                                                   rows_on ? 1 : 0, lc_on ? 1 : 0, list, counts, lcap);
	if (nsegs) {
		const uint64_t g = (nsegs + 255) / 256;  // a wave per 64 segments
		k_seg_gather<<<(unsigned)(g < 65536 ? g : 65536), 256, 0, s>>>(base, seg_off, seg_len, pre, segflag, nsegs,
		                                                                   staging, total_bytes);
	}
	XxhParams P{};
	P.base = staging;
	P.offsets = ch_off;
	P.lengths = ch_len;
	P.count = nchains;
	P.seed = seed;
	P.seeds = seeds;
	P.out = out;
	P.ws_bytes = xxh3_workspace_bytes_for(nchains ? nchains : 1, (uint64_t)num_cus * xxh3_blocks_per_cu() * kWavesPerBlock,
	                                      xxh3_long_blocks_bound(total_bytes));
	if (launch_xxh3(P, num_cus, eng, s)) return -1;
	if (lc_on) {  // over the varlen pass's empty digests of the listed chains
		LChainP C{};
		C.base = base;
		C.seg_off = seg_off;
		C.seg_len = seg_len;
		C.list = list;
		C.counts = counts;
		C.lcap = lcap;
		C.seed = seed;
		C.seeds = seeds;
		C.out = out;
		if (launch_xxh3_lchain(C, num_cus, s)) return -1;
	}
	if (!rows_on) return 0;
	SegRowsP R{};
	R.base = base;
	R.seg_off = seg_off;
	R.seg_len = seg_len;
	R.starts = starts;
	R.flag = chflag;
	R.nchains = nchains;
	R.seed = seed;
	R.seeds = seeds;
	R.out = out;
	return launch_xxh3_segrows(R, num_cus, s);
}

}  // namespace fdbxxh

// Tests / A-B: the LDS route for short chains on (1, the default) or off (0)
// in later calls; returns the previous setting.
extern "C" int fdbxxh_set_lchain(int on) {
	const int prev = fdbxxh::lchain_on() ? 1 : 0;
	__atomic_store_n(&fdbxxh::g_lchain, on ? 1 : 0, __ATOMIC_RELAXED);
	return prev;
}

// Development / tests: hash qualifying multi-segment chains in place (1) or
// all from staging (0) in later calls; returns the previous setting.
extern "C" int fdbxxh_set_segrows(int on) {
	const int prev = fdbxxh::segrows_on() ? 1 : 0;
	__atomic_store_n(&fdbxxh::g_segrows, on ? 1 : 0, __ATOMIC_RELAXED);
	return prev;
}
