// Batched Redwood page checks (gfx950): the checksum half of
// ArenaPage::postReadHeader / postReadPayload and ArenaPage::preWrite
// (fdbserver/kvstore/IPager.h:480-560) for whole batches of device-resident
// pages, called per page by the pager at
// fdbserver/kvstore/VersionedBTree.cpp:1027-1028, 2595, 2842-2844, 2908-2910
// and fdbserver/kvstore/IPager.cpp:37-43.
//
// Page layout, header version 1 (IPager.h:246-313, byte-packed):
//   [0] headerVersion  [1] encodingType  [2] encodingHeaderOffset  [3] payloadOffset
//   RedwoodHeaderV1 at 4: pageType, pageSubType, pageFormat, checksum u64 at 7,
//   firstPhysicalPageID u32 at 15, lastKnown(Parent)LogicalPageID, writeTime,
//   writeVersion (39 bytes: the encoding header at 43, the payload at 51 for
//   XXHash64, whose encoding header is one u64 checksum, :318-331).
// Checks, in the reference's order (a thrown error ends a page's checks):
//   headerVersion != 1                        -> page_header_version_not_supported
//   XXH3_64bits([0, payloadOffset)) with the checksum field zeroed
//     != checksum  (:297-313)                 -> page_header_checksum_failed
//   firstPhysicalPageID != pageID             -> page_header_wrong_page_id
//   encodingType != XXHash64 (the deprecated XOR test encoding needs the
//     caller's xorWith, absent here: the reference's not-present path) -> page_encoding_not_supported
//   XXH3_64bits_withSeed(payload, logicalSize - payloadOffset, pageID)
//     != the encoding header's checksum       -> page_decoding_failed
// preWrite(pageID): the payload checksum into the encoding header, then (for
// header version 1) the header checksum over [0, payloadOffset) with the
// field zeroed; encoding checked first, version second (:500-525).
//
// Kernels: k_rw_head (one thread per page: header bytes, header hash, the
// payload job), the XXH3 varlen engine over every payload with its page ID as
// seed (xxh3_kernels.hip: rows of 16 lanes, byte-unaligned payloads loaded
// dword-aligned), k_rw_verify_fin / k_rw_seal_fin (the compare, or the
// encoding-header and header-checksum stores).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "redwood.h"
#include "xxh3_device.h"

namespace fdbrw {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The default secret as little-endian u64 words (xxhash.h:2500-2511, algorithm constant).
__constant__ uint64_t kRSec[24] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
    0xcb00c391bb52283cull, 0xa32e531b8b65d088ull, 0x4ef90da297486471ull, 0xd8acdea946ef1938ull,
    0x3f349ce33f76faa8ull, 0x1d4f0bc7c7bbdcf9ull, 0x3159b4cd4be0518aull, 0x647378d9c97e9fc8ull,
    0xc3ebd33483acc5eaull, 0xeb6313faffa081c5ull, 0x49daf0b751dd0d17ull, 0x9e68d429265516d3ull,
    0xfca1477d58be162bull, 0xce31d07ad1b8f88full, 0x280416958f3acb45ull, 0x7e404bbbcafbd7afull,
};
constexpr uint64_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint64_t mulfold(uint64_t a, uint64_t b) { return a * b ^ __umul64hi(a, b); }
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t avalanche3(uint64_t h) {  // xxhash.h:2680-2685
	h ^= h >> 37;
	h *= 0x165667919E3779F9ull;
	return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t avalanche64(uint64_t h) {  // xxhash.h:1711-1718
	h ^= h >> 33;
	h *= P64_2;
	h ^= h >> 29;
	h *= P64_3;
	return h ^ (h >> 32);
}
// Secret bytes at any offset (default secret): two words and a shift.
__device__ __forceinline__ uint64_t sec64(uint32_t off) {
	const uint32_t w = off >> 3, s = (off & 7) * 8;
	const uint64_t lo = kRSec[w];
	return s ? (lo >> s) | (kRSec[w + 1] << (64 - s)) : lo;
}
__device__ __forceinline__ uint32_t sec32(uint32_t off) { return (uint32_t)sec64(off); }

// ---- the common layout: a 51-byte header in the page's first 64 bytes ----
// Bytes [O, O+8) of the 64 bytes held as 16 dwords (O a compile-time offset).
template <int O>
__device__ __forceinline__ uint64_t rd64c(const uint32_t (&w)[16]) {
	constexpr int i = O >> 2, s = O & 3;
	if constexpr (s == 0) {
		return (uint64_t)w[i] | ((uint64_t)w[i + 1] << 32);
	} else {
		const uint32_t lo = __builtin_amdgcn_alignbyte(w[i + 1], w[i], s);
		const uint32_t hi = __builtin_amdgcn_alignbyte(w[i + 2], w[i + 1], s);
		return (uint64_t)lo | ((uint64_t)hi << 32);
	}
}
template <int O, int S>
__device__ __forceinline__ uint64_t mix16c(const uint32_t (&w)[16]) {  // xxhash.h:2834-2863, seed 0
	return mulfold(rd64c<O>(w) ^ kRSec[S / 8], rd64c<O + 8>(w) ^ kRSec[S / 8 + 1]);
}
// XXH3_64bits of bytes [0, 51) (len_17to128, xxhash.h:2866-2894).
__device__ __forceinline__ uint64_t xxh3_51(const uint32_t (&w)[16]) {
	uint64_t acc = 51 * P64_1;
	acc += mix16c<16, 32>(w);
	acc += mix16c<51 - 32, 48>(w);
	acc += mix16c<0, 0>(w);
	acc += mix16c<51 - 16, 16>(w);
	return avalanche3(acc);
}

// ---- any layout: a byte image of [0, len <= 263) ----------------------------
// The page's bytes with the checksum field [7, 15) zeroed and, when sealing,
// the payload checksum written at the encoding header first (preWrite writes
// it before clearing the field, so the zeroes win where the two overlap).
struct Img {
	const uint8_t* p;
	int dlo;       // the encoding header's offset, or -1
	uint64_t dig;  // the payload checksum written there
	__device__ uint32_t byte(uint32_t k) const {
		if (k >= 7 && k < 15) return 0;
		if (dlo >= 0 && (int)k >= dlo && (int)k < dlo + 8) return (uint32_t)(dig >> (8 * (k - dlo))) & 255u;
		return p[k];
	}
	__device__ uint64_t rd64(uint32_t k) const {
		uint64_t v = 0;
		for (int b = 7; b >= 0; --b) v = (v << 8) | byte(k + b);
		return v;
	}
};
__device__ uint64_t mix16g(const Img& m, uint32_t k, uint32_t s) {
	return mulfold(m.rd64(k) ^ sec64(s), m.rd64(k + 8) ^ sec64(s + 8));
}
// XXH3_64bits (seed 0, default secret) of the image's [0, len), len <= 255:
// the closed forms and, for 241..255 bytes, the long form's single partial
// block (xxhash.h:2734-2951, 3641-3718).
__device__ uint64_t xxh3_img(const Img& m, uint32_t len) {
	if (len <= 16) {
		if (len > 8) {
			const uint64_t lo = m.rd64(0) ^ (sec64(24) ^ sec64(32));
			const uint64_t hi = m.rd64(len - 8) ^ (sec64(40) ^ sec64(48));
			return avalanche3(len + __builtin_bswap64(lo) + hi + mulfold(lo, hi));
		}
		if (len >= 4) {
			const uint64_t i1 = (uint32_t)m.rd64(0), i2 = (uint32_t)m.rd64(len - 4);
			uint64_t h = (i2 + (i1 << 32)) ^ (sec64(8) ^ sec64(16));
			h ^= rotl64(h, 49) ^ rotl64(h, 24);  // rrmxmx, xxhash.h:2692-2699
			h *= 0x9FB21C651E98DF25ull;
			h ^= (h >> 35) + len;
			h *= 0x9FB21C651E98DF25ull;
			return h ^ (h >> 28);
		}
		if (len) {
			const uint32_t c1 = m.byte(0), c2 = m.byte(len >> 1), c3 = m.byte(len - 1);
			const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
			return avalanche64((uint64_t)comb ^ (uint64_t)(sec32(0) ^ sec32(4)));
		}
		return avalanche64(sec64(56) ^ sec64(64));
	}
	if (len <= 128) {
		uint64_t acc = len * P64_1;
		if (len > 32) {
			if (len > 64) {
				if (len > 96) {
					acc += mix16g(m, 48, 96);
					acc += mix16g(m, len - 64, 112);
				}
				acc += mix16g(m, 32, 64);
				acc += mix16g(m, len - 48, 80);
			}
			acc += mix16g(m, 16, 32);
			acc += mix16g(m, len - 32, 48);
		}
		acc += mix16g(m, 0, 0);
		acc += mix16g(m, len - 16, 16);
		return avalanche3(acc);
	}
	if (len <= 240) {
		uint64_t acc = len * P64_1;
		for (uint32_t i = 0; i < 8; ++i) acc += mix16g(m, 16 * i, 16 * i);
		acc = avalanche3(acc);
		for (uint32_t i = 8; i < len / 16; ++i) acc += mix16g(m, 16 * i, 16 * (i - 8) + 3);
		acc += mix16g(m, len - 16, 136 - 17);
		return avalanche3(acc);
	}
	uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
	auto stripe = [&](uint32_t k, uint32_t s) {  // accumulate_512, xxhash.h:3474-3488
		for (uint32_t i = 0; i < 8; ++i) {
			const uint64_t v = m.rd64(k + 8 * i), x = v ^ sec64(s + 8 * i);
			acc[i ^ 1] += v;
			acc[i] += (uint64_t)(uint32_t)x * (x >> 32);
		}
	};
	for (uint32_t s = 0; s < (len - 1) / 64; ++s) stripe(64 * s, 8 * s);
	stripe(len - 64, 192 - 64 - 7);
	uint64_t r = (uint64_t)len * P64_1;
	for (uint32_t i = 0; i < 4; ++i) r += mulfold(acc[2 * i] ^ sec64(11 + 16 * i), acc[2 * i + 1] ^ sec64(19 + 16 * i));
	return avalanche3(r);
}

__device__ __forceinline__ void load64(const uint8_t* p, uint32_t (&w)[16]) {
	typedef __attribute__((address_space(1))) const u32x4 gq;
#pragma unroll
	for (int q = 0; q < 4; ++q) {
		const u32x4 v = *((gq*)reinterpret_cast<uintptr_t>(p + 16 * q));
		w[4 * q] = v[0];
		w[4 * q + 1] = v[1];
		w[4 * q + 2] = v[2];
		w[4 * q + 3] = v[3];
	}
}

constexpr uint8_t kPending = 0xFF;

}  // namespace

// One thread per page: the header checks (verify) or the encoding check
// (seal), and the page's payload job for the XXH3 engine (a page whose checks
// already failed gets an empty job).
template <bool SEAL>
__global__ __launch_bounds__(256) void k_rw_head(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                                                 const uint32_t* __restrict__ ids, uint32_t first_id, Ws w,
                                                 uint64_t* __restrict__ d_bad) {
	if (!SEAL && d_bad && blockIdx.x == 0 && threadIdx.x == 0) *d_bad = 0;  // k_rw_verify_fin counts into it
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count) return;
	const uint8_t* p = pages + i * ps;
	uint32_t h[16];
	load64(p, h);
	const uint32_t id = ids ? ids[i] : first_id + (uint32_t)i;
	const uint32_t ver = h[0] & 255u, enc = (h[0] >> 8) & 255u, eho = (h[0] >> 16) & 255u, po = h[0] >> 24;
	const bool common = po == 51 && eho == 43;
	uint8_t st = kPending;
	uint64_t expect = 0;
	if (SEAL) {
		if (enc != 0) st = kEncoding;
	} else if (ver != 1) {
		st = kVersion;
	} else {
		const uint64_t saved = rd64c<7>(h);
		uint64_t calc;
		if (common) {
			uint32_t z[16];
#pragma unroll
			for (int k = 0; k < 16; ++k) z[k] = h[k];
			z[1] &= 0x00FFFFFFu;  // bytes 7 .. 14: the checksum field, zeroed
			z[2] = 0;
			z[3] &= 0xFF000000u;
			calc = xxh3_51(z);
		} else {
			calc = xxh3_img(Img{p, -1, 0}, po);
		}
		if (saved != calc) {
			st = kHeaderChecksum;
		} else if ((uint32_t)rd64c<15>(h) != id) {
			st = kWrongPageId;
		} else if (enc != 0) {
			st = kEncoding;
		} else if (common) {
			expect = rd64c<43>(h);
		} else {  // the stored payload checksum, raw (the checksum field restored, :303-307)
			for (int b = 7; b >= 0; --b) expect = (expect << 8) | p[eho + b];
		}
	}
	w.off[i] = i * ps + po;
	w.len[i] = st == kPending ? ps - po : 0;
	w.seed[i] = id;
	if (!SEAL) w.expect[i] = expect;
	w.st[i] = st;
}

// The payload checksums against the stored ones; the status per page and the
// number of pages that failed (one add per wave).
// The compare, and the bad-page count: per thread over a grid stride, then
// one atomic per workgroup.  (One atomic per wave -- 8 Ki waves on one word,
// ~12 ns each when serialised -- took the kernel to 100 us on the bench's
// mixed batch.)
constexpr unsigned kFinGrid = 256;
__global__ __launch_bounds__(256) void k_rw_verify_fin(uint64_t count, Ws w, uint8_t* __restrict__ status,
                                                       unsigned long long* __restrict__ d_bad) {
	__shared__ uint32_t wsum[4];
	uint32_t nbad = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
		uint8_t st = w.st[i];
		if (st == kPending) st = w.hash[i] == w.expect[i] ? kOk : kDecoding;
		status[i] = st;
		nbad += st != kOk ? 1u : 0u;
	}
	if (!d_bad) return;
	for (int o = 32; o > 0; o >>= 1) nbad += (uint32_t)__shfl_xor((int)nbad, o);
	if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = nbad;
	__syncthreads();
	if (threadIdx.x == 0) {
		const uint32_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
		if (t) atomicAdd(d_bad, (unsigned long long)t);
	}
}

// preWrite: the payload checksum into the encoding header, then (header
// version 1) the header checksum over [0, payloadOffset) with the field
// zeroed.  The common layout rewrites the page's first 64-byte line whole
// (nontemporal: a partly written line costs the next pass over the pages its
// read-modify-write, pagecheck.hip k_sq_seal).
__global__ __launch_bounds__(256) void k_rw_seal_fin(uint8_t* __restrict__ pages, uint64_t ps, uint64_t count, Ws w,
                                                     uint8_t* __restrict__ status) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count) return;
	uint8_t st = w.st[i];
	if (st == kPending) {
		uint8_t* p = pages + i * ps;
		const uint64_t dig = w.hash[i];
		uint32_t h[16];
		load64(p, h);
		const uint32_t ver = h[0] & 255u, eho = (h[0] >> 16) & 255u, po = h[0] >> 24;
		if (po == 51 && eho == 43) {
			// the digest at 43 (dwords 10..12, shifted by 3 bytes)
			h[10] = (h[10] & 0x00FFFFFFu) | ((uint32_t)dig << 24);
			h[11] = (uint32_t)(dig >> 8);
			h[12] = (h[12] & 0xFF000000u) | (uint32_t)(dig >> 40);
			if (ver == 1) {
				h[1] &= 0x00FFFFFFu;
				h[2] = 0;
				h[3] &= 0xFF000000u;
				const uint64_t c = xxh3_51(h);
				h[1] |= (uint32_t)c << 24;
				h[2] = (uint32_t)(c >> 8);
				h[3] |= (uint32_t)(c >> 40);
				st = kOk;
			} else {
				st = kVersion;
			}
			typedef uint32_t u32x4n __attribute__((ext_vector_type(4)));
#pragma unroll
			for (int q = 0; q < 4; ++q)
				__builtin_nontemporal_store(u32x4n{h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]},
				                            reinterpret_cast<u32x4n*>(p + 16 * q));
		} else {
			for (int b = 0; b < 8; ++b) p[eho + b] = (uint8_t)(dig >> (8 * b));
			// (preWrite reads the version after the encoding header is written:
			// an encoding header at 0 overwrites it)
			if ((eho == 0 ? (uint32_t)(dig & 255u) : ver) == 1) {
				const uint64_t c = xxh3_img(Img{p, (int)eho, dig}, po);
				for (int b = 0; b < 8; ++b) p[7 + b] = (uint8_t)(c >> (8 * b));
				st = kOk;
			} else {
				st = kVersion;
			}
		}
	}
	if (status) status[i] = st;
}

// ---------------------------------------------------------------------------
static uint64_t al16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

static uint64_t xxh3_room(uint64_t count, uint64_t ps) {
	return ps - 51 > fdbxxh::kXSplitMin ? fdbxxh::xxh3_long_blocks_bound(count * ps) : 0;
}

uint64_t workspace_bytes(uint64_t count, uint64_t ps, int num_cus) {
	return 6 * al16(8 * count) + 16 +
	       fdbxxh::xxh3_workspace_bytes_for(count, fdbxxh::xxh3_nwave(num_cus), xxh3_room(count, ps));
}

static Ws carve(void* ws, uint64_t count, uint8_t** eng) {
	uint8_t* p = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(ws) + 15) & ~uintptr_t(15));
	Ws w;
	w.off = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * count);
	w.len = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * count);
	w.seed = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * count);
	w.hash = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * count);
	w.expect = reinterpret_cast<uint64_t*>(p);
	p += al16(8 * count);
	w.st = p;
	p += al16(8 * count);
	*eng = p;
	return w;
}

static int hash_payloads(const uint8_t* pages, uint64_t ps, uint64_t count, const Ws& w, uint8_t* eng,
                         uint64_t eng_bytes, int num_cus, hipStream_t s) {
	fdbxxh::XxhParams P{};
	P.base = pages;
	P.offsets = w.off;
	P.lengths = w.len;
	P.count = count;
	P.seeds = w.seed;
	P.out = w.hash;
	P.ws_bytes = eng_bytes;
	return fdbxxh::launch_xxh3(P, num_cus, eng, s);
}

int verify(const uint8_t* pages, uint64_t ps, uint64_t count, const uint32_t* ids, uint32_t first_id,
           uint8_t* status, uint64_t* d_bad, int num_cus, void* ws, uint64_t ws_bytes, hipStream_t s) {
	uint8_t* eng = nullptr;
	const Ws w = carve(ws, count, &eng);
	const uint64_t eng_bytes = ws_bytes - (uint64_t)(eng - static_cast<uint8_t*>(ws));
	const unsigned g = (unsigned)((count + 255) / 256);
	k_rw_head<false><<<g, 256, 0, s>>>(pages, ps, count, ids, first_id, w, d_bad);
	if (hash_payloads(pages, ps, count, w, eng, eng_bytes, num_cus, s)) return -1;
	k_rw_verify_fin<<<g < kFinGrid ? g : kFinGrid, 256, 0, s>>>(count, w, status,
	                                                        reinterpret_cast<unsigned long long*>(d_bad));
	return 0;
}

int seal(uint8_t* pages, uint64_t ps, uint64_t count, const uint32_t* ids, uint32_t first_id, uint8_t* status,
         int num_cus, void* ws, uint64_t ws_bytes, hipStream_t s) {
	uint8_t* eng = nullptr;
	const Ws w = carve(ws, count, &eng);
	const uint64_t eng_bytes = ws_bytes - (uint64_t)(eng - static_cast<uint8_t*>(ws));
	const unsigned g = (unsigned)((count + 255) / 256);
	k_rw_head<true><<<g, 256, 0, s>>>(pages, ps, count, ids, first_id, w, nullptr);
	if (hash_payloads(pages, ps, count, w, eng, eng_bytes, num_cus, s)) return -1;
	k_rw_seal_fin<<<g, 256, 0, s>>>(pages, ps, count, w, status);
	return 0;
}

}  // namespace fdbrw
