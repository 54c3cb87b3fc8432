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
// Pipeline (all on the caller's stream): a classify kernel compacts the page
// numbers that need each algorithm into device lists, the windowed page
// kernels (crc32c_kernels.hip, xxh3_kernels.hip) checksum only those pages, a
// compare kernel writes the status, and the rare pages left undecided get
// lookup3 serially, one lane each.  Every page is read by the algorithm its
// trailer/header selects and by no other (for the SQLite fall-through, a
// page whose CRC check failed is also offered to XXH3, as in the reference).
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

// lookup3 hashlittle2 (flow/Hash3.c:566-700), one lane, 4-byte aligned data.
__device__ void hashlittle2(const uint8_t* k, uint64_t length, uint32_t* pc, uint32_t* pb) {
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + (uint32_t)length + *pc;
	c += *pb;
#define ROT(x, r) (((x) << (r)) | ((x) >> (32 - (r))))
	while (length > 12) {
		a += ld32(k);
		b += ld32(k + 4);
		c += ld32(k + 8);
		a -= c; a ^= ROT(c, 4);  c += b;
		b -= a; b ^= ROT(a, 6);  a += c;
		c -= b; c ^= ROT(b, 8);  b += a;
		a -= c; a ^= ROT(c, 16); c += b;
		b -= a; b ^= ROT(a, 19); a += c;
		c -= b; c ^= ROT(b, 4);  b += a;
		length -= 12;
		k += 12;
	}
	if (length == 0) {
		*pc = c;
		*pb = b;
		return;
	}
	// tail of 1..12 bytes: whole words where the word is complete, bytes
	// otherwise (same values as the reference's masked reads)
	uint32_t w[3] = {0, 0, 0};
	for (uint64_t i = 0; i < length; ++i) w[i >> 2] |= (uint32_t)k[i] << (8 * (i & 3));
	a += w[0];
	b += w[1];
	c += w[2];
	c ^= b; c -= ROT(b, 14);
	a ^= c; a -= ROT(c, 11);
	b ^= a; b -= ROT(a, 25);
	c ^= b; c -= ROT(b, 16);
	a ^= c; a -= ROT(c, 4);
	b ^= a; b -= ROT(a, 14);
	c ^= b; c -= ROT(b, 24);
#undef ROT
	*pc = c;
	*pb = b;
}

// ---------------------------------------------------------------------------
// SQLite
// ---------------------------------------------------------------------------
constexpr uint8_t kPending = 0xFF;

__global__ void k_sq_classify(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                              uint8_t* __restrict__ status, uint32_t* __restrict__ crc_list,
                              unsigned long long* __restrict__ ctr) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const bool in = i < count;
	const uint32_t part1 = in ? ld32(pages + i * ps + ps - 8) : 1u;
	if (in) status[i] = kPending;
	push(in && part1 == 0, (uint32_t)i, crc_list, &ctr[0]);
}

// CRC results (list order) -> status 1; then every undecided page whose part1
// has a zero top byte goes to the XXH3 list.
__global__ void k_sq_after_crc(const uint8_t* __restrict__ pages, uint64_t ps, const uint32_t* __restrict__ crc_list,
                               const unsigned long long* __restrict__ ctr, const uint32_t* __restrict__ crc_out,
                               uint8_t* __restrict__ status) {
	const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= ctr[0]) return;
	const uint64_t i = crc_list[j];
	if (crc_out[j] == ld32(pages + i * ps + ps - 4)) status[i] = 1;
}

__global__ void k_sq_xxh_classify(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                                  const uint8_t* __restrict__ status, uint32_t* __restrict__ xxh_list,
                                  unsigned long long* __restrict__ ctr) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const bool in = i < count;
	bool want = false;
	if (in && status[i] == kPending) want = (ld32(pages + i * ps + ps - 8) >> 24) == 0;
	push(want, (uint32_t)i, xxh_list, &ctr[1]);
}

__global__ void k_sq_after_xxh(const uint8_t* __restrict__ pages, uint64_t ps, const uint32_t* __restrict__ xxh_list,
                               const unsigned long long* __restrict__ ctr, const uint64_t* __restrict__ xxh_out,
                               uint8_t* __restrict__ status) {
	const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= ctr[1]) return;
	const uint64_t i = xxh_list[j];
	const uint64_t h = xxh_out[j];
	const uint8_t* t = pages + i * ps + ps - 8;
	if (ld32(t) == (uint32_t)((h >> 32) & 0x00ffffffu) && ld32(t + 4) == (uint32_t)h) status[i] = 2;
}

// Undecided pages: hashlittle2 with the page number, then the final status
// and the corrupt-page count.
__global__ void k_sq_final(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count, uint32_t first_pgno,
                           uint8_t* __restrict__ status, unsigned long long* __restrict__ ctr) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count || status[i] != kPending) return;
	const uint8_t* p = pages + i * ps;
	uint32_t c = first_pgno + (uint32_t)i, b = 0x5ca1ab1eu;
	hashlittle2(p, ps - 8, &c, &b);
	const bool ok = c == ld32(p + ps - 8) && b == ld32(p + ps - 4);
	status[i] = ok ? 3 : 0;
	if (!ok) atomicAdd(&ctr[2], 1ull);
}

__global__ void k_store_bad(const unsigned long long* __restrict__ ctr, uint64_t* __restrict__ d_bad) {
	*d_bad = ctr[2];
}

// CRC results indexed by page (page sizes other than 4 KiB: all pages were checksummed)
__global__ void k_sq_after_crc_all(const uint8_t* __restrict__ pages, uint64_t ps, uint64_t count,
                                   const uint32_t* __restrict__ crc_all, uint8_t* __restrict__ status) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count) return;
	const uint8_t* t = pages + i * ps + ps - 8;
	if (ld32(t) == 0 && crc_all[i] == ld32(t + 4)) status[i] = 1;
}

// ---------------------------------------------------------------------------
// DiskQueue (4096-byte pages)
// ---------------------------------------------------------------------------
__global__ void k_dq_classify(const uint8_t* __restrict__ pages, uint64_t count, uint8_t* __restrict__ ok,
                              uint32_t* __restrict__ v1_list, uint32_t* __restrict__ v2_list,
                              unsigned long long* __restrict__ ctr) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const bool in = i < count;
	const uint32_t ver = in ? (ld32(pages + i * 4096 + 8) >> 16) : 0xFFFFu;  // implementationVersion, bytes 10..11
	if (in) ok[i] = ver == 0 ? kPending : 0;
	push(ver == 1, (uint32_t)i, v1_list, &ctr[0]);
	push(ver == 2, (uint32_t)i, v2_list, &ctr[1]);
}

__global__ void k_dq_compare(const uint8_t* __restrict__ pages, const uint32_t* __restrict__ v1_list,
                             const uint32_t* __restrict__ v2_list, const unsigned long long* __restrict__ ctr,
                             const uint32_t* __restrict__ crc_out, const uint64_t* __restrict__ xxh_out,
                             uint8_t* __restrict__ ok) {
	const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (j < ctr[0]) {
		const uint64_t i = v1_list[j];
		ok[i] = crc_out[j] == ld32(pages + i * 4096) ? 1 : 0;
	}
	if (j < ctr[1]) {
		const uint64_t i = v2_list[j];
		ok[i] = xxh_out[j] == ld64(pages + i * 4096) ? 1 : 0;
	}
}

__global__ void k_dq_final(const uint8_t* __restrict__ pages, uint64_t count, uint8_t* __restrict__ ok,
                           unsigned long long* __restrict__ ctr) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= count) return;
	const uint8_t* p = pages + i * 4096;
	bool good = ok[i] == 1;
	if (ok[i] == kPending) {  // V0: hashlittle2 over [16, 4096) -> UID(c << 32 | b, 0xFDB)
		uint32_t c = 0x12345678u, b = 0xbeefabcdu;
		hashlittle2(p + 16, 4080, &c, &b);
		good = ld64(p) == (((uint64_t)c << 32) | b) && ld64(p + 8) == 0xFDBull;
		ok[i] = good ? 1 : 0;
	}
	if (!good) atomicAdd(&ctr[2], 1ull);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
uint64_t workspace_bytes(uint64_t count) {
	// counters, two u32 lists, u32 CRC results, u64 XXH3 results, and the
	// general engine's workspace (page sizes other than 4 KiB)
	return 64 + 4 * count + 4 * count + 4 * count + 8 * count + 64 + fdbcrc::varlen7_workspace_bytes(count, 0) + 16;
}

struct Ws {
	unsigned long long* ctr;
	uint32_t *list_a, *list_b, *crc_out;
	uint64_t* xxh_out;
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
	w.crc_out = reinterpret_cast<uint32_t*>(p);
	p += 4 * count;
	w.eng = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
	return w;
}

static unsigned blocks(uint64_t n) { return (unsigned)((n + 255) / 256); }

int sqlite_verify(const uint8_t* pages, uint64_t ps, uint64_t count, uint32_t first_pgno, uint8_t* status,
                  uint64_t* d_bad, const fdbcrc::DevTables* tabs, int num_cus, void* ws, hipStream_t s) {
	const Ws w = carve(ws, count);
	if (hipMemsetAsync(w.ctr, 0, 64, s) != hipSuccess) return -1;
	k_sq_classify<<<blocks(count), 256, 0, s>>>(pages, ps, count, status, w.list_a, w.ctr);
	const uint64_t* n_crc = reinterpret_cast<const uint64_t*>(&w.ctr[0]);
	const uint64_t* n_xxh = reinterpret_cast<const uint64_t*>(&w.ctr[1]);
	if (ps == 4096) {
		if (fdbcrc::launch_pages_window_list(pages, 4096, w.list_a, n_crc, count, 0, 8, 0xFDBEEFDBu, w.crc_out, tabs,
		                                     num_cus, s))
			return -1;
		k_sq_after_crc<<<blocks(count), 256, 0, s>>>(pages, ps, w.list_a, w.ctr, w.crc_out, status);
	} else {
		// other page sizes: every page through the general fixed-stride engine
		fdbcrc::launch_fixed_general(pages, ps, ps - 8, count, 0xFDBEEFDBu, nullptr, w.crc_out, tabs, num_cus, w.eng, s);
		k_sq_after_crc_all<<<blocks(count), 256, 0, s>>>(pages, ps, count, w.crc_out, status);
	}
	k_sq_xxh_classify<<<blocks(count), 256, 0, s>>>(pages, ps, count, status, w.list_b, w.ctr);
	fdbxxh::XxhParams P{};
	P.base = pages;
	P.stride = ps;
	P.length = ps - 8;
	P.count = count;
	P.out = w.xxh_out;
	P.idx = w.list_b;
	P.d_count = n_xxh;
	if (fdbxxh::launch_xxh3_pages_list(P, num_cus, s)) return -1;
	k_sq_after_xxh<<<blocks(count), 256, 0, s>>>(pages, ps, w.list_b, w.ctr, w.xxh_out, status);
	k_sq_final<<<blocks(count), 256, 0, s>>>(pages, ps, count, first_pgno, status, w.ctr);
	if (d_bad) k_store_bad<<<1, 1, 0, s>>>(w.ctr, d_bad);
	return 0;
}

int diskqueue_check(const uint8_t* pages, uint64_t count, uint8_t* ok, uint64_t* d_bad,
                    const fdbcrc::DevTables* tabs, int num_cus, void* ws, hipStream_t s) {
	const Ws w = carve(ws, count);
	if (hipMemsetAsync(w.ctr, 0, 64, s) != hipSuccess) return -1;
	k_dq_classify<<<blocks(count), 256, 0, s>>>(pages, count, ok, w.list_a, w.list_b, w.ctr);
	const uint64_t* n1 = reinterpret_cast<const uint64_t*>(&w.ctr[0]);
	const uint64_t* n2 = reinterpret_cast<const uint64_t*>(&w.ctr[1]);
	// V1: crc32c(0xfdbeefdb, bytes [4, 4096))
	if (fdbcrc::launch_pages_window_list(pages, 4096, w.list_a, n1, count, 4, 0, 0xFDBEEFDBu, w.crc_out, tabs, num_cus, s))
		return -1;
	// V2: XXH3_64bits(bytes [8, 4096))
	fdbxxh::XxhParams P{};
	P.base = pages + 8;
	P.stride = 4096;
	P.length = 4088;
	P.count = count;
	P.out = w.xxh_out;
	P.idx = w.list_b;
	P.d_count = n2;
	if (fdbxxh::launch_xxh3_pages_list(P, num_cus, s)) return -1;
	k_dq_compare<<<blocks(count), 256, 0, s>>>(pages, w.list_a, w.list_b, w.ctr, w.crc_out, w.xxh_out, ok);
	k_dq_final<<<blocks(count), 256, 0, s>>>(pages, count, ok, w.ctr);
	if (d_bad) k_store_bad<<<1, 1, 0, s>>>(w.ctr, d_bad);
	return 0;
}

}  // namespace fdbpc
