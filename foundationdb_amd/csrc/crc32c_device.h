// Shared between the HIP kernels and the host engine: the compact operator
// tables that each workgroup expands into its bank-replicated LDS image.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include <mutex>

namespace fdbcrc {

// Window engine (crc32c_varlen.hip): slots per table (4 slots per pass, 16
// passes: two blocks in ping-pong, so the next table's first pass lands in the
// first block again).
constexpr uint32_t kV7TabSlots = 64u;

struct DevTables {
	uint32_t slice[2][256];     // [0] byte + one zero byte (T1), [1] single byte (T0)
	uint32_t block[8][16];      // nibble tables of x^(8*4096): block-to-block shift
	uint32_t lane[64][8][16];   // nibble tables of x^(8*64*(63-l)): lane l to end of block
	uint32_t slice4[4][256];    // [k]: byte followed by 3-k zero bytes (4-byte slicing T3..T0)
	uint32_t inv_z[16][8][16];  // nibble tables of x^(-8z), z = 0..15: drop z trailing zero bytes
	uint32_t pow2[64][8][16];   // nibble tables of x^(8*2^m): shift by arbitrary byte counts
	uint32_t corr[4][16][8][16];  // x^(-8(z + 1024(3-t))): quarter t's team value -> piece register, minus z zeros
	// varlen v7 (1 KiB window slots, 64 slots per table)
	uint32_t table_shift[8][16];     // x^(8*1024*kV7TabSlots): a piece's register carried across a table
	uint32_t slotw[64][16][8][16];   // x^(8*(1024*(d-3) - z)): slot sum of pass p -> its buffer's end
	                                 // (d = last slot - 4p, z trailing zeros)
	uint32_t carryw[64][16][8][16];  // x^(8*(1024*(k+1) - z)): a register carried into a table -> its
	                                 // buffer's end at slot k
	uint32_t chunkpow[256][8][16];   // x^(8*16*(255-c)): 16-byte chunk c of a pass block to the block's end
	// big-buffer block route: block k (from the buffer's end) -> the buffer's end
	uint32_t bpow[4][256][8][16];    // [i][j]: x^(8*4096*j*256^i)
	// extent route (crc32c_extent.hip)
	uint32_t xinv64[65][8][16];      // x^(-8*64*j): a prefix positioned at the block end -> back to lane span j before it
	uint32_t pow64[64][8][16];       // x^(8*64*c)
	uint32_t pow1[64][8][16];        // x^(8*d)   (with pow64 and bpow: x^(8*len) for any len < 2^40)
	// strided page layout (k_pages4k<..., STRIDED>): lane l's chain over the page's dwords at 4l + 256k
	uint32_t stride4[4][256];        // [k]: byte k of a register word times x^(8*256) (one 256-byte stride)
	uint32_t lane_s[64][8][16];      // x^(-8*4l): lane l's chain end (4l + 4096) back to the page end
};

// Build the tables on the host (crc32c_tables.cpp).
void build_dev_tables(DevTables* t);

// Grab counters of the page kernels (crc32c_kernels.hip): kPageCtrWords words
// per workgroup, owned by the launch stream (page kernels on one stream run in
// order), zero between launches.  Allocated on a stream's first page launch.
constexpr uint32_t kPageCtrWords = 32;

// Static per-workgroup ranges of k_pages4k weighted by XCD parity: workgroup b
// runs on XCD b % 8, and per-wave timestamps put the odd XCDs' workgroups ~6 %
// behind the even ones' on equal ranges (1 Mi pages: 603-612 us on XCDs
// 0/2/4/6, 641-646 us on 1/3/5/7), so an even workgroup's range is kXcdEvenW /
// kXcdOddW as long (after: 621-635 us on every XCD; bench 0.686 -> 0.676 ms).
// The same weighting in k_xgrab and k_bigblocks measured neutral (their grabs
// are finer), so they keep equal ranges.  [g0, g1) of n items.
#ifndef FDBCRC_XCD_EVEN_W
#define FDBCRC_XCD_EVEN_W 33
#define FDBCRC_XCD_ODD_W 31
#endif
constexpr uint64_t kXcdEvenW = FDBCRC_XCD_EVEN_W, kXcdOddW = FDBCRC_XCD_ODD_W;  // (32nds)
struct XcdRanges {
	uint64_t n, pe, po;  // items; an even / odd workgroup's range
	__device__ __forceinline__ XcdRanges(uint64_t n_, uint64_t G) : n(n_) {
		const uint64_t ne = (G + 1) / 2, no = G / 2;
		const uint64_t den = ne * kXcdEvenW + no * kXcdOddW;
		const uint64_t unit = (n * 32 + den - 1) / den;
		pe = (unit * kXcdEvenW + 31) / 32;
		po = (unit * kXcdOddW + 31) / 32;
	}
	__device__ __forceinline__ void get(uint64_t b, uint64_t& g0, uint64_t& g1) const {
		const uint64_t s0 = ((b + 1) / 2) * pe + (b / 2) * po;  // the even and odd workgroups before b
		const uint64_t e0 = s0 + ((b & 1) ? po : pe);
		g0 = s0 < n ? s0 : n;
		g1 = e0 < n ? e0 : n;
	}
};
__device__ __forceinline__ void xcd_range(uint64_t n, uint64_t b, uint64_t G, uint64_t& g0, uint64_t& g1) {
	XcdRanges(n, G).get(b, g0, g1);
}
int page_counters(hipStream_t stream, int num_cus, uint32_t** ctr);  // crc32c_capi.cpp
// per-stream counter words (crc32c_capi.cpp: stream_aux), zero between calls
constexpr uint64_t kAuxBytes = 256;
constexpr int kAuxPktFrames = 0;  // u64: the packet verifier's frame counter
constexpr int kAuxPageCtr = 8;    // u64[8]: the page verifiers' list counters and failures
// hold (may be null): receives the stream's counter lock, to be kept until the
// call's last kernel using the counters is enqueued
int stream_aux(hipStream_t stream, uint64_t** aux, std::unique_lock<std::mutex>* hold = nullptr);

int launch_pages(int blocks_per_page, const uint8_t* base, uint64_t stride, uint64_t count, uint32_t seed,
                 const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream);
// Bytes [h, 4096 - t) of 4 KiB pages (h, t < 16); `pages` 16-byte aligned.
int launch_pages_window(const uint8_t* pages, uint64_t stride, uint64_t count, uint32_t h, uint32_t t, uint32_t seed,
                        const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, hipStream_t stream);
int launch_pages_window_list(const uint8_t* pages, uint64_t stride, const uint32_t* idx, const uint64_t* d_count,
                             uint64_t max_count, uint32_t h, uint32_t t, uint32_t seed, uint32_t* out,
                             const DevTables* tabs, int num_cus, hipStream_t stream);
// Variable-length engine (crc32c_varlen.hip).  ws: varlen_workspace_bytes().
// route: which streaming kernels run.  kRouteBoth: spans of 4 KiB or more on
// 4 KiB blocks (k_bigblocks), the rest on 1 KiB window slots (k_varlen7);
// kRouteWindows: windows only; kRouteBlocks: blocks only.  Every route gives
// the same checksums; it only decides speed (and which launches a batch pays).
// hstat (host-mapped, may be null) receives the first 256 buffers' bytes by
// span class: [0] 128 B < span < 4 KiB, [1] 4 KiB - 16 KiB, [2] 16 KiB and
// more (route_for_stats() turns them into the next batch's route: blocks
// when 16 KiB+ spans hold most bytes -- alone if no span is under 4 KiB --,
// else windows).
// kRouteExtent: the batch looks PACKED (buffers ascending, no overlaps, small
// gaps -- packets back to back in a receive buffer, chunks of a file): the
// extent route (crc32c_extent.hip) streams the whole covering byte range as
// 4 KiB blocks and derives every buffer's CRC from two prefix registers; the
// device checks the packing first (k_v7count), and a batch that is not packed
// (or whose extent outgrew the stream's arrays) is checksummed buffer by
// buffer by the finishing kernel's fallback -- correct, slow, and the stream's
// next kXfailBackoff batches leave the route (kHstatXfail).
enum : int { kRouteBoth = 0, kRouteWindows = 1, kRouteBlocks = 2, kRouteExtent = 3 };
// Host-mapped per-stream words (u64 indices): [0..2] span classes of the last
// batch's first 256 buffers, [3] extent blocks the last extent-checked batch
// needed, [4] 1 if the last batch's first 256 buffers were packed, [5] 1 if
// the last extent-route batch failed the full packing check, [6] refusal flag.
constexpr int kHstatNblk = 3, kHstatPacked = 4, kHstatXfail = 5;
// After a batch fails the extent route's packing check, the stream's next
// kXfailBackoff batches that look packed still take the window engine (each
// window/block-route batch counts the word down), then the route is tried again.
constexpr uint64_t kXfailBackoff = 16;
inline int route_for_stats(const volatile uint64_t* s) {
	const uint64_t win = s[0], mid = s[1], large = s[2];
	const bool big = large != 0 && large >= win + mid;  // 16 KiB+ spans hold most bytes: the block route's ground
	// packed batches of packets take the extent route; packed batches of big
	// buffers (file chunks) stay on the blocks, which measured faster for them
	// (chunks: 0.204 ms on blocks, 0.220 ms on the extent: its finishing pass
	// and the fallback's guarded launches cost more than the blocks' padding)
	if (s[kHstatPacked] == 1 && s[kHstatXfail] == 0 && !big) return kRouteExtent;
	if (!big) return kRouteWindows;  // (nothing windowed at all: windows, the cheaper launch)
	return win == 0 ? kRouteBlocks : kRouteBoth;
}
// Extent route state of one stream (device memory owned by the library):
// xhdr[0] the epoch of the last launch whose batch was found not packed,
// xhdr[1] the epoch of the last launch whose extent exceeded kXMaxExtent;
// per buffer its start and end points' captured values {G, Y}; per wave of
// the streaming kernel its range's aggregate register.
constexpr uint64_t kXMaxExtent = 1ull << 40;  // 32-bit block numbers with room
// Grabs of the dynamic stream kernel (k_xgrab): kXGrabMin blocks, more when the
// extent has more than capg grabs of that size, so the per-grab arrays never
// overflow whatever the extent.
#ifndef FDBX_GRAB_MIN
#define FDBX_GRAB_MIN 8
#endif
constexpr uint64_t kXGrabMin = FDBX_GRAB_MIN;
// k_xgrab reads the next grab's window start on a grab's last step and sets it
// up on its first step: a grab needs at least two steps of 4 blocks
static_assert(kXGrabMin >= 8 && (kXGrabMin & (kXGrabMin - 1)) == 0, "grabs: a power of two of at least 8 blocks");
// (a power of two: grab numbers are shifts, not 64-bit divisions)
__host__ __device__ inline uint64_t x_gsz(uint64_t nblk, uint64_t capg) {
	uint64_t gsz = kXGrabMin;
	while (capg && (nblk + gsz - 1) / gsz > capg) gsz <<= 1;
	return gsz;
}
__host__ __device__ inline uint32_t x_log2(uint64_t v) {  // v a power of two
	uint32_t l = 0;
	while ((1ull << l) < v) ++l;
	return l;
}
constexpr uint64_t kXGrabCap = 1ull << 18;  // grabs the per-stream state holds (2 MiB)
// u64 word of xhdr (256 bytes) from which the extent route's count kernel
// stages the route statistics (hstat's layout, words 0..kHstatPacked): k_xfin
// copies them to the stream's host-mapped words beside its back-off word, so
// the count kernel touches no host memory (its PCIe read-modify-write of the
// back-off word and the system-scope release cost ~2 us of a ~6 us kernel)
constexpr int kXStage = 8;
struct XState {
	uint32_t* xhdr;
	uint32_t* ps;         // per buffer, 2 words: its start point's G and Y (k_xstream)
	uint32_t* pe;         // ... its end point's
	uint32_t* dummy;      // 128 words per wave of the stream kernel
	uint32_t* ragg;       // per stream wave: the range-local prefix at its range's end (k_xstream)
	uint32_t* wq;         // per grab: the first buffer ending past its start (k_v7count; k_xgrab)
	uint32_t* gagg;       // per grab: its grab-local prefix at its end (k_xgrab)
	uint64_t capg;        // grabs wq / gagg hold
	uint32_t* ctr;        // the stream's page-kernel grab counters (k_xgrab); null: static ranges
	uint32_t epoch;       // this launch (never 0)
};
uint64_t extent_state_bytes(uint64_t count, uint64_t capg, int num_cus);
void extent_state_carve(void* mem, uint64_t count, uint64_t capg, int num_cus, XState* x);
uint64_t varlen_workspace_bytes(uint64_t count, uint64_t nwave);
// err (device-visible, may be null): set to 1 (never cleared here) when the
// planner refuses the batch -- 2^32 - 1 or more 1 KiB windows or 4 KiB route
// blocks, which its 32-bit indices cannot number.  A refused batch writes no
// checksums (the streaming kernels do nothing); the refusal is also left in
// the workspace: varlen_refused_word(ws) is 1 after such a batch, else 0.
int launch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count, uint32_t seed,
                  const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, void* ws,
                  hipStream_t stream, int route = kRouteBoth, uint64_t* hstat = nullptr, uint32_t* err = nullptr,
                  const XState* xs = nullptr, uint32_t* bacc = nullptr, uint32_t* pctr = nullptr);
inline const uint64_t* varlen_refused_word(const void* ws) { return static_cast<const uint64_t*>(ws) + 6; }
// Fixed stride, any length/alignment (same engine, same workspace size as varlen).
int launch_fixed_general(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                         const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus, void* ws,
                         hipStream_t stream);
// v7 workspace and launch (ws: varlen7_workspace_bytes(count, nwave), 16-byte aligned)
uint64_t varlen7_workspace_bytes(uint64_t count, uint64_t nwave);
int launch_varlen7(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t stride,
                   uint64_t length, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                   const DevTables* tabs, int num_cus, void* ws, hipStream_t stream, int route, uint64_t* hstat,
                   uint32_t* err = nullptr, const XState* xs = nullptr, uint32_t* bacc = nullptr,
                   uint32_t* pctr = nullptr);
// The extent route's streaming and finishing kernels (crc32c_extent.hip),
// launched by launch_varlen7 for kRouteExtent after the packing check.
int launch_extent(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t stride,
                  uint64_t length, uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out,
                  const DevTables* tabs, int num_cus, const XState& xs, uint64_t* hstat, hipStream_t stream,
                  int phase);
// Grouped chains (crc32c_chain.hip): out[c] = fold of segments [starts[c], starts[c+1])
// whose independent registers segcrc[j] = crc32c_append(0xffffffff, segment j).
int launch_chain_fold(const uint64_t* starts, uint64_t nchains, const uint64_t* lengths, const uint32_t* segcrc,
                      uint32_t seed, const uint32_t* seeds, uint32_t* out, const DevTables* tabs, int num_cus,
                      hipStream_t stream);
// Big-buffer block route (crc32c_kernels.hip): buffers the varlen prep kernel
// routed to 4 KiB blocks aligned to their end.  Entry q of the route's list
// (in buffer order) is buffer ent[q].idx: its blocks are [ent[q].s,
// ent[q+1].s) of the route (hdr[2] blocks, hdr[3] entries in total), ent[q].E
// is its end rounded up to 16 bytes, ent[q].lot = lo/16 | k0 << 8 | t << 12
// (lo: bytes of its first block before its first 16-byte chunk, k0: its start
// mod 16, t: bytes from its end to E) and ent[q].sd = ~seed.  out[] starts at ~0 (prep); every block
// XORs in its raw register weighted to the buffer's end.
struct BigEnt {     // one routed buffer (24 bytes: one dwordx4 + one dwordx2 load per lane)
	uint64_t E;     // end rounded up to 16 bytes
	uint32_t s;     // first block of the route
	uint32_t idx;   // output index
	uint32_t lot;   // lo / 16 | k0 << 8 | t << 12
	uint32_t sd;    // ~seed
};
struct BigParams {
	const uint64_t* hdr;
	const BigEnt* ent;
	uint32_t* out;
	uint32_t* ctr;  // kPageCtrWords per workgroup, zeroed by prep (prep-free form: by the previous launch)
	const DevTables* tabs;
	// Prep-free form (k_bigblocks<U, true>: the block route alone, lists of at
	// most kNPMax buffers, 8 per thread): the batch's own metadata, read by
	// every workgroup
	const uint8_t* base;
	const uint64_t* offsets;
	const uint64_t* lengths;
	uint64_t nbuf;
	uint32_t seed;
	const uint32_t* seeds;
	uint32_t* acc;   // [kNPMax] parts' XORs, [kNPMax] blocks done (zero between launches), u64[4] statistics
	BigEnt* priv;    // route entries of workgroup w's blocks at q + 2w (its sentinel included)
	uint64_t* hstat;
	uint32_t* err;
};
constexpr uint64_t kNPMax = 6144;  // (k_bigblocks<U, true> keeps 5 words per buffer in LDS before its table fill)
constexpr uint64_t kNPAccBytes = 8 * kNPMax + 32;  // P.acc
int launch_bigblocks_np(const BigParams& P, int num_cus, hipStream_t stream);
constexpr uint64_t kBigMax = 1ull << 40;  // spans routed are below this (block index from the end < 2^28)
int launch_bigblocks(const BigParams& P, int num_cus, hipStream_t stream);
int launch_fill_seeds(uint64_t count, uint32_t seed, const uint32_t* seeds, uint32_t* out, hipStream_t stream);

}  // namespace fdbcrc
