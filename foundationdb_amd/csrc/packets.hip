// Batched FlowTransport receive verification (gfx950): the checksum half of
// scanPackets (fdbrpc/FlowTransport.cpp:1260-1366) over many connections'
// receive buffers at once.  A receive buffer holds frames
//     [u32 len][u64 XXH3_64bits(payload)][payload: len bytes]
// back to back ([u32 len][payload] for TLS peers, whose checksum is off,
// :1275).  The reference walks one buffer's frames in order on the network
// thread and, per complete frame, rejects len > PACKET_LIMIT (:1299-1304,
// checked before the frame's bytes have all arrived), stops at an incomplete
// frame (:1306-1307), rejects len < sizeof(UID) (:1309-1319), recomputes the
// payload's XXH3 and throws checksum_failed on a mismatch (:1346-1358); every
// frame before the one that stops or throws is delivered, and
// unprocessed_begin moves past it.
//
// Here the length walk and the hashing are separated, so the hashing is
// balanced over the whole GPU instead of one buffer per thread:
//   k_pkt_walk    one lane per receive buffer walks its frame headers -- a
//                 serial chain, each header's length locating the next --
//                 reading the header bytes only (one 16-byte load per header),
//                 and appends every complete, well-sized frame to a frame list
//                 (staged in registers, one atomic per wave every 8 steps)
//   XXH3 varlen   the frame payloads through the XXH3 engine
//                 (xxh3_kernels.hip / xxh3_split.hip), batch size read on the
//                 device from the walk's frame counter
//   k_pkt_check   per frame: a mismatch lowers its buffer's first failing
//                 ordinal (and header position) with atomicMin
//   k_pkt_final   per buffer: the reference's outcome -- the frames it
//                 delivers, the bytes it consumes, and why it stopped
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/fdb_packets.h"
#include "packets.h"
#include "xxh3_device.h"

namespace fdbpkt {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint64_t g_u64;



}  // namespace

struct WalkP {
	const uint8_t* base;
	const uint64_t* boff;
	const uint64_t* blen;
	uint64_t nbuf;
	uint32_t hdr;     // 12 (checksums on) or 4
	uint32_t limit;   // FLOW_KNOBS->PACKET_LIMIT
	Ws w;
};

// One LANE per receive buffer: each lane walks its buffer's frame headers --
// a serial chain, each header's length locating the next -- with one 16-byte
// load per header, at the header's own address (a following header inside it
// costs no load).  The walk's time is its longest chain times a load round
// trip, and the round trip grows with the requests in flight: on the bench's
// 1 GiB of Zipf packets, a 64-byte window of four aligned loads took 93 us,
// two aligned loads 73 us, one load 63 us; and 64-thread workgroups (one wave
// on each of 256 CUs, not four waves on 64) 110 -> 90 us.  The first design
// staged every buffer whole in LDS (one wave per buffer), which read the
// batch's bytes a second time: the walk was HBM-bound (257 us).
constexpr int kWalkStage = 8;  // walk steps per list flush

__global__ __launch_bounds__(256) void k_pkt_walk(WalkP P) {
	const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63;
	const bool in = b < P.nbuf;
	const uint64_t B0 = in ? reinterpret_cast<uint64_t>(P.base) + *((g_u64*)reinterpret_cast<uintptr_t>(P.boff + b)) : 0;
	const uint64_t len = in ? *((g_u64*)reinterpret_cast<uintptr_t>(P.blen + b)) : 0;
	const uint64_t E = B0 + len;
	const uint64_t last_chunk = len ? (E - 1) & ~uint64_t(15) : 0;
#ifndef FDBPKT_WIN_CHUNKS
#define FDBPKT_WIN_CHUNKS 1
#endif
	// window chunks of 16 bytes: >= 2 aligned ones (a header fits in two), or
	// one at the header's own address
	constexpr int kWinC = FDBPKT_WIN_CHUNKS;
	uint64_t wbeg = ~uint64_t(0);  // window: bytes [wbeg, wbeg + 16 kWinC)
	u32x4 win[kWinC];
	typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
	typedef __attribute__((address_space(1))) const u32x4u g_u32x4u;
	const uint64_t hi16 = (E + 15) & ~uint64_t(15);  // the end of the buffer's last 16-byte chunk
	auto restage = [&](uint64_t a) {
		if (kWinC == 1) {
			// one 16-byte load at the header itself (unaligned), moved back to end
			// at hi16 near the buffer's end: the 12-byte header stays inside it
			wbeg = a + 16 <= hi16 ? a : hi16 - 16;
			win[0] = *((g_u32x4u*)reinterpret_cast<uintptr_t>(wbeg));
			return;
		}
		wbeg = a & ~uint64_t(15);
#pragma unroll
		for (int i = 0; i < kWinC; ++i) {
			// chunks past the buffer re-read its last one (never used: the walk
			// checks every length against the buffer's end)
			const uint64_t c = wbeg + 16ull * i;
			win[i] = *((g_u32x4*)reinterpret_cast<uintptr_t>(c <= last_chunk ? c : last_chunk));
		}
	};
	// little-endian u32 at absolute address a inside the window (a - wbeg <= 16 kWinC - 4)
	auto rd32 = [&](uint64_t a) -> uint32_t {
		const uint32_t o = (uint32_t)(a - wbeg), wi = o >> 2;
		uint32_t w0 = 0, w1 = 0;
#pragma unroll
		for (uint32_t k = 0; k < 4 * kWinC; ++k) {
			const uint32_t v = win[k >> 2][k & 3];
			w0 = wi == k ? v : w0;
			w1 = wi + 1 == k ? v : w1;
		}
		return __builtin_amdgcn_alignbyte(w1, w0, o & 3u);
	};
	uint64_t p = 0;    // bytes of the buffer walked
	uint32_t ord = 0;  // frames walked
	int32_t status = FDB_PACKET_OK;
	bool live = in, overflow = false;
	uint64_t* const fcount = P.w.fcount;
	// The frames of kWalkStage steps are held in the lane's registers (slot s
	// of the unrolled group: the step index is wave-uniform) and leave together:
	// one reservation atomic per wave and group, the lane's frames contiguous
	// in the list.  Per-step reservations and stores put an atomic and a store
	// acknowledgement on the walk's chain (vmcnt counts stores and loads in
	// issue order: the next header load's wait waited for them).
	uint64_t s_off[kWalkStage], s_ck[kWalkStage];
	uint32_t s_len[kWalkStage];
	uint32_t smask = 0;
	auto step = [&](int slot) __attribute__((always_inline)) {
		if (!live) return;
		const uint64_t a = B0 + p;
		if (len - p < 4) {                                   // FlowTransport.cpp:1285-1286
			live = false;
			return;
		}
		if (P.hdr == 12 && len - p - 4 < 8) {                // :1293-1294
			live = false;
			return;
		}
		if (a < wbeg || a + P.hdr > wbeg + 16 * kWinC) restage(a);
		const uint32_t fl = rd32(a);
		if (fl > P.limit) {                                  // :1299-1304 (before the frame is complete)
			status = FDB_PACKET_LIMIT_EXCEEDED;
			live = false;
		} else if (len - p - P.hdr < fl) {                   // :1306-1307
			live = false;
		} else if (fl < 16) {                                // :1309-1319 (sizeof(UID))
			status = FDB_PACKET_TOO_SMALL;
			live = false;
		} else {
			s_ck[slot] = P.hdr == 12 ? ((uint64_t)rd32(a + 8) << 32) | rd32(a + 4) : 0;
			s_off[slot] = a + P.hdr - reinterpret_cast<uint64_t>(P.base);
			s_len[slot] = fl;
			smask |= 1u << slot;
			p += P.hdr + fl;
			++ord;
		}
	};
	auto flush = [&]() __attribute__((always_inline)) {
		const uint32_t n = (uint32_t)__builtin_popcount(smask);
		// the wave's exclusive prefix of n, and its total
		uint32_t incl = n;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t v = (uint32_t)__shfl_up((int)incl, d);
			incl += lane >= (uint32_t)d ? v : 0u;
		}
		const uint32_t total = (uint32_t)__shfl((int)incl, 63);
		if (total == 0) return;
		uint64_t at = 0;
		if (lane == 0) at = atomicAdd((unsigned long long*)fcount, (unsigned long long)total);
		at = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(at >> 32), 0) << 32) | (uint64_t)(uint32_t)__shfl((int)(uint32_t)at, 0);
		uint64_t f = at + (incl - n);
		uint32_t o = ord - n;
#pragma unroll
		for (int s = 0; s < kWalkStage; ++s) {
			if (smask & (1u << s)) {
				if (f < P.w.cap) {
					P.w.foff[f] = s_off[s];
					P.w.flen[f] = s_len[s];
					P.w.fexp[f] = s_ck[s];
					P.w.fbuf[f] = (uint32_t)b;
					P.w.ford[f] = o;
				} else {
					overflow = true;
				}
				++f;
				++o;
			}
		}
		smask = 0;
	};
	while (__ballot(live) != 0) {
#pragma unroll
		for (int s = 0; s < kWalkStage; ++s) step(s);
		flush();
	}
	if (b == 0) {  // the batch's shape, for fdb_packets_frames' check of its arguments
		P.w.hdr[1] = P.nbuf;
		P.w.hdr[2] = P.w.cap;
	}
	if (in) {
		P.w.walked[b] = ord;
		P.w.wstat[b] = overflow ? FDB_PACKET_ECAPACITY : status;
		P.w.wend[b] = p;
		P.w.bad_ord[b] = ~0u;
		P.w.bad_pos[b] = ~0ull;
	}
}

// Per frame: the digest against the header's checksum.
__global__ __launch_bounds__(256) void k_pkt_check(CheckP P) {
	const uint64_t n = *P.w.fcount < P.w.cap ? *P.w.fcount : P.w.cap;
	for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (uint64_t)gridDim.x * blockDim.x) {
		if (P.w.fh[f] != P.w.fexp[f]) {
			const uint32_t b = P.w.fbuf[f];
			atomicMin(P.w.bad_ord + b, P.w.ford[f]);
			// the frame's header position in its buffer: the bytes consumed before it
			const uint64_t pos = reinterpret_cast<uint64_t>(P.base) + P.w.foff[f] - P.hdr -
			                     (reinterpret_cast<uint64_t>(P.base) + P.boff[b]);
			atomicMin((unsigned long long*)(P.w.bad_pos + b), (unsigned long long)pos);
		}
	}
}

// Per buffer: the reference's outcome.  Thread 0 also moves the frame count
// into the workspace (fdb_packets_frames reads it there) and puts the
// stream's counter back to zero for the next call (no kernel of this launch
// reads it).
__global__ __launch_bounds__(256) void k_pkt_final(CheckP P) {
	const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (b == 0) {
		P.w.hdr[0] = *P.w.fcount;
		*P.w.fcount = 0;
	}
	if (b >= P.nbuf) return;
	const uint32_t n = P.w.walked[b], bo = P.w.bad_ord[b];
	fdb_packet_result r;
	if (bo < n) {  // the first frame that fails its checksum comes before the walk's stop
		r.consumed = P.w.bad_pos[b];
		r.frames = bo;
		r.status = FDB_PACKET_CHECKSUM_FAILED;
	} else {
		r.consumed = P.w.wend[b];
		r.frames = n;
		r.status = P.w.wstat[b];
	}
	P.out[b] = r;
}

__global__ __launch_bounds__(256) void k_pkt_frames(Ws w, uint64_t nbuf, fdb_packet_frame* out, uint64_t capacity,
                                                    uint64_t* d_n) {
	if (w.hdr[1] != nbuf || w.hdr[2] != w.cap) {  // not the shape of the last verify in this workspace
		if (blockIdx.x == 0 && threadIdx.x == 0 && d_n) *d_n = ~0ull;
		return;
	}
	const uint64_t n0 = *w.hdr < w.cap ? *w.hdr : w.cap;
	const uint64_t n = n0 < capacity ? n0 : capacity;
	if (blockIdx.x == 0 && threadIdx.x == 0 && d_n) *d_n = n0;
	for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (uint64_t)gridDim.x * blockDim.x) {
		fdb_packet_frame r;
		r.offset = w.foff[f];
		r.length = w.flen[f];
		r.checksum = w.fexp[f];
		r.buffer = w.fbuf[f];
		r.ordinal = w.ford[f];
		out[f] = r;
	}
}

int launch_frames(const Ws& w, uint64_t nbuf, fdb_packet_frame* out, uint64_t capacity, uint64_t* d_n, hipStream_t s) {
	const uint64_t g = (w.cap < capacity ? w.cap : capacity) / 256 + 1;
	k_pkt_frames<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, s>>>(w, nbuf, out, capacity, d_n);
	return 0;
}

static uint64_t a256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

uint64_t workspace_bytes(uint64_t nbuf, uint64_t max_frames, uint64_t total_bytes, int num_cus) {
	const uint64_t own = 256 + a256(4 * nbuf) * 3 + a256(8 * nbuf) * 2 + a256(8 * max_frames) * 4 +
	                     a256(4 * max_frames) * 2;
	const uint64_t xw = fdbxxh::xxh3_workspace_bytes_for(max_frames, fdbxxh::xxh3_nwave(num_cus),
	                                                     fdbxxh::xxh3_long_blocks_bound(total_bytes));
	return own + a256(xw);
}

Ws carve(void* ws, uint64_t nbuf, uint64_t max_frames, uint64_t ws_bytes, void** xws, uint64_t* xws_bytes) {
	uint8_t* p = static_cast<uint8_t*>(ws);
	Ws w{};
	w.hdr = reinterpret_cast<uint64_t*>(p);
	p += 256;
	w.walked = reinterpret_cast<uint32_t*>(p);
	p += a256(4 * nbuf);
	w.wstat = reinterpret_cast<int32_t*>(p);
	p += a256(4 * nbuf);
	w.bad_ord = reinterpret_cast<uint32_t*>(p);
	p += a256(4 * nbuf);
	w.wend = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * nbuf);
	w.bad_pos = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * nbuf);
	w.foff = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * max_frames);
	w.flen = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * max_frames);
	w.fexp = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * max_frames);
	w.fh = reinterpret_cast<uint64_t*>(p);
	p += a256(8 * max_frames);
	w.fbuf = reinterpret_cast<uint32_t*>(p);
	p += a256(4 * max_frames);
	w.ford = reinterpret_cast<uint32_t*>(p);
	p += a256(4 * max_frames);
	w.cap = max_frames;
	*xws = p;
	*xws_bytes = ws_bytes - (uint64_t)(p - static_cast<uint8_t*>(ws));
	return w;
}

int launch_verify(const uint8_t* base, const uint64_t* boff, const uint64_t* blen, uint64_t nbuf, int checksum,
                  uint32_t limit, uint64_t max_frames, fdb_packet_result* out, void* ws, uint64_t ws_bytes,
                  int num_cus, uint64_t* fcount, uint64_t room_blocks, uint64_t* hneed, hipStream_t s) {
	void* xws = nullptr;
	uint64_t xws_bytes = 0;
	Ws w = carve(ws, nbuf, max_frames, ws_bytes, &xws, &xws_bytes);
	w.fcount = fcount;
	WalkP W{};
	W.base = base;
	W.boff = boff;
	W.blen = blen;
	W.nbuf = nbuf;
	W.hdr = checksum ? 12u : 4u;
	W.limit = limit;
	W.w = w;
#ifndef FDBPKT_WALK_BLOCK
#define FDBPKT_WALK_BLOCK 64
#endif
	k_pkt_walk<<<(unsigned)((nbuf + FDBPKT_WALK_BLOCK - 1) / FDBPKT_WALK_BLOCK), FDBPKT_WALK_BLOCK, 0, s>>>(W);
	CheckP C{};
	C.base = base;
	C.boff = boff;
	C.nbuf = nbuf;
	C.hdr = W.hdr;
	C.w = w;
	C.out = out;
	if (checksum && max_frames) {
		fdbxxh::XxhParams X{};
		X.base = base;
		X.offsets = w.foff;
		X.lengths = w.flen;
		X.count = max_frames;
		X.d_count = w.fcount;
		X.out = w.fh;
		// the split route's room: none when the limit keeps every frame within
		// 16 KiB (its launch would be empty), else what the caller asks for
		const uint64_t nw = fdbxxh::xxh3_nwave(num_cus);
		uint64_t xb = xws_bytes;
		if (limit <= fdbxxh::kXSplitMin) {
			const uint64_t b0 = fdbxxh::xxh3_workspace_bytes(max_frames, nw);
			xb = xb < b0 ? xb : b0;
		} else if (room_blocks != ~0ull) {
			const uint64_t b1 = fdbxxh::xxh3_workspace_bytes_for(max_frames, nw, room_blocks);
			xb = xb < b1 ? xb : b1;
		}
		X.ws_bytes = xb;
		X.hneed = hneed;
		if (fdbxxh::launch_xxh3(X, num_cus, xws, s)) return -1;
		const uint64_t g = (max_frames + 255) / 256;
		k_pkt_check<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, s>>>(C);
	}
	k_pkt_final<<<(unsigned)((nbuf + 255) / 256), 256, 0, s>>>(C);
	return 0;
}

}  // namespace fdbpkt
