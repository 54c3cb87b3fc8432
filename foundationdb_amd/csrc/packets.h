// Device-side interface of the packet-verify kernels (packets.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fdb_packets.h"

namespace fdbpkt {

// Workspace: [0] the frame counter, then per buffer the walk's results and the
// first failing frame, per frame slot the list the walk appends to.
struct Ws {
	uint64_t* hdr;       // [0]: frames appended by the last verify (may exceed cap: then some were not
	                     // recorded; copied from fcount by k_pkt_final); [1], [2]: nbuf and max_frames of
	                     // the batch (k_pkt_walk)
	uint64_t* fcount;    // the walk's frame counter: the stream's counter word (fdbcrc::stream_aux),
	                     // zero on entry, put back to zero by k_pkt_final
	uint32_t* walked;    // per buffer: frames walked
	int32_t* wstat;      // ... why the walk stopped
	uint32_t* bad_ord;   // ... first frame whose checksum failed (~0: none)
	uint64_t* wend;      // ... bytes walked
	uint64_t* bad_pos;   // ... header position of that frame
	uint64_t* foff;      // per frame: payload offset from base
	uint64_t* flen;      // ... payload bytes
	uint64_t* fexp;      // ... the header's checksum
	uint64_t* fh;        // ... XXH3 of the payload
	uint32_t* fbuf;      // ... buffer
	uint32_t* ford;      // ... ordinal in its buffer
	uint64_t cap;
};
struct CheckP {
	const uint8_t* base;
	const uint64_t* boff;
	uint64_t nbuf;
	uint32_t hdr;
	Ws w;
	fdb_packet_result* out;
};
uint64_t workspace_bytes(uint64_t nbuf, uint64_t max_frames, uint64_t total_bytes, int num_cus);
Ws carve(void* ws, uint64_t nbuf, uint64_t max_frames, uint64_t ws_bytes, void** xws, uint64_t* xws_bytes);
// fcount: the stream's frame counter word; room_blocks: the 1 KiB blocks of
// long frames (> 16 KiB) to leave split-route room for (~0: all the
// workspace holds; long frames beyond the room are hashed by the row kernel);
// hneed (host-mapped, may be null): receives the blocks this batch's long
// frames needed.
int launch_verify(const uint8_t* base, const uint64_t* boff, const uint64_t* blen, uint64_t nbuf, int checksum,
                  uint32_t limit, uint64_t max_frames, fdb_packet_result* out, void* ws, uint64_t ws_bytes,
                  int num_cus, uint64_t* fcount, uint64_t room_blocks, uint64_t* hneed, hipStream_t s);
int launch_frames(const Ws& w, uint64_t nbuf, fdb_packet_frame* out, uint64_t capacity, uint64_t* d_n, hipStream_t s);

}  // namespace fdbpkt
