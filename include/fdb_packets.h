/*
 * Batched FlowTransport receive verification on MI355X -- C ABI of
 * libfdb_crc32c.so.
 *
 * Replaces, for receive buffers resident in device memory, the frame walk and
 * checksum check that scanPackets runs per connection on the network thread
 * (fdbrpc/FlowTransport.cpp:1260-1366).  Receive buffer b is the bytes
 * [d_base + d_buf_offsets[b], + d_buf_lengths[b]); it holds frames
 *     [u32 len][u64 XXH3_64bits(payload)][payload: len bytes]     (checksum_enabled)
 *     [u32 len][payload: len bytes]                                (TLS peers, :1275)
 * back to back, little-endian, at any alignment.  Per buffer the result is
 * what scanPackets does with it:
 *   frames    the frames it delivers (each complete, len >= 16, checksum ok)
 *   consumed  how far unprocessed_begin moves: the end of the last delivered
 *             frame (the start of the frame that stopped the walk)
 *   status    FDB_PACKET_OK                the walk stopped at an incomplete
 *                                          frame or the buffer's end (:1285-1307)
 *             FDB_PACKET_CHECKSUM_FAILED   frame `frames` failed its checksum:
 *                                          the reference throws checksum_failed (:1346-1358)
 *             FDB_PACKET_LIMIT_EXCEEDED    frame `frames` declares len > packet_limit,
 *                                          whether or not it is complete: platform_error
 *                                          (PacketLimitExceeded, :1299-1304)
 *             FDB_PACKET_TOO_SMALL         frame `frames` is complete with len < 16
 *                                          (sizeof(UID)): platform_error (PacketTooSmall, :1309-1319)
 *             FDB_PACKET_ECAPACITY         the batch has more complete frames than
 *                                          max_frames: this buffer's result is not
 *                                          known (raise max_frames and call again)
 * The checks come in the reference's order, so a checksum failure before a
 * limit or size violation is the one reported.  packet_limit is
 * FLOW_KNOBS->PACKET_LIMIT (100 MiB by default, flow/Knobs.cpp:237).
 *
 * The frames found (when d_frames is not null) are written to
 * d_frames[0 .. *d_nframes) in no particular order, each with its buffer and
 * its ordinal in that buffer: payload at d_base + offset.  A buffer's frames
 * with ordinal < result.frames are the ones delivered.
 *
 * Conventions as include/fdb_crc32c.h: device pointers, caller owns every
 * buffer, asynchronous on `stream`, return 0 or a negative FDB_CRC32C_E*.
 * The walk reads 16-byte-aligned chunks that intersect a buffer, so the bytes
 * sharing a buffer's first or last 16-byte chunk are read (never written).
 * Limits: nbuf < 2^32, buffers shorter than 2^40 bytes, total_bytes >= the sum
 * of the buffer lengths (it sizes the hashing engine's room for payloads over
 * 16 KiB).
 */
#ifndef FDB_PACKETS_H
#define FDB_PACKETS_H

#include <stdint.h>

#include "fdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
	FDB_PACKET_OK = 0,
	FDB_PACKET_CHECKSUM_FAILED = 1,
	FDB_PACKET_LIMIT_EXCEEDED = 2,
	FDB_PACKET_TOO_SMALL = 3,
	FDB_PACKET_ECAPACITY = 4
};

typedef struct fdb_packet_result {
	uint64_t consumed;
	uint32_t frames;
	int32_t status;
} fdb_packet_result;

typedef struct fdb_packet_frame {
	uint64_t offset;    /* payload, from d_base */
	uint64_t length;    /* payload bytes */
	uint64_t checksum;  /* the header's XXH3 (0 when checksums are off) */
	uint32_t buffer;
	uint32_t ordinal;
} fdb_packet_frame;

uint64_t fdb_packets_workspace_bytes(uint64_t nbuf, uint64_t max_frames, uint64_t total_bytes);
int fdb_packets_verify_ws(const void* d_base, const uint64_t* d_buf_offsets, const uint64_t* d_buf_lengths,
                          uint64_t nbuf, uint64_t total_bytes, int checksum_enabled, uint32_t packet_limit,
                          uint64_t max_frames, fdb_packet_result* d_results, void* d_workspace,
                          uint64_t workspace_bytes, void* stream);
/* Same with the library's per-stream workspace.
 * Both forms keep the walk's frame counter in a word of the stream's own
 * (zeroed when the stream is first used, put back to zero by each call's last
 * kernel: no memset per call), so calls on one stream run in stream order
 * (host threads sharing a stream are serialised by a per-stream lock held
 * through the call's last launch), and a captured graph of a call replays on
 * the stream it was captured on, one replay at a time.  The first call on a
 * stream allocates that word and is refused (FDB_CRC32C_EINVAL) inside a
 * stream capture: use the stream once outside the capture first.  Frames over
 * 16 KiB take the XXH3 split route only when the packet limit allows them and
 * the stream's previous batch had some (a host-mapped hint, no
 * synchronisation); otherwise the row kernel hashes them -- the same digests,
 * and no empty split-route launch for batches of short frames. */
int fdb_packets_verify(const void* d_base, const uint64_t* d_buf_offsets, const uint64_t* d_buf_lengths,
                       uint64_t nbuf, uint64_t total_bytes, int checksum_enabled, uint32_t packet_limit,
                       uint64_t max_frames, fdb_packet_result* d_results, void* stream);
/* The frame list of the last fdb_packets_verify_ws in d_workspace: copies up
 * to `capacity` frames into d_frames and their count (<= max_frames) into
 * *d_nframes (device u64).  nbuf and max_frames must be the ones that call
 * was given (they place the frame arrays in the workspace); with any other
 * values nothing is copied and *d_nframes is set to UINT64_MAX.  Asynchronous
 * on `stream`: launch it on the verify call's stream, or after it. */
int fdb_packets_frames(const void* d_workspace, uint64_t nbuf, uint64_t max_frames, fdb_packet_frame* d_frames,
                       uint64_t capacity, uint64_t* d_nframes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FDB_PACKETS_H */
