/*
 * fdb_crc32c.h -- C ABI of the MI355X batched CRC-32C engine.
 *
 * Drop-in boundary for FoundationDB's CRC-32C path.  The reference exposes a
 * single C-linkage function,
 *     extern "C" uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length);
 * declared at contrib/crc32/include/crc32/crc32c.h:36-39 and implemented at
 * contrib/crc32/crc32c.cpp:346-356, from the static library `crc32`
 * (contrib/crc32/CMakeLists.txt:1) that flow links PUBLIC
 * (flow/CMakeLists.txt:125).  Every caller loops it one buffer at a time:
 *   - SQLite page codec, 4088 B, seed 0xfdbeefdb  (fdbserver/kvstore/KeyValueStoreSQLite.cpp:118-129)
 *   - AsyncFileWriteChecker, 4096 B pages, seed 0xab12fd93 (fdbrpc/AsyncFileWriteChecker.h:283-331)
 *   - DiskQueue V1 pages, 4092 B, seed 0xfdbeefdb  (fdbserver/kvstore/DiskQueue.cpp:1083-1085)
 *   - FileTransfer chained 8 KiB reads, seed 0      (fdbrpc/FileTransfer.cpp:29-37)
 *
 * This library exports that symbol unchanged (host, synchronous) and adds the
 * batched entry points the reference lacks.  All checksums are bit-identical
 * to crc32c_append for every (seed, bytes, length), including length 0
 * (returns the seed) and any alignment.
 *
 * Conventions: plain pointers and sizes only.  `d_` pointers are device
 * (HBM) pointers of the current HIP device; `h_` pointers are host pointers.
 * `stream` is a hipStream_t passed as void* (NULL = the legacy default
 * stream).  Device calls are asynchronous on `stream` and return an int
 * status: 0 on success, a negative FDB_CRC32C_E* code on failure (never a
 * silent fallback -- there is no CPU path behind the device entry points).
 */
#ifndef FDB_CRC32C_H
#define FDB_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDB_CRC32C_OK 0
#define FDB_CRC32C_EINVAL (-1)  /* bad argument (null pointer with count>0, misaligned workspace, ...) */
#define FDB_CRC32C_ENODEV (-2)  /* no HIP device / gfx950 code object not loadable */
#define FDB_CRC32C_EHIP (-3)    /* a HIP runtime call failed; see crc32c_gpu_last_error() */
#define FDB_CRC32C_ENOMEM (-4)  /* device or pinned host allocation failed */

/* ---- Scalar, host: the reference symbol -------------------------------- */

/* Replaces contrib/crc32/include/crc32/crc32c.h:36-39 (impl crc32c.cpp:346-356).
 * Same name, arguments, return value and total behaviour. */
uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length);

/* Which host implementation crc32c_append uses: "sse4.2" (the CPU has the
 * crc32 instruction; the reference's hw_available, crc32c.cpp:326-344) or
 * "sliced" (table fallback, the reference's append_table, :124-172; also
 * forced by FDB_CRC32C_FORCE_SOFTWARE=1 in the environment at load time). */
const char* crc32c_host_impl(void);

/* ---- GF(2) helpers, host ----------------------------------------------- */

/* Raw register times x^(8*nbytes) mod P: the zeros operator that the
 * reference applies by table in shift_crc (contrib/crc32/crc32c.cpp:175-178). */
uint32_t crc32c_shift(uint32_t reg, uint64_t nbytes);

/* crc32c_append(s, A||B) from crc_a = crc32c_append(s, A) and
 * crc_b = crc32c_append(0, B).  Lets independently checksummed chunks
 * reproduce the reference's chained form (fdbrpc/FileTransfer.cpp:29-37). */
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* crc32c_append(crc, <nzeros zero bytes>) in O(log nzeros). */
uint32_t crc32c_append_zeros(uint32_t crc, uint64_t nzeros);

/* ---- Batched, device-resident ------------------------------------------ */

/* Prepare the current device (upload operator tables).  Optional: every
 * device entry point does it on first use, but calling it up front keeps the
 * one synchronous upload out of a stream capture.  Thread-safe.
 * The page kernels (4 KiB / 8 KiB pages, the page verifiers) also keep a
 * small per-stream array of load-balancing counters (32 words per CU,
 * allocated and zeroed on the stream's first page batch, left at zero by
 * every launch): run one page batch on a stream before capturing it. */
int crc32c_gpu_init(void);

/* Buffer i (0 <= i < count) is the `length` bytes at d_base + i*stride.
 * Seed of buffer i: d_seeds ? d_seeds[i] : seed.  Writes d_out[i].
 * Replaces `for i: out[i] = crc32c_append(seed, base + i*stride, length)`,
 * the loop of AsyncFileWriteChecker::updateChecksumHistory
 * (fdbrpc/AsyncFileWriteChecker.h:283-331) and of a whole-file page scan
 * (SQLiteDB::checkAllPageChecksums, KeyValueStoreSQLite.cpp:1378-1470). */
int crc32c_gpu_batch_fixed(const void* d_base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                           const uint32_t* d_seeds, uint32_t* d_out, void* stream);

/* Buffer i is the d_lengths[i] bytes at d_base + d_offsets[i] (any alignment,
 * any order, overlaps allowed).  Seed as above.  Writes d_out[i].  d_base may
 * be NULL (then the offsets are absolute device addresses; a zero-length
 * buffer is never read, whatever its address -- as the reference accepts any
 * pointer for length 0).
 * Work is balanced by bytes across the GPU, so one 1 MiB buffer among many
 * 64 B packets is split over several wavefronts and merged on the device.
 * Uses a library-owned workspace per (device, stream); it is allocated on
 * first use and grown (with one stream synchronisation) when a larger batch
 * arrives.
 * Thread-safe: concurrent calls on the same stream serialise on the
 * stream's workspace from lookup to enqueue.
 * Concurrency contract: the kernels read whole 16-byte-aligned chunks, so the
 * bytes that share a buffer's first or last 16-byte chunk (outside the
 * buffer) are read too, and more than once: they must not be modified while
 * the call is in flight, or that buffer's checksum is undefined.  They are
 * never written, and they always lie in the same page as buffer bytes.
 * Limit: the engine numbers 1 KiB windows (and 4 KiB blocks) with 32-bit
 * indices, so a batch must cover fewer than 2^32 - 1 of them (about 4 TiB of
 * checksummed bytes, overlapping buffers counted once each) -- far above what
 * one GPU holds unless buffers overlap heavily.  The lengths live in device
 * memory, so such a batch is refused ON THE DEVICE: the planner reads only
 * the metadata and each buffer's first chunk, the streaming kernels read
 * nothing, the batch's checksums are undefined, and
 * crc32c_gpu_stream_status(stream) reports FDB_CRC32C_EINVAL
 * (crc32c_gpu_workspace_status for the _ws form). */
int crc32c_gpu_batch_varlen(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                            uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* stream);

/* Same, with a caller-owned device workspace (no allocation, no implicit
 * synchronisation: safe inside stream capture).  The workspace holds the
 * per-tile byte prefix and the wave map of the byte-balanced planner;
 * crc32c_gpu_varlen_workspace_bytes(count) gives its size (16-byte aligned). */
uint64_t crc32c_gpu_varlen_workspace_bytes(uint64_t count);
int crc32c_gpu_batch_varlen_ws(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                               uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace,
                               uint64_t workspace_bytes, void* stream);

/* Grouped chains: one checksum per CHAIN of non-contiguous segments, the
 * value of feeding the segments one after another through crc32c_append with
 * the running CRC as seed -- the reference's chained call sites:
 *   crc = type; crc = append(crc, param1); crc = append(crc, param2)
 *     (MutationRef checksums, fdbclient/include/fdbclient/CommitTransaction.h:302-304, 330-332)
 *   crc = 0; for each 8 KiB read: crc = append(crc, read)   (fdbrpc/FileTransfer.cpp:29-37)
 * Segment j is the d_seg_lengths[j] bytes at d_base + d_seg_offsets[j] (any
 * alignment, any order, overlaps allowed); chain c is segments
 * [d_chain_starts[c], d_chain_starts[c+1]) in that order (d_chain_starts holds
 * nchains + 1 non-decreasing values <= nsegs; an empty chain yields its seed).
 * Seed of chain c: d_seeds ? d_seeds[c] : seed.  Writes d_out[c].  Segments
 * are checksummed independently (byte-balanced over the GPU) and every chain
 * is folded on the device with GF(2) shifts: no host round trip.  The _ws form
 * takes a caller-owned workspace of crc32c_gpu_chained_workspace_bytes(nsegs)
 * bytes (16-byte aligned). */
int crc32c_gpu_batch_chained(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                             uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint32_t seed,
                             const uint32_t* d_seeds, uint32_t* d_out, void* stream);
uint64_t crc32c_gpu_chained_workspace_bytes(uint64_t nsegs);
int crc32c_gpu_batch_chained_ws(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                                uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint32_t seed,
                                const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace, uint64_t workspace_bytes,
                                void* stream);

/* Refusals made on the device (see crc32c_gpu_batch_varlen's limit).
 * crc32c_gpu_stream_status waits for `stream` and returns FDB_CRC32C_EINVAL if
 * a variable-length or chained batch enqueued on it through the
 * library-workspace entry points has been refused since the last call (and
 * clears the flag), else 0.  crc32c_gpu_workspace_status waits for `stream`
 * and returns FDB_CRC32C_EINVAL if the LAST batch planned in the caller-owned
 * workspace d_workspace (crc32c_gpu_batch_varlen_ws / _chained_ws) was
 * refused, else 0.  Both synchronise: call them off the hot path. */
int crc32c_gpu_stream_status(void* stream);
int crc32c_gpu_workspace_status(const void* d_workspace, void* stream);

/* Per-stream library state.  The library keeps, per (device, stream) it has
 * seen, the planning workspace of the convenience entry points and the page
 * kernels' counters (crc32c_gpu_stream_bytes reports how many device bytes).
 * Call crc32c_gpu_release_stream before hipStreamDestroy: it waits for the
 * stream's work and frees that state, so a later stream that reuses the handle
 * starts clean.  A stream never seen is a no-op.  Returns 0 or FDB_CRC32C_EHIP. */
int crc32c_gpu_release_stream(void* stream);
uint64_t crc32c_gpu_stream_bytes(void* stream);

/* ---- Batched, host-resident (pinned H2D -> kernel -> D2H, overlapped) -- */

/* The bytes start and end in host memory (pages read from disk, chunks of a
 * file, packets from a socket).  The pipeline cuts each submitted batch (a
 * JOB) into segments of at most `segment_bytes` (covering byte range), runs
 * them on `nstreams` HIP streams of the current device, and overlaps each
 * segment's H2D copy with the previous segments' kernels and result copies.
 * Fixed-stride batches of 4 KiB / 8 KiB pages (and the 4088 B / 4092 B page
 * windows, at the same host alignment) run the page kernel; everything else
 * the variable-length engine.  Host memory registered with
 * crc32c_host_register (or allocated pinned) is copied directly; pageable
 * memory is staged through the pipeline's pinned buffers.  A pipeline object
 * is not thread-safe; use one per thread (or per Flow run loop).
 *
 * Asynchronous form (FoundationDB's file wrappers return Futures,
 * fdbrpc/AsyncFileWriteChecker.h:59-67; the run loop must never block):
 *   crc32c_pipeline_submit_*  queue a job, start what fits on free streams,
 *                             return a ticket at once.  The host arrays (data,
 *                             offsets, lengths, seeds, out) must stay valid and
 *                             unchanged until the job completes.
 *   crc32c_pipeline_poll      non-blocking (event queries only): retire
 *                             finished segments, start queued ones, and return
 *                             1 if job `ticket` is complete (h_out filled),
 *                             0 if pending, < 0 its error.  Jobs advance only
 *                             inside poll/wait/submit calls: poll from the run
 *                             loop until it returns non-zero.
 *   crc32c_pipeline_wait      block until job `ticket` completes: 0 or < 0.
 * Synchronous form: crc32c_pipeline_varlen / _fixed = submit + wait.
 * Any buffer length is accepted (the reference's crc32c_append is total,
 * contrib/crc32/crc32c.cpp:346-356): a buffer longer than segment_bytes is
 * checksummed in segment-sized pieces on the free streams and the pieces are
 * folded on the host with crc32c_combine -- exact by CRC linearity.  (Only
 * the page verifiers need a whole page per segment: page_size <=
 * segment_bytes.) */
typedef struct fdb_crc32c_pipeline fdb_crc32c_pipeline;
int crc32c_pipeline_create(fdb_crc32c_pipeline** out, uint64_t segment_bytes, int nstreams);
void crc32c_pipeline_destroy(fdb_crc32c_pipeline* p);
int crc32c_pipeline_varlen(fdb_crc32c_pipeline* p, const void* h_base, const uint64_t* h_offsets,
                           const uint64_t* h_lengths, uint64_t count, uint32_t seed, const uint32_t* h_seeds,
                           uint32_t* h_out);
int crc32c_pipeline_fixed(fdb_crc32c_pipeline* p, const void* h_base, uint64_t stride, uint64_t length,
                          uint64_t count, uint32_t seed, const uint32_t* h_seeds, uint32_t* h_out);
int crc32c_pipeline_submit_varlen(fdb_crc32c_pipeline* p, const void* h_base, const uint64_t* h_offsets,
                                  const uint64_t* h_lengths, uint64_t count, uint32_t seed, const uint32_t* h_seeds,
                                  uint32_t* h_out, uint64_t* ticket);
int crc32c_pipeline_submit_fixed(fdb_crc32c_pipeline* p, const void* h_base, uint64_t stride, uint64_t length,
                                 uint64_t count, uint32_t seed, const uint32_t* h_seeds, uint32_t* h_out,
                                 uint64_t* ticket);
int crc32c_pipeline_poll(fdb_crc32c_pipeline* p, uint64_t ticket);
int crc32c_pipeline_wait(fdb_crc32c_pipeline* p, uint64_t ticket);
int crc32c_host_register(void* h_ptr, uint64_t bytes);
int crc32c_host_unregister(void* h_ptr);

/* Text of the last error recorded on the calling thread ("" if none). */
const char* crc32c_gpu_last_error(void);

/* Library build identification, e.g. "fdb_crc32c 0.1 gfx950". */
const char* crc32c_gpu_version(void);

#ifdef __cplusplus
}
#endif

#endif /* FDB_CRC32C_H */
