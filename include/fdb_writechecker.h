/*
 * Batched lost-write checker -- C ABI of libfdb_crc32c.so.
 *
 * Mirrors fdbrpc/AsyncFileWriteChecker.h (the IAsyncFile wrapper that
 * remembers the CRC-32C of recently written 4 KiB pages and re-verifies them
 * on reads): the same page numbering (1-based, full pages only, the last
 * full page of an I/O excluded exactly as updateChecksumHistory's
 * `pageEnd` does, :283-331), the same LRU history (:107-194), the same
 * process-wide history budget (:222-227, FLOW_KNOBS->PAGE_WRITE_CHECKSUM_HISTORY),
 * the same sync/timestamp rule for verification (:244-275) and truncate
 * accounting (:76-84).  What changes is how the page checksums are computed:
 * all full pages of one I/O form one batch --
 *   host buffers:   host CRC-32C for a few pages, the pinned H2D -> kernel
 *                   -> D2H pipeline for many (fdb_wc_set_gpu_threshold),
 *   device buffers: one asynchronous crc32c_gpu_batch_fixed launch on the
 *                   checker's stream; the history update is applied, in
 *                   submission order, by fdb_wc_poll (non-blocking, call it
 *                   from the event loop) or fdb_wc_wait.
 * Times are milliseconds (the reference's transformTime(now()), :100).
 *
 * Every call returns 0 or a negative FDB_CRC32C_E* status.  A checker is
 * not thread-safe (the reference runs on the single Flow network thread).
 */
#ifndef FDB_WRITECHECKER_H
#define FDB_WRITECHECKER_H

#include <stdint.h>

#include "fdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fdb_write_checker fdb_write_checker;

/* The process-wide budget is initialised from `history_budget` by the first
 * checker created while it is unset (later values are ignored, as the
 * reference's static Optional<int>). */
int fdb_wc_create(fdb_write_checker** out, int64_t history_budget);
/* Destroying a checker returns its history entries to the budget (:205-208). */
void fdb_wc_destroy(fdb_write_checker* wc);
/* Test hook: forget the process-wide budget (the next create sets it). */
void fdb_wc_reset_budget(void);
int64_t fdb_wc_budget(void);
/* Host I/O of at least this many full pages goes through the GPU pipeline
 * (default 64); 0 disables the GPU for host buffers. */
int fdb_wc_set_gpu_threshold(fdb_write_checker* wc, uint64_t pages);

/* write(): record the checksum of every full page of [offset, offset+length)
 * of `buf`.  Pages recorded (and marked "writing") are returned through
 * pages_out[0..*n_pages) when pages_out is not NULL (capacity `cap`). */
int fdb_wc_write(fdb_write_checker* wc, const void* buf, int64_t length, int64_t offset, uint64_t now_ms,
                 uint32_t* pages_out, uint64_t cap, uint64_t* n_pages);
/* The wrapped write finished: clear the "writing" marks (:61-66). */
int fdb_wc_write_done(fdb_write_checker* wc, const uint32_t* pages, uint64_t n);
/* read() completed with `length` bytes at `offset`: verify every full page
 * against the history; *failures (optional) = lost writes detected by this read. */
int fdb_wc_read(fdb_write_checker* wc, const void* buf, int64_t length, int64_t offset, uint64_t* failures);
int fdb_wc_sync(fdb_write_checker* wc, uint64_t now_ms);
int fdb_wc_truncate(fdb_write_checker* wc, int64_t size);

/* Device-resident I/O buffers, asynchronous: the checksums are computed by
 * one batch on the checker's own stream and the history operation is queued;
 * *ticket identifies it.  d_buf must already hold the data when the call is
 * made (any producer stream synchronised) and stay valid until the ticket is
 * applied.  Host-buffer calls above first drain the queue so that every
 * operation applies in submission order. */
int fdb_wc_write_device(fdb_write_checker* wc, const void* d_buf, int64_t length, int64_t offset, uint64_t now_ms,
                        uint64_t* ticket);
int fdb_wc_read_device(fdb_write_checker* wc, const void* d_buf, int64_t length, int64_t offset, uint64_t* ticket);
/* Apply every queued operation whose checksums are ready (never blocks);
 * *applied = tickets applied so far. */
int fdb_wc_poll(fdb_write_checker* wc, uint64_t* applied);
/* Block until `ticket` (and everything before it) is applied. */
int fdb_wc_wait(fdb_write_checker* wc, uint64_t ticket);

/* Sweep: the reference's background actor (fdbrpc/AsyncFileWriteChecker.h:218-232)
 * re-reads the least recently used history page, waiting while that page is
 * being written.  As written it reads offset page*4096, one page past the
 * 1-based page's bytes [(page-1)*4096, page*4096), and a 4096-byte read there
 * covers no full page by updateChecksumHistory's rule (pageEnd excludes the
 * last full page, :287-297), so it verifies nothing.  This call gives the
 * pages such a sweep should visit, in its order: from the least recently used
 * on, stopping before the first page being written; the caller reads each
 * page's bytes [(page-1)*4096, page*4096) -- in one batch, e.g. with the
 * pipeline or a device read -- and passes them to fdb_wc_read /
 * fdb_wc_read_device, which verify synced pages and drop the verified ones. */
int fdb_wc_sweep_pages(fdb_write_checker* wc, uint32_t* pages_out, uint64_t cap, uint64_t* n);
/* Counters and history inspection. */
int fdb_wc_stats(fdb_write_checker* wc, uint64_t* checked_succeed, uint64_t* checked_fail, uint64_t* history_size,
                 uint64_t* writing);
/* 1 and the stored (checksum, timestamp) if `page` is in the history, else 0. */
int fdb_wc_history(fdb_write_checker* wc, uint32_t page, uint32_t* checksum, uint64_t* timestamp_ms);

#ifdef __cplusplus
}
#endif

#endif /* FDB_WRITECHECKER_H */
