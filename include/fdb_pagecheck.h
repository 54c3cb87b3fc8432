/*
 * Batched page-format verifiers on MI355X -- C ABI of libfdb_crc32c.so.
 *
 * fdb_sqlite_verify_pages replaces a loop of
 *   PageChecksumCodec::checksum(pageNumber, page, pageLen, write = false)
 * (fdbserver/kvstore/KeyValueStoreSQLite.cpp:100-201) over a batch of pages,
 * e.g. the whole-file scan of SQLiteDB::checkAllPageChecksums (:1378-1470).
 * Page i is bytes [d_pages + i*page_size, +page_size) with page number
 * first_pgno + i.  d_status[i]:
 *   1  the CRC-32C trailer matched   (part1 == 0, part2 == crc32c_append(0xfdbeefdb, page, page_size-8))
 *   2  the XXH3 trailer matched      (part1 >> 24 == 0, (part1, part2) == XXH3_64bits split 24/32)
 *   3  the hashlittle2 trailer matched (hashlittle2(page, page_size-8, pgno, 0x5ca1ab1e))
 *   0  corrupt (the reference returns false and raises checksum_failed)
 * checked in the reference's order, so the status is the check that the
 * reference would have accepted.
 *
 * fdb_diskqueue_check_pages replaces a loop of DiskQueue Page::checkHash
 * (fdbserver/kvstore/DiskQueue.cpp:1047-1120) over 4096-byte pages, by the
 * header's implementationVersion: V0 hashlittle2 UID, V1 CRC-32C of [4,4096),
 * V2 XXH3-64 of [8,4096); d_ok[i] = 1 when the stored hash matches, 0 otherwise.
 *
 * Both: device pointers, asynchronous on `stream`, d_bad (optional, device
 * u64) receives the number of pages that failed.  Pages must be 16-byte
 * aligned, page_size a multiple of 16 in (248, 2^31) (every page 16-byte aligned;
 * SQLite page sizes are powers of two from 512), count < 2^32.  Return
 * 0 or a negative FDB_CRC32C_E* status (crc32c_gpu_last_error() explains).
 */
#ifndef FDB_PAGECHECK_H
#define FDB_PAGECHECK_H

#include <stdint.h>

#include "fdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

int fdb_sqlite_verify_pages(const void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno,
                            uint8_t* d_status, uint64_t* d_bad, void* stream);
int fdb_diskqueue_check_pages(const void* d_pages, uint64_t count, uint8_t* d_ok, uint64_t* d_bad, void* stream);

/* Caller-owned workspace variants; size from fdb_pagecheck_workspace_bytes(count),
 * 16-byte aligned.  Every form keeps its list counters in words of the
 * stream's own (allocated and zeroed when the stream is first used, put back
 * to zero by each call's last kernel, also on an error after its first
 * launch: no memset per call).
 * Threading: calls on one stream from several host threads are serialised by
 * the library (a per-stream lock held from the counter lookup through the
 * call's last launch), whatever workspace each passes.
 * Capture: the _ws forms allocate nothing once the stream has been used; the
 * first call on a stream allocates its counters and is refused with
 * FDB_CRC32C_EINVAL inside a stream capture -- make one call on the stream
 * outside the capture first.  A captured graph uses the counters of the stream
 * it was captured on: replay it on that stream (or on one no other call is
 * using at the same time), one replay at a time. */
uint64_t fdb_pagecheck_workspace_bytes(uint64_t count);
int fdb_sqlite_verify_pages_ws(const void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno,
                               uint8_t* d_status, uint64_t* d_bad, void* d_workspace, uint64_t workspace_bytes,
                               void* stream);
int fdb_diskqueue_check_pages_ws(const void* d_pages, uint64_t count, uint8_t* d_ok, uint64_t* d_bad,
                                 void* d_workspace, uint64_t workspace_bytes, void* stream);

/* The write side, in place.  fdb_sqlite_seal_pages replaces the codec's page
 * writes (op 6 db page / op 7 journal page, KeyValueStoreSQLite.cpp:203-244)
 * over a batch: every page's trailer [page_size-8, page_size) becomes
 * PageChecksumCodec::checksum(write = true) (:107-116), XXH3_64bits of
 * [0, page_size-8) split part1 = (h >> 32) & 0xffffff, part2 = (uint32_t)h;
 * the page numbered 1 (first_pgno + i == 1) is first sealed as a 1024-byte
 * page when page_size > 1024 (SQLITE_DEFAULT_PAGE_SIZE, :221-224), exactly as
 * the codec does, so it verifies at both sizes.
 * fdb_diskqueue_seal_pages replaces Page::updateHash (DiskQueue.cpp:1089-1105,
 * called at commit, :955-965) over 4096-byte pages by implementationVersion:
 * V0 the hashlittle2 UID (bytes 8..15 become 0xFDB), V1 hash32 =
 * crc32c_append(0xfdbeefdb, page + 4, 4092), V2 -- and, as the reference's
 * switch default, every other version -- hash64 = XXH3_64bits(page + 8, 4088).
 * (checkHash then rejects versions above 2, as the reference does.)
 * Same page constraints as the verifiers; the _ws forms take a workspace of
 * fdb_pagecheck_workspace_bytes(count). */
int fdb_sqlite_seal_pages(void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno, void* stream);
int fdb_sqlite_seal_pages_ws(void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno, void* d_workspace,
                             uint64_t workspace_bytes, void* stream);
int fdb_diskqueue_seal_pages(void* d_pages, uint64_t count, void* stream);
int fdb_diskqueue_seal_pages_ws(void* d_pages, uint64_t count, void* d_workspace, uint64_t workspace_bytes,
                                void* stream);

/* The pager's codec hook (PageChecksumCodec::codec, KeyValueStoreSQLite.cpp:203-244,
 * registered through SQLite's xCodec, contrib/sqlite/sqlite3.h:3990-3996) over
 * a batch of pages of one database, in place: op 3 (page read) verifies, ops 6
 * and 7 (db page / journal page write) seal; any other op is refused with
 * FDB_CRC32C_EINVAL (the reference asserts).  reserve_size is the codec's
 * current reserve size (sizeChange): when it is not 8 (sizeof(SumType)) the
 * hook returns nullptr for every page but page 1 and leaves them untouched
 * (:225-237).  d_status[i] = 0 where codec() returns nullptr (a failed check,
 * or that reserve-size rule), else the page is returned: for reads the check
 * that accepted it (1 CRC-32C, 2 XXH3, 3 hashlittle2, as fdb_sqlite_verify_pages),
 * for writes 2 (sealed with the XXH3 trailer; page 1 also at 1024 bytes). */
int fdb_sqlite_codec_pages(void* d_pages, uint64_t page_size, uint32_t reserve_size, uint64_t count,
                           uint32_t first_pgno, int op, uint8_t* d_status, void* stream);
int fdb_sqlite_codec_pages_ws(void* d_pages, uint64_t page_size, uint32_t reserve_size, uint64_t count,
                              uint32_t first_pgno, int op, uint8_t* d_status, void* d_workspace,
                              uint64_t workspace_bytes, void* stream);

/* Host-resident pages (a file scan reading pages from disk, as
 * checkAllPageChecksums does, KeyValueStoreSQLite.cpp:1378-1470, or a DiskQueue
 * recovery reading page runs, DiskQueue.cpp:1230-1290): the same verification
 * through a crc32c_pipeline (pinned H2D -> verifier kernels -> D2H of one
 * status byte per page, overlapped over the pipeline's streams).  Host
 * pointers; *h_bad receives the number of failed pages.  The _submit forms
 * return a ticket for crc32c_pipeline_poll / crc32c_pipeline_wait (host arrays
 * must stay valid until then); the others block until done. */
int fdb_sqlite_verify_pages_host(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t page_size, uint64_t count,
                                 uint32_t first_pgno, uint8_t* h_status, uint64_t* h_bad);
int fdb_sqlite_verify_pages_host_submit(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t page_size,
                                        uint64_t count, uint32_t first_pgno, uint8_t* h_status, uint64_t* h_bad,
                                        uint64_t* ticket);
int fdb_diskqueue_check_pages_host(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t count, uint8_t* h_ok,
                                   uint64_t* h_bad);
int fdb_diskqueue_check_pages_host_submit(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t count, uint8_t* h_ok,
                                          uint64_t* h_bad, uint64_t* ticket);

#ifdef __cplusplus
}
#endif

#endif /* FDB_PAGECHECK_H */
