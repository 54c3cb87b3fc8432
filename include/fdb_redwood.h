/*
 * Batched Redwood page checks on MI355X (gfx950) -- C ABI of libfdb_crc32c.so.
 *
 * Replaces, for batches of device-resident pages, the per-page checksum work
 * of the Redwood pager's ArenaPage (fdbserver/kvstore/IPager.h):
 *   void postReadHeader(PhysicalPageID pageID, bool verify = true);  (:527-547)
 *   void postReadPayload(PhysicalPageID pageID, ...);                (:551-565)
 *   void preWrite(PhysicalPageID pageID);                            (:500-525)
 * as the pager calls them page by page (fdbserver/kvstore/VersionedBTree.cpp:
 * 1027-1028, 2595, 2842-2844, 2908-2910; IPager.cpp:37-43), built from
 *   RedwoodHeaderV1::updateChecksum / verifyChecksum   (IPager.h:297-313):
 *       XXH3_64bits(page bytes [0, payloadOffset)) with the checksum field
 *       (bytes [7, 15)) zeroed
 *   XXHashEncoder::encode / decode                     (IPager.h:318-331):
 *       XXH3_64bits_withSeed(payload, logicalSize - payloadOffset, pageID)
 * with the same byte layout (header version 1, byte-packed structs: version
 * at 0, encoding type at 1, encoding header offset at 2, payload offset at 3,
 * checksum at 7, firstPhysicalPageID at 15) and the same order of checks.
 * Results are bit-identical to the reference composition for every page
 * content, including layouts other than the writer's (payload offset 51,
 * encoding header 43).
 *
 * Conventions (include/fdb_crc32c.h): device pointers, 16-byte aligned pages
 * of page_size bytes back to back (page_size a multiple of 16, 512 .. 2^31 - 1:
 * the pager's logical page, which for a multi-block BTreeSuperNode spans
 * several physical blocks and is checked with its first block's ID), calls
 * asynchronous on `stream`, 0 or a negative FDB_CRC32C_E* status.
 * Page i's PhysicalPageID is d_page_ids[i] when d_page_ids is not NULL, else
 * first_page_id + i.
 */
#ifndef FDB_REDWOOD_H
#define FDB_REDWOOD_H

#include <stdint.h>

#include "fdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Status per page: the error the reference would throw first, or OK. */
#define FDB_REDWOOD_OK 0
#define FDB_REDWOOD_HEADER_VERSION_NOT_SUPPORTED 1 /* page_header_version_not_supported */
#define FDB_REDWOOD_HEADER_CHECKSUM_FAILED 2       /* page_header_checksum_failed */
#define FDB_REDWOOD_HEADER_WRONG_PAGE_ID 3         /* page_header_wrong_page_id */
#define FDB_REDWOOD_ENCODING_NOT_SUPPORTED 4       /* page_encoding_not_supported (also the deprecated
                                                      XOR test encoding: it needs the pager's xorWith) */
#define FDB_REDWOOD_DECODING_FAILED 5              /* page_decoding_failed */

/* postReadHeader(pageID, verify = true) then postReadPayload(pageID) for every
 * page: d_status[i] as above; *d_bad (may be NULL) = pages not OK.  Pages are
 * not modified. */
int fdb_redwood_verify_pages(const void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                             uint32_t first_page_id, uint8_t* d_status, uint64_t* d_bad, void* stream);

/* preWrite(pageID) in place for every page: the payload checksum into the
 * encoding header, then the header checksum.  d_status (may be NULL): OK,
 * ENCODING_NOT_SUPPORTED (page untouched) or HEADER_VERSION_NOT_SUPPORTED
 * (payload checksum written, header checksum not -- where the reference
 * throws). */
int fdb_redwood_seal_pages(void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                           uint32_t first_page_id, uint8_t* d_status, void* stream);

/* Caller-owned workspace forms (16-byte aligned, fdb_redwood_workspace_bytes
 * bytes): no allocation, no state outside the workspace, so calls on one
 * stream with distinct workspaces never interfere and a stream capture
 * records them. */
uint64_t fdb_redwood_workspace_bytes(uint64_t count, uint64_t page_size);
int fdb_redwood_verify_pages_ws(const void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                                uint32_t first_page_id, uint8_t* d_status, uint64_t* d_bad, void* d_workspace,
                                uint64_t workspace_bytes, void* stream);
int fdb_redwood_seal_pages_ws(void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                              uint32_t first_page_id, uint8_t* d_status, void* d_workspace, uint64_t workspace_bytes,
                              void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FDB_REDWOOD_H */
