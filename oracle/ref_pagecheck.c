/*
 * ref_pagecheck.c -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py cpu_baseline leg
 * of the verifier workloads).  The reference's page checks as FoundationDB runs
 * them, one page at a time, composed from the reference's own primitives
 * compiled unmodified into oracle/_ref/libpagecheck_ref.so:
 *   crc32c_append  contrib/crc32/crc32c.cpp:346-356
 *   XXH3_64bits    flow/xxhash.c (xxHash v0.8.0)
 *   hashlittle2    flow/Hash3.c:566
 *
 * ref_sqlite_verify_pages restates PageChecksumCodec::checksum(write = false)
 * (fdbserver/kvstore/KeyValueStoreSQLite.cpp:118-155): CRC-32C when part1 == 0,
 * then XXH3 when part1 >> 24 == 0, then hashlittle2 seeded (pgno, 0x5ca1ab1e);
 * status 1 / 2 / 3 for the check that accepted the page, 0 for a bad page.
 * ref_diskqueue_check_pages restates DiskQueue Page::checkHash
 * (fdbserver/kvstore/DiskQueue.cpp:1077-1120) by implementationVersion.
 * Both return the number of bad pages (SQLiteDB::checkAllPageChecksums,
 * KeyValueStoreSQLite.cpp:1378-1470, counts them).
 *
 * The write side, in place: ref_sqlite_seal_pages restates the codec's page
 * writes (op 6 / 7, KeyValueStoreSQLite.cpp:203-244): page 1 of a database
 * whose page size exceeds SQLITE_DEFAULT_PAGE_SIZE (1024) is first sealed as
 * a 1024-byte page (:221-224), then every page gets checksum(write = true)
 * (:107-116): XXH3_64bits of [0, pageLen - 8), part1 = (h >> 32) & 0xffffff,
 * part2 = (uint32_t)h.  ref_diskqueue_seal_pages restates Page::updateHash
 * (DiskQueue.cpp:1089-1105) by implementationVersion: V0 the hashlittle2 UID,
 * V1 hash32 = crc32c_append(0xfdbeefdb, &_unused, 4092), V2 and every other
 * version hash64 = XXH3_64bits(&magic, 4088).
 *
 * Redwood (fdbserver/kvstore/IPager.h): ref_redwood_verify_pages restates
 * ArenaPage::postReadHeader(pageID, verify = true) then postReadPayload(pageID)
 * (:527-565) -- header version 1, RedwoodHeaderV1::verifyChecksum (:303-313:
 * the checksum field at byte 7 zeroed, XXH3_64bits over [0, payloadOffset),
 * restored), firstPhysicalPageID (byte 15) == pageID, XXHashEncoder::decode
 * (:325-331: XXH3_64bits_withSeed(payload, logicalSize - payloadOffset,
 * pageID) against the u64 at the encoding header); status 0 or the first
 * failure (1 version, 2 header checksum, 3 page ID, 4 encoding, 5 decoding).
 * ref_redwood_seal_pages restates preWrite(pageID) (:500-525): encode, then
 * RedwoodHeaderV1::updateChecksum (:297-301).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length);
uint64_t XXH3_64bits(const void* data, size_t len);
uint64_t XXH3_64bits_withSeed(const void* data, size_t len, uint64_t seed);
void hashlittle2(const void* key, size_t length, uint32_t* pc, uint32_t* pb);

static uint32_t rd32(const uint8_t* p) {
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}
static uint64_t rd64(const uint8_t* p) {
	uint64_t v;
	memcpy(&v, p, 8);
	return v;
}

static void wr32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }
static void wr64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }

static void sqlite_seal(uint8_t* page, uint64_t page_len) {
	const size_t n = (size_t)page_len - 8;
	const uint64_t h = XXH3_64bits(page, n);
	wr32(page + n, (uint32_t)((h >> 32) & 0x00ffffffu));
	wr32(page + n + 4, (uint32_t)h);
}

void ref_sqlite_seal_pages(uint8_t* pages, uint64_t page_size, uint64_t count, uint32_t first_pgno) {
	for (uint64_t i = 0; i < count; ++i) {
		uint8_t* page = pages + i * page_size;
		if (first_pgno + (uint32_t)i == 1 && page_size > 1024) sqlite_seal(page, 1024);
		sqlite_seal(page, page_size);
	}
}

void ref_diskqueue_seal_pages(uint8_t* pages, uint64_t count) {
	for (uint64_t i = 0; i < count; ++i) {
		uint8_t* page = pages + 4096 * i;
		uint16_t ver;
		memcpy(&ver, page + 10, 2);
		if (ver == 0) {
			uint32_t part[2] = {0x12345678u, 0xbeefabcdu};
			hashlittle2(page + 16, 4096 - 16, &part[0], &part[1]);
			wr64(page, ((uint64_t)part[0] << 32) | part[1]);
			wr64(page + 8, 0xFDBull);
		} else if (ver == 1) {
			wr32(page, crc32c_append(0xfdbeefdbu, page + 4, 4096 - 4));
		} else {
			wr64(page, XXH3_64bits(page + 8, 4096 - 8));
		}
	}
}

static int sqlite_check(const uint8_t* page, uint64_t page_size, uint32_t pgno) {
	const size_t n = (size_t)page_size - 8;
	const uint32_t part1 = rd32(page + n), part2 = rd32(page + n + 4);
	if (part1 == 0 && part2 == crc32c_append(0xfdbeefdbu, page, n)) return 1;
	if ((part1 >> 24) == 0) {
		const uint64_t h = XXH3_64bits(page, n);
		if (part1 == (uint32_t)((h >> 32) & 0x00ffffffu) && part2 == (uint32_t)h) return 2;
	}
	uint32_t c = pgno, b = 0x5ca1ab1eu;
	hashlittle2(page, n, &c, &b);
	return (c == part1 && b == part2) ? 3 : 0;
}

uint64_t ref_sqlite_verify_pages(const uint8_t* pages, uint64_t page_size, uint64_t count, uint32_t first_pgno,
                                 uint8_t* status) {
	uint64_t bad = 0;
	for (uint64_t i = 0; i < count; ++i) {
		const int s = sqlite_check(pages + i * page_size, page_size, first_pgno + (uint32_t)i);
		status[i] = (uint8_t)s;
		bad += s == 0;
	}
	return bad;
}

/* PageHeader (DiskQueue.cpp:1047-1063, packed, 36 bytes): hash64 / hash32 at 0,
 * magic at 8, implementationVersion at 10, seq from 16. */
static int diskqueue_check(const uint8_t* page) {
	uint16_t ver;
	memcpy(&ver, page + 10, 2);
	switch (ver) {
	case 0: {
		uint32_t part[2] = {0x12345678u, 0xbeefabcdu};
		hashlittle2(page + 16, 4096 - 16, &part[0], &part[1]);
		return rd64(page) == (((uint64_t)part[0] << 32) | part[1]) && rd64(page + 8) == 0xFDBull;
	}
	case 1: return rd32(page) == crc32c_append(0xfdbeefdbu, page + 4, 4096 - 4);
	case 2: return rd64(page) == XXH3_64bits(page + 8, 4096 - 8);
	default: return 0;
	}
}

uint64_t ref_diskqueue_check_pages(const uint8_t* pages, uint64_t count, uint8_t* ok) {
	uint64_t bad = 0;
	for (uint64_t i = 0; i < count; ++i) {
		ok[i] = (uint8_t)diskqueue_check(pages + 4096 * i);
		bad += !ok[i];
	}
	return bad;
}

/* Redwood: PageHeader (4 bytes) + RedwoodHeaderV1 (39 bytes), byte-packed. */
static int redwood_check(uint8_t* page, uint64_t page_size, uint32_t id) {
	const uint8_t ver = page[0], enc = page[1], eho = page[2], po = page[3];
	if (ver != 1) return 1;
	const uint64_t saved = rd64(page + 7);
	wr64(page + 7, 0);
	const uint64_t calc = XXH3_64bits(page, po);
	wr64(page + 7, saved);
	if (saved != calc) return 2;
	if (rd32(page + 15) != id) return 3;
	if (enc != 0) return 4;
	if (rd64(page + eho) != XXH3_64bits_withSeed(page + po, (size_t)(page_size - po), id)) return 5;
	return 0;
}

uint64_t ref_redwood_verify_pages(uint8_t* pages, uint64_t page_size, uint64_t count, const uint32_t* ids,
                                  uint32_t first_id, uint8_t* status) {
	uint64_t bad = 0;
	for (uint64_t i = 0; i < count; ++i) {
		const int s = redwood_check(pages + i * page_size, page_size, ids ? ids[i] : first_id + (uint32_t)i);
		status[i] = (uint8_t)s;
		bad += s != 0;
	}
	return bad;
}

void ref_redwood_seal_pages(uint8_t* pages, uint64_t page_size, uint64_t count, const uint32_t* ids,
                            uint32_t first_id, uint8_t* status) {
	for (uint64_t i = 0; i < count; ++i) {
		uint8_t* page = pages + i * page_size;
		const uint32_t id = ids ? ids[i] : first_id + (uint32_t)i;
		const uint8_t enc = page[1], eho = page[2], po = page[3];
		if (enc != 0) {
			status[i] = 4;
			continue;
		}
		wr64(page + eho, XXH3_64bits_withSeed(page + po, (size_t)(page_size - po), id));
		if (page[0] != 1) {
			status[i] = 1;
			continue;
		}
		wr64(page + 7, 0);
		wr64(page + 7, XXH3_64bits(page, po));
		status[i] = 0;
	}
}
