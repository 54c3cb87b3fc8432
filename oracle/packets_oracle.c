/*
 * packets_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker of
 * fdb_packets_verify; never linked into the product).
 *
 * A plain C restatement of the receive side of FlowTransport's scanPackets
 * (fdbrpc/FlowTransport.cpp:1260-1366), one receive buffer at a time, with
 * the outcome the kernels report per buffer: frames delivered, bytes consumed
 * (how far unprocessed_begin moves) and why the walk stopped.  The hash is
 * XXH3_64bits: built twice by oracle/Makefile, over our restatement
 * (xxh3_oracle.c: liboracle_packets.so) and over the reference's own
 * flow/xxhash.c compiled unmodified (-DREF_XXH3: _ref/libpackets_ref.so).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef REF_XXH3
uint64_t XXH3_64bits(const void* data, size_t len);
static uint64_t h64(const void* p, size_t n) { return XXH3_64bits(p, n); }
#else
uint64_t oracle_xxh3_64(const void* data, size_t len, uint64_t seed);
static uint64_t h64(const void* p, size_t n) { return oracle_xxh3_64(p, n, 0); }
#endif

enum { OK = 0, CHECKSUM_FAILED = 1, LIMIT_EXCEEDED = 2, TOO_SMALL = 3 };

/* One buffer [b, e): FlowTransport.cpp:1273-1366 without the delivery. */
static void scan(const uint8_t* b, const uint8_t* e, int checksum, uint32_t limit, uint64_t* consumed,
                 uint32_t* frames, int32_t* status) {
	const uint8_t* unprocessed_begin = b;
	const uint8_t* p = b;
	uint32_t n = 0;
	int32_t st = OK;
	for (;;) {
		uint32_t packetLen;
		uint64_t packetChecksum = 0;
		if (e - p < 4) break;                         /* :1285-1286 */
		memcpy(&packetLen, p, 4);                     /* :1287 */
		p += 4;
		if (checksum) {
			if (e - p < 8) break;                     /* :1293-1294 */
			memcpy(&packetChecksum, p, 8);            /* :1295 */
			p += 8;
		}
		if (packetLen > limit) {                      /* :1299-1304: platform_error */
			st = LIMIT_EXCEEDED;
			break;
		}
		if ((uint64_t)(e - p) < packetLen) break;     /* :1306-1307 */
		if (packetLen < 16) {                         /* :1309-1319: sizeof(UID), platform_error */
			st = TOO_SMALL;
			break;
		}
		if (checksum && h64(p, packetLen) != packetChecksum) {  /* :1346-1358: checksum_failed */
			st = CHECKSUM_FAILED;
			break;
		}
		p += packetLen;                               /* the packet is delivered */
		unprocessed_begin = p;
		++n;
	}
	*consumed = (uint64_t)(unprocessed_begin - b);
	*frames = n;
	*status = st;
}

void oracle_packets_verify(const uint8_t* base, const uint64_t* boff, const uint64_t* blen, uint64_t nbuf,
                           int checksum, uint32_t limit, uint64_t* consumed, uint32_t* frames, int32_t* status) {
	for (uint64_t i = 0; i < nbuf; ++i)
		scan(base + boff[i], base + boff[i] + blen[i], checksum, limit, consumed + i, frames + i, status + i);
}
