/*
 * CPU restatement of XXH3_64bits / XXH3_64bits_withSeed (xxHash v0.8.0, as
 * vendored at flow/include/flow/xxhash.h) and of Bob Jenkins' lookup3
 * hashlittle2 (flow/Hash3.c) -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this file (through oracle/oracle.py); the product path never links it.
 * Parity is pinned by the reference's own code compiled unmodified into
 * oracle/_ref/libxxhash_ref.so (tests/golden/make_golden.py) and by the
 * known answers printed in flow/Hash3.c:1248-1263 (driver5).
 *
 * Plain scalar C written for clarity, one function per reference routine;
 * each cites the lines it restates.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* xxhash.h:1166-1168, 1678-1687 */
#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull

/* The 192-byte default secret, xxhash.h:2500-2511 (algorithm constant). */
static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint32_t swap32(uint32_t x) { return __builtin_bswap32(x); }
static uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }

/* xxhash.h:2665-2668 */
static uint64_t mul128_fold64(uint64_t a, uint64_t b) {
	const unsigned __int128 p = (unsigned __int128)a * b;
	return (uint64_t)p ^ (uint64_t)(p >> 64);
}

/* xxhash.h:1711-1718 */
static uint64_t xxh64_avalanche(uint64_t h) {
	h ^= h >> 33;
	h *= P64_2;
	h ^= h >> 29;
	h *= P64_3;
	h ^= h >> 32;
	return h;
}

/* xxhash.h:2680-2685 */
static uint64_t xxh3_avalanche(uint64_t h) {
	h ^= h >> 37;
	h *= 0x165667919E3779F9ull;
	h ^= h >> 32;
	return h;
}

/* xxhash.h:2692-2699 */
static uint64_t rrmxmx(uint64_t h, uint64_t len) {
	h ^= rotl64(h, 49) ^ rotl64(h, 24);
	h *= 0x9FB21C651E98DF25ull;
	h ^= (h >> 35) + len;
	h *= 0x9FB21C651E98DF25ull;
	return h ^ (h >> 28);
}

/* xxhash.h:2734-2806: lengths 0..16 */
static uint64_t len_0to16(const uint8_t* in, size_t len, const uint8_t* sec, uint64_t seed) {
	if (len > 8) { /* :2775-2790 */
		const uint64_t f1 = (rd64(sec + 24) ^ rd64(sec + 32)) + seed;
		const uint64_t f2 = (rd64(sec + 40) ^ rd64(sec + 48)) - seed;
		const uint64_t lo = rd64(in) ^ f1;
		const uint64_t hi = rd64(in + len - 8) ^ f2;
		return xxh3_avalanche(len + swap64(lo) + hi + mul128_fold64(lo, hi));
	}
	if (len >= 4) { /* :2757-2773 */
		seed ^= (uint64_t)swap32((uint32_t)seed) << 32;
		const uint32_t i1 = rd32(in), i2 = rd32(in + len - 4);
		const uint64_t flip = (rd64(sec + 8) ^ rd64(sec + 16)) - seed;
		return rrmxmx(((uint64_t)i2 + ((uint64_t)i1 << 32)) ^ flip, len);
	}
	if (len) { /* :2734-2755 */
		const uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
		const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
		const uint64_t flip = (uint64_t)(rd32(sec) ^ rd32(sec + 4)) + seed;
		return xxh64_avalanche((uint64_t)comb ^ flip);
	}
	return xxh64_avalanche(seed ^ (rd64(sec + 56) ^ rd64(sec + 64))); /* :2804 */
}

/* xxhash.h:2834-2863 */
static uint64_t mix16(const uint8_t* in, const uint8_t* sec, uint64_t seed) {
	return mul128_fold64(rd64(in) ^ (rd64(sec) + seed), rd64(in + 8) ^ (rd64(sec + 8) - seed));
}

/* xxhash.h:2866-2894 */
static uint64_t len_17to128(const uint8_t* in, size_t len, const uint8_t* sec, uint64_t seed) {
	uint64_t acc = len * P64_1;
	if (len > 32) {
		if (len > 64) {
			if (len > 96) {
				acc += mix16(in + 48, sec + 96, seed);
				acc += mix16(in + len - 64, sec + 112, seed);
			}
			acc += mix16(in + 32, sec + 64, seed);
			acc += mix16(in + len - 48, sec + 80, seed);
		}
		acc += mix16(in + 16, sec + 32, seed);
		acc += mix16(in + len - 32, sec + 48, seed);
	}
	acc += mix16(in, sec, seed);
	acc += mix16(in + len - 16, sec + 16, seed);
	return xxh3_avalanche(acc);
}

/* xxhash.h:2898-2951 (start offset 3, last offset 17, secret size min 136) */
static uint64_t len_129to240(const uint8_t* in, size_t len, const uint8_t* sec, uint64_t seed) {
	uint64_t acc = len * P64_1;
	const int rounds = (int)len / 16;
	for (int i = 0; i < 8; ++i) acc += mix16(in + 16 * i, sec + 16 * i, seed);
	acc = xxh3_avalanche(acc);
	for (int i = 8; i < rounds; ++i) acc += mix16(in + 16 * i, sec + 16 * (i - 8) + 3, seed);
	acc += mix16(in + len - 16, sec + 136 - 17, seed);
	return xxh3_avalanche(acc);
}

/* xxhash.h:3474-3488: one 64-byte stripe into the 8 accumulators */
static void accumulate_512(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
	for (int i = 0; i < 8; ++i) {
		const uint64_t v = rd64(in + 8 * i);
		const uint64_t k = v ^ rd64(sec + 8 * i);
		acc[i ^ 1] += v;
		acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
	}
}

/* xxhash.h:3490-3503 */
static void scramble(uint64_t acc[8], const uint8_t* sec) {
	for (int i = 0; i < 8; ++i) {
		uint64_t a = acc[i];
		a ^= a >> 47;
		a ^= rd64(sec + 8 * i);
		acc[i] = a * P32_1;
	}
}

/* xxhash.h:3641-3676 (192-byte secret: 16 stripes = 1 KiB per block),
 * 3678-3700 mergeAccs, 3702-3718 hashLong_64b_internal */
static uint64_t hash_long(const uint8_t* in, size_t len, const uint8_t* sec) {
	uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
	const size_t block = 1024, nblocks = (len - 1) / block;
	for (size_t n = 0; n < nblocks; ++n) {
		for (size_t s = 0; s < 16; ++s) accumulate_512(acc, in + n * block + 64 * s, sec + 8 * s);
		scramble(acc, sec + 192 - 64);
	}
	const size_t stripes = ((len - 1) - block * nblocks) / 64;
	for (size_t s = 0; s < stripes; ++s) accumulate_512(acc, in + nblocks * block + 64 * s, sec + 8 * s);
	accumulate_512(acc, in + len - 64, sec + 192 - 64 - 7);
	uint64_t r = (uint64_t)len * P64_1;
	for (int i = 0; i < 4; ++i)
		r += mul128_fold64(acc[2 * i] ^ rd64(sec + 11 + 16 * i), acc[2 * i + 1] ^ rd64(sec + 11 + 16 * i + 8));
	return xxh3_avalanche(r);
}

/* xxhash.h:3800-3837: XXH3_64bits_internal / XXH3_64bits / XXH3_64bits_withSeed;
 * long inputs with a nonzero seed use the custom secret of :3550-3566 */
uint64_t oracle_xxh3_64(const void* data, size_t len, uint64_t seed) {
	const uint8_t* in = (const uint8_t*)data;
	if (len <= 16) return len_0to16(in, len, kSecret, seed);
	if (len <= 128) return len_17to128(in, len, kSecret, seed);
	if (len <= 240) return len_129to240(in, len, kSecret, seed);
	if (seed == 0) return hash_long(in, len, kSecret);
	uint8_t sec[192];
	for (int i = 0; i < 12; ++i) {
		const uint64_t lo = rd64(kSecret + 16 * i) + seed, hi = rd64(kSecret + 16 * i + 8) - seed;
		memcpy(sec + 16 * i, &lo, 8);
		memcpy(sec + 16 * i + 8, &hi, 8);
	}
	return hash_long(in, len, sec);
}

/* ------------------------------------------------------------------------ */
/* lookup3 hashlittle2, flow/Hash3.c:566-700 (little-endian byte semantics:
 * the aligned, unaligned and byte-wise branches of the reference all compute
 * the same function of the bytes). */
#define ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))
void oracle_hashlittle2(const void* key, size_t length, uint32_t* pc, uint32_t* pb) {
	const uint8_t* k = (const uint8_t*)key;
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + (uint32_t)length + *pc;
	c += *pb;
	while (length > 12) { /* Hash3.c:589-596 with mix() of :118-138 */
		a += rd32(k);
		b += rd32(k + 4);
		c += rd32(k + 8);
		a -= c; a ^= ROT(c, 4);  c += b;
		b -= a; b ^= ROT(a, 6);  a += c;
		c -= b; c ^= ROT(b, 8);  b += a;
		a -= c; a ^= ROT(c, 16); c += b;
		b -= a; b ^= ROT(a, 19); a += c;
		c -= b; c ^= ROT(b, 4);  b += a;
		length -= 12;
		k += 12;
	}
	if (length == 0) { /* :650-653 */
		*pc = c;
		*pb = b;
		return;
	}
	uint8_t t[12] = {0};
	memcpy(t, k, length); /* the masked tail reads of :608-648 */
	a += rd32(t);
	b += rd32(t + 4);
	c += rd32(t + 8);
	/* final(), :165-181 */
	c ^= b; c -= ROT(b, 14);
	a ^= c; a -= ROT(c, 11);
	b ^= a; b -= ROT(a, 25);
	c ^= b; c -= ROT(b, 16);
	a ^= c; a -= ROT(c, 4);
	b ^= a; b -= ROT(a, 14);
	c ^= b; c -= ROT(b, 24);
	*pc = c;
	*pb = b;
}

/* ------------------------------------------------------------------------ */
/* Batch drivers (checker side): fixed stride or (offset, length) lists. */
struct job {
	const uint8_t* base;
	const uint64_t* off;
	const uint64_t* len;
	uint64_t stride, length, lo, hi, seed;
	const uint64_t* seeds;
	uint64_t* out;
};

static void* run(void* p) {
	const struct job* j = (const struct job*)p;
	for (uint64_t i = j->lo; i < j->hi; ++i) {
		const uint8_t* q = j->off ? j->base + j->off[i] : j->base + i * j->stride;
		const uint64_t n = j->len ? j->len[i] : j->length;
		j->out[i] = oracle_xxh3_64(q, n, j->seeds ? j->seeds[i] : j->seed);
	}
	return NULL;
}

static void batch(struct job proto, uint64_t count, int threads) {
	if (threads < 1) threads = 1;
	if (threads > 64) threads = 64;
	pthread_t th[64];
	struct job jobs[64];
	for (int t = 0; t < threads; ++t) {
		jobs[t] = proto;
		jobs[t].lo = count * t / threads;
		jobs[t].hi = count * (t + 1) / threads;
		pthread_create(&th[t], NULL, run, &jobs[t]);
	}
	for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

void oracle_xxh3_batch_fixed(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint64_t seed,
                             const uint64_t* seeds, uint64_t* out, int threads) {
	struct job j = {base, NULL, NULL, stride, length, 0, 0, seed, seeds, out};
	batch(j, count, threads);
}

void oracle_xxh3_batch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count,
                              uint64_t seed, const uint64_t* seeds, uint64_t* out, int threads) {
	struct job j = {base, offsets, lengths, 0, 0, 0, 0, seed, seeds, out};
	batch(j, count, threads);
}
