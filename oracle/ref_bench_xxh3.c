/*
 * ref_bench_xxh3.c -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py cpu_baseline leg).
 * A plain loop over the reference's own XXH3_64bits / XXH3_64bits_withSeed,
 * linked into oracle/_ref/libxxhash_ref.so next to the unmodified
 * flow/xxhash.c, one buffer at a time as FoundationDB's callers drive it
 * (fdbserver/kvstore/KeyValueStoreSQLite.cpp:112, DiskQueue.cpp:1086-1088).
 */
#include <stddef.h>
#include <stdint.h>

uint64_t XXH3_64bits(const void* data, size_t len);
uint64_t XXH3_64bits_withSeed(const void* data, size_t len, uint64_t seed);

void ref_xxh3_batch_fixed(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint64_t seed,
                          uint64_t* out) {
	if (seed == 0)
		for (uint64_t i = 0; i < count; ++i) out[i] = XXH3_64bits(base + i * stride, (size_t)length);
	else
		for (uint64_t i = 0; i < count; ++i) out[i] = XXH3_64bits_withSeed(base + i * stride, (size_t)length, seed);
}

/* The FlowTransport packet shape: one packet per (offset, length). */
void ref_xxh3_batch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count,
                           uint64_t* out) {
	for (uint64_t i = 0; i < count; ++i) out[i] = XXH3_64bits(base + offsets[i], (size_t)lengths[i]);
}
