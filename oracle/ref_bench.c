/*
 * ref_bench.c -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py cpu_baseline leg).
 * A plain loop over the reference's own crc32c_append, linked into
 * oracle/_ref/libcrc32c_ref.so next to the unmodified contrib/crc32/crc32c.cpp,
 * so the CPU baseline times the reference path exactly as FoundationDB's
 * callers drive it: one buffer at a time (fdbrpc/AsyncFileWriteChecker.h:283-331).
 */
#include <stddef.h>
#include <stdint.h>

uint32_t crc32c_append(uint32_t crc, const uint8_t* input, size_t length);

void ref_batch_fixed(const uint8_t* base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                     uint32_t* out) {
	for (uint64_t i = 0; i < count; ++i) out[i] = crc32c_append(seed, base + i * stride, (size_t)length);
}

void ref_batch_varlen(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, uint64_t count,
                      uint32_t seed, uint32_t* out) {
	for (uint64_t i = 0; i < count; ++i) out[i] = crc32c_append(seed, base + offsets[i], (size_t)lengths[i]);
}
