/* The scalar drop-in against the reference, the way the reference measures
 * it: flow/bench/BenchHash.cpp:48-70 times crc32c_append(0xfdbeefdb, key,
 * 2^k) for k = 2..18 on one resident key.  This loads two crc32c_append
 * symbols side by side (RTLD_LOCAL, so they do not clash) -- the library's
 * (foundationdb_amd/lib/libfdb_crc32c.so) and the reference's own
 * contrib/crc32/crc32c.cpp compiled unmodified (oracle/_ref/libcrc32c_ref.so)
 * -- and times each on the same buffer, one pinned thread, best of 7 runs of
 * ~20 ms.  Prints one JSON object per size.
 *   gcc -O2 -o build/bench_scalar tools/bench_scalar.c -ldl && build/bench_scalar [ours.so] [ref.so]
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uint32_t (*crc_fn)(uint32_t, const uint8_t*, size_t);

static double now(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9 * t.tv_nsec;
}

static crc_fn load(const char* path) {
	void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
	if (!h) {
		fprintf(stderr, "%s\n", dlerror());
		exit(2);
	}
	crc_fn f = (crc_fn)dlsym(h, "crc32c_append");
	if (!f) {
		fprintf(stderr, "no crc32c_append in %s\n", path);
		exit(2);
	}
	return f;
}

static volatile uint32_t sink;

/* ns per call, best of 7 runs of about 20 ms */
static double time_fn(crc_fn f, const uint8_t* key, size_t len) {
	size_t iters = 1;
	for (;;) {  /* calibrate */
		double t = now();
		for (size_t i = 0; i < iters; ++i) sink = f(0xfdbeefdb, key, len);
		if (now() - t > 0.02) break;
		iters *= 2;
	}
	double best = 1e30;
	for (int r = 0; r < 7; ++r) {
		double t = now();
		for (size_t i = 0; i < iters; ++i) sink = f(0xfdbeefdb, key, len);
		t = (now() - t) / iters;
		if (t < best) best = t;
	}
	return best * 1e9;
}

int main(int argc, char** argv) {
	const char* ours = argc > 1 ? argv[1] : "foundationdb_amd/lib/libfdb_crc32c.so";
	const char* ref = argc > 2 ? argv[2] : "oracle/_ref/libcrc32c_ref.so";
	crc_fn a = load(ours), b = load(ref);
	cpu_set_t set;
	CPU_ZERO(&set);
	CPU_SET(sched_getcpu(), &set);
	sched_setaffinity(0, sizeof set, &set);
	uint8_t* key = aligned_alloc(64, 1 << 18);
	uint64_t z = 0x5EED;
	for (size_t i = 0; i < (1 << 18); ++i) {
		z = z * 6364136223846793005ull + 1442695040888963407ull;
		key[i] = (uint8_t)(z >> 56);
	}
	for (int k = 2; k <= 18; ++k) {
		size_t len = (size_t)1 << k;
		if (a(0xfdbeefdb, key, len) != b(0xfdbeefdb, key, len)) {
			fprintf(stderr, "mismatch at length %zu\n", len);
			return 1;
		}
		double ta = time_fn(a, key, len), tb = time_fn(b, key, len);
		printf("{\"length\": %zu, \"ours_ns\": %.2f, \"reference_ns\": %.2f, \"ours_GBps\": %.2f, "
		       "\"reference_GBps\": %.2f, \"speedup\": %.3f}\n",
		       len, ta, tb, len / ta, len / tb, tb / ta);
	}
	return 0;
}
