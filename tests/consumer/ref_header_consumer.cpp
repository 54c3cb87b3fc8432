// A FoundationDB-side translation unit: it includes the REFERENCE's header
// (contrib/crc32/include/crc32/crc32c.h, found via -I) and nothing of ours,
// and is linked against libfdb_crc32c.so in place of contrib/crc32's static
// library -- the link-time drop-in of include/fdb_crc32c.h.
//
// stdin, one case per line:
//   <seed> <length> <hex bytes or -> <expected crc>          known answers
//   chain <splitmix64 state> <nbytes> <read size> <expected> FileTransfer-style
//                                                            chained CRC (fdbrpc/FileTransfer.cpp:29-37)
// prints "ok <cases>" or the first mismatch.
#include <crc32/crc32c.h>

#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

static std::vector<uint8_t> splitmix64_bytes(uint64_t state, size_t nbytes) {
	std::vector<uint8_t> out((nbytes + 7) / 8 * 8);
	for (size_t k = 0; k < out.size() / 8; ++k) {
		uint64_t z = state + (k + 1) * 0x9E3779B97F4A7C15ull;
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		z ^= z >> 31;
		memcpy(&out[8 * k], &z, 8);
	}
	out.resize(nbytes);
	return out;
}

int main() {
	std::string line;
	int cases = 0;
	while (std::getline(std::cin, line)) {
		if (line.empty()) continue;
		std::istringstream in(line);
		std::string first;
		in >> first;
		uint32_t got = 0;
		unsigned long long want = 0;
		if (first == "chain") {
			unsigned long long state, nbytes, read;
			in >> state >> nbytes >> read >> want;
			std::vector<uint8_t> data = splitmix64_bytes(state, nbytes);
			for (size_t i = 0; i < nbytes; i += read)
				got = crc32c_append(got, data.data() + i, i + read <= nbytes ? read : nbytes - i);
		} else {
			unsigned long long seed = std::stoull(first), len;
			std::string hex;
			in >> len >> hex >> want;
			std::vector<uint8_t> data(len);
			for (size_t i = 0; i < len; ++i) data[i] = (uint8_t)std::stoul(hex.substr(2 * i, 2), nullptr, 16);
			got = crc32c_append((uint32_t)seed, data.data(), data.size());
		}
		if (got != want) {
			printf("mismatch on line %d: got %08x want %08llx\n", cases + 1, got, want);
			return 1;
		}
		++cases;
	}
	printf("ok %d\n", cases);
	return 0;
}
