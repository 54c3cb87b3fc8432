// Host-resident batches: pinned H2D copies, device checksums, D2H results,
// overlapped across streams.  This is the path FoundationDB's callers actually
// have -- pages come from disk (KAIO, fdbrpc/AsyncFileKAIO.h:694), backup
// chunks from files (fdbrpc/FileTransfer.cpp:29-37), packets from sockets --
// so the checksum of host bytes must include the PCIe transfer.
//
// A batch is cut into segments of consecutive buffers whose covering byte
// range is at most `segment_bytes`; segment k goes to stream k % nstreams:
//   hipMemcpyAsync H2D (covering range)  ->  varlen kernel (offsets rebased)
//   ->  hipMemcpyAsync D2H (4 B per buffer)
// With >= 2 streams, segment k+1's H2D overlaps segment k's kernel and D2H;
// the engine is PCIe-bound by design (the kernel runs ~100x faster than the
// link).  Host memory should be pinned (crc32c_host_register / hipHostMalloc);
// pageable memory is staged through the pipeline's own pinned buffers.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/fdb_crc32c.h"
#include "crc32c_device.h"

namespace fdbcrc {
int device_tables(const DevTables** tabs, int* num_cus);  // crc32c_capi.cpp
int set_error(int code, const char* what, hipError_t e);  // crc32c_capi.cpp
}  // namespace fdbcrc

using namespace fdbcrc;

struct fdb_crc32c_pipeline {
	int device = 0;
	uint64_t seg_bytes = 0;
	uint64_t max_bufs = 0;  // buffers per segment (metadata capacity)
	struct Lane {
		hipStream_t stream = nullptr;
		uint8_t* d_data = nullptr;
		uint64_t* d_meta = nullptr;  // [max_bufs offsets][max_bufs lengths]
		uint32_t* d_seeds = nullptr;
		uint32_t* d_out = nullptr;
		void* d_ws = nullptr;
		uint64_t ws_bytes = 0;
		uint64_t* h_meta = nullptr;  // pinned
		uint32_t* h_seeds = nullptr; // pinned
		uint8_t* h_stage = nullptr;  // pinned staging for pageable sources
		hipEvent_t done = nullptr;
		bool busy = false;
	};
	std::vector<Lane> lanes;
};

namespace {

int hip_fail(const char* what, hipError_t e) { return set_error(FDB_CRC32C_EHIP, what, e); }

bool is_pinned(const void* p) {
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	return a.type == hipMemoryTypeHost;
}

}  // namespace

extern "C" {

int crc32c_host_register(void* h_ptr, uint64_t bytes) {
	hipError_t e = hipHostRegister(h_ptr, bytes, hipHostRegisterDefault);
	return e == hipSuccess ? 0 : hip_fail("hipHostRegister", e);
}

int crc32c_host_unregister(void* h_ptr) {
	hipError_t e = hipHostUnregister(h_ptr);
	return e == hipSuccess ? 0 : hip_fail("hipHostUnregister", e);
}

int crc32c_pipeline_create(fdb_crc32c_pipeline** out, uint64_t segment_bytes, int nstreams) {
	if (!out || nstreams < 1 || nstreams > 16) return set_error(FDB_CRC32C_EINVAL, "pipeline_create: bad args", hipSuccess);
	if (segment_bytes < (1u << 20)) segment_bytes = 1u << 20;
	const DevTables* tabs;
	int cus;
	if (int rc = device_tables(&tabs, &cus)) return rc;
	auto* p = new fdb_crc32c_pipeline;
	(void)hipGetDevice(&p->device);
	p->seg_bytes = segment_bytes;
	p->max_bufs = segment_bytes / 64 + 1024;  // >= 64 B average per buffer
	p->lanes.resize(nstreams);
	for (auto& L : p->lanes) {
		hipError_t e;
		if ((e = hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking)) != hipSuccess ||
		    (e = hipMalloc(&L.d_data, segment_bytes)) != hipSuccess ||
		    (e = hipMalloc(&L.d_meta, 16 * p->max_bufs)) != hipSuccess ||
		    (e = hipMalloc(&L.d_seeds, 4 * p->max_bufs)) != hipSuccess ||
		    (e = hipMalloc(&L.d_out, 4 * p->max_bufs)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_meta, 16 * p->max_bufs, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_seeds, 4 * p->max_bufs, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipEventCreateWithFlags(&L.done, hipEventDisableTiming)) != hipSuccess) {
			crc32c_pipeline_destroy(p);
			return set_error(FDB_CRC32C_ENOMEM, "pipeline_create: allocation", e);
		}
		L.ws_bytes = crc32c_gpu_varlen_workspace_bytes(p->max_bufs);
		if ((e = hipMalloc(&L.d_ws, L.ws_bytes)) != hipSuccess) {
			crc32c_pipeline_destroy(p);
			return set_error(FDB_CRC32C_ENOMEM, "pipeline_create: workspace", e);
		}
	}
	*out = p;
	return 0;
}

void crc32c_pipeline_destroy(fdb_crc32c_pipeline* p) {
	if (!p) return;
	for (auto& L : p->lanes) {
		if (L.stream) (void)hipStreamSynchronize(L.stream);
		if (L.d_data) (void)hipFree(L.d_data);
		if (L.d_meta) (void)hipFree(L.d_meta);
		if (L.d_seeds) (void)hipFree(L.d_seeds);
		if (L.d_out) (void)hipFree(L.d_out);
		if (L.d_ws) (void)hipFree(L.d_ws);
		if (L.h_meta) (void)hipHostFree(L.h_meta);
		if (L.h_seeds) (void)hipHostFree(L.h_seeds);
		if (L.h_stage) (void)hipHostFree(L.h_stage);
		if (L.done) (void)hipEventDestroy(L.done);
		if (L.stream) (void)hipStreamDestroy(L.stream);
	}
	delete p;
}

int crc32c_pipeline_varlen(fdb_crc32c_pipeline* p, const void* h_base, const uint64_t* h_offsets,
                           const uint64_t* h_lengths, uint64_t count, uint32_t seed, const uint32_t* h_seeds,
                           uint32_t* h_out) {
	if (count == 0) return 0;
	if (!p || !h_base || !h_offsets || !h_lengths || !h_out)
		return set_error(FDB_CRC32C_EINVAL, "pipeline_varlen: null pointer", hipSuccess);
	int cur_dev = -1;
	(void)hipGetDevice(&cur_dev);
	if (cur_dev != p->device) (void)hipSetDevice(p->device);
	const uint8_t* base = static_cast<const uint8_t*>(h_base);
	const bool pinned = is_pinned(h_base);
	uint64_t i = 0;
	size_t k = 0;
	int rc = 0;
	while (i < count && rc == 0) {
		auto& L = p->lanes[k % p->lanes.size()];
		if (L.busy) {  // retire this lane's previous segment before reusing its buffers
			hipError_t e = hipEventSynchronize(L.done);
			if (e != hipSuccess) { rc = hip_fail("hipEventSynchronize", e); break; }
			L.busy = false;
		}
		// segment: consecutive buffers whose covering range fits seg_bytes
		uint64_t lo = ~0ull, hi = 0, n = 0;
		while (i + n < count && n < p->max_bufs) {
			const uint64_t o = h_offsets[i + n], l = h_lengths[i + n];
			const uint64_t nlo = std::min(lo, l ? o : lo), nhi = std::max(hi, l ? o + l : hi);
			if (l > p->seg_bytes) {
				if (n == 0) { rc = set_error(FDB_CRC32C_EINVAL, "pipeline_varlen: buffer larger than segment", hipSuccess); }
				break;
			}
			if (n && nhi > nlo && nhi - nlo > p->seg_bytes) break;
			lo = nlo; hi = nhi;
			++n;
		}
		if (rc) break;
		if (hi < lo) lo = hi = 0;  // all empty
		const uint64_t span = hi - lo;
		for (uint64_t j = 0; j < n; ++j) {
			L.h_meta[j] = h_lengths[i + j] ? h_offsets[i + j] - lo : 0;
			L.h_meta[p->max_bufs + j] = h_lengths[i + j];
		}
		if (h_seeds) memcpy(L.h_seeds, h_seeds + i, 4 * n);
		hipError_t e = hipSuccess;
		const uint8_t* src = base + lo;
		if (!pinned && span) {
			if (!L.h_stage && (e = hipHostMalloc(&L.h_stage, p->seg_bytes, hipHostMallocDefault)) != hipSuccess) {
				rc = set_error(FDB_CRC32C_ENOMEM, "pipeline: staging", e);
				break;
			}
			memcpy(L.h_stage, src, span);
			src = L.h_stage;
		}
		if (span && (e = hipMemcpyAsync(L.d_data, src, span, hipMemcpyHostToDevice, L.stream)) != hipSuccess) {
			rc = hip_fail("H2D data", e); break;
		}
		if ((e = hipMemcpyAsync(L.d_meta, L.h_meta, 8 * n, hipMemcpyHostToDevice, L.stream)) != hipSuccess ||
		    (e = hipMemcpyAsync(L.d_meta + p->max_bufs, L.h_meta + p->max_bufs, 8 * n, hipMemcpyHostToDevice,
		                        L.stream)) != hipSuccess) {
			rc = hip_fail("H2D metadata", e); break;
		}
		if (h_seeds && (e = hipMemcpyAsync(L.d_seeds, L.h_seeds, 4 * n, hipMemcpyHostToDevice, L.stream)) != hipSuccess) {
			rc = hip_fail("H2D seeds", e); break;
		}
		rc = crc32c_gpu_batch_varlen_ws(L.d_data, L.d_meta, L.d_meta + p->max_bufs, n, seed, h_seeds ? L.d_seeds : nullptr,
		                                L.d_out, L.d_ws, L.ws_bytes, L.stream);
		if (rc) break;
		if ((e = hipMemcpyAsync(h_out + i, L.d_out, 4 * n, hipMemcpyDeviceToHost, L.stream)) != hipSuccess) {
			rc = hip_fail("D2H results", e); break;
		}
		if ((e = hipEventRecord(L.done, L.stream)) != hipSuccess) { rc = hip_fail("hipEventRecord", e); break; }
		L.busy = true;
		i += n;
		++k;
	}
	for (auto& L : p->lanes) {
		if (L.busy) {
			hipError_t e = hipEventSynchronize(L.done);
			if (e != hipSuccess && rc == 0) rc = hip_fail("hipEventSynchronize", e);
			L.busy = false;
		}
	}
	if (cur_dev != p->device) (void)hipSetDevice(cur_dev);
	return rc;
}

int crc32c_pipeline_fixed(fdb_crc32c_pipeline* p, const void* h_base, uint64_t stride, uint64_t length,
                          uint64_t count, uint32_t seed, const uint32_t* h_seeds, uint32_t* h_out) {
	// expressed through the varlen path in chunks of offsets (host-side, cheap)
	const uint64_t B = 1 << 16;
	std::vector<uint64_t> off(std::min(count, B)), len(std::min(count, B), length);
	for (uint64_t i0 = 0; i0 < count; i0 += B) {
		const uint64_t n = std::min(B, count - i0);
		for (uint64_t j = 0; j < n; ++j) off[j] = (i0 + j) * stride;
		if (int rc = crc32c_pipeline_varlen(p, h_base, off.data(), len.data(), n, seed, h_seeds ? h_seeds + i0 : nullptr,
		                                    h_out + i0))
			return rc;
	}
	return 0;
}

}  // extern "C"
