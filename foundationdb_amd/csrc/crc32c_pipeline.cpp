// Host-resident batches: pinned H2D copies, device checksums, D2H results,
// overlapped across streams.  This is the path FoundationDB's callers actually
// have -- pages come from disk (KAIO, fdbrpc/AsyncFileKAIO.h:694), backup
// chunks from files (fdbrpc/FileTransfer.cpp:29-37), packets from sockets --
// so the checksum of host bytes must include the PCIe transfer.
//
// A submitted batch is a JOB.  Jobs are cut into SEGMENTS of consecutive
// buffers whose covering byte range is at most `segment_bytes`; each segment
// runs on a free lane (one stream + its device and pinned buffers):
//   hipMemcpyAsync H2D (covering range)  ->  kernel(s)  ->  hipMemcpyAsync D2H
//   of the per-buffer results into the lane's pinned result buffer
// and is RETIRED (results copied to the caller's array) once its event has
// completed.  Progress is made by crc32c_pipeline_poll (non-blocking: only
// hipEventQuery, never a wait -- for Flow's run loop, as the reference's file
// wrappers return Futures, fdbrpc/AsyncFileWriteChecker.h:59-67) and by
// crc32c_pipeline_wait (blocking).  The synchronous entry points are
// submit + wait.  With >= 2 lanes segment k+1's H2D overlaps segment k's
// kernel and D2H; the engine is PCIe-bound by design (the kernel runs ~100x
// faster than the link).
//
// Job kinds and the device entry point each segment runs:
//   VARLEN     crc32c_gpu_batch_varlen_ws   (offsets rebased to the segment)
//   FIXED      crc32c_gpu_batch_fixed       (page-shaped batches run the page
//                                            kernel; the segment keeps the host
//                                            address's alignment mod 16, so the
//                                            4088 B / 4092 B page windows too)
//   SQLITE     fdb_sqlite_verify_pages_ws   (status byte per page + bad count)
//   DISKQUEUE  fdb_diskqueue_check_pages_ws (ok byte per page + bad count)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <map>
#include <vector>

#include "../../include/fdb_crc32c.h"
#include "../../include/fdb_pagecheck.h"
#include "crc32c_device.h"

namespace fdbcrc {
int device_tables(const DevTables** tabs, int* num_cus);  // crc32c_capi.cpp
int set_error(int code, const char* what, hipError_t e);  // crc32c_capi.cpp
}  // namespace fdbcrc

using namespace fdbcrc;

namespace {

enum Kind { VARLEN, FIXED, SQLITE, DISKQUEUE };

struct Job {
	uint64_t ticket = 0;
	Kind kind = VARLEN;
	const uint8_t* base = nullptr;
	const uint64_t* offs = nullptr;
	const uint64_t* lens = nullptr;
	uint64_t stride = 0, length = 0, count = 0;
	uint32_t seed = 0;
	const uint32_t* seeds = nullptr;
	uint8_t* out = nullptr;  // uint32_t per buffer (CRC kinds) or uint8_t per page (verifiers)
	uint64_t* bad_out = nullptr;
	uint32_t first_pgno = 0;
	bool pinned = false;
	uint64_t next = 0;      // first buffer not yet issued
	uint64_t piece = 0;     // next piece of buffer `next` when it is longer than a segment
	uint32_t inflight = 0;  // segments issued, not retired
	uint64_t bad = 0;
	int rc = 0;
	// buffers longer than a segment: checksummed in segment-sized pieces (piece 0
	// with the buffer's seed, the others with seed 0) and folded with
	// crc32c_combine once every piece has retired, in any order
	struct Long {
		std::vector<uint32_t> crc;
		std::vector<uint64_t> len;
		uint64_t left = 0;
	};
	std::map<uint64_t, Long> longs;
	bool finished() const { return inflight == 0 && (rc != 0 || next >= count); }
	size_t esize() const { return (kind == VARLEN || kind == FIXED) ? 4 : 1; }
};

}  // namespace

struct fdb_crc32c_pipeline {
	int device = 0;
	uint64_t seg_bytes = 0;
	uint64_t max_bufs = 0;  // buffers per segment (metadata capacity)
	struct Lane {
		hipStream_t stream = nullptr;
		uint8_t* d_data = nullptr;   // seg_bytes + 64
		uint64_t* d_meta = nullptr;  // [max_bufs offsets][max_bufs lengths]
		uint32_t* d_seeds = nullptr;
		uint32_t* d_res = nullptr;   // per-buffer results
		uint64_t* d_bad = nullptr;
		void* d_ws = nullptr;
		uint64_t ws_bytes = 0;
		uint64_t* h_meta = nullptr;   // pinned
		uint32_t* h_seeds = nullptr;  // pinned
		uint32_t* h_res = nullptr;    // pinned
		uint64_t* h_bad = nullptr;    // pinned
		uint8_t* h_stage = nullptr;   // pinned staging for pageable sources
		hipEvent_t done = nullptr;
		bool busy = false;
		uint64_t ticket = 0, start = 0, n = 0, seq = 0;
		uint64_t piece = ~0ull;  // piece index of a long buffer's segment (~0: a segment of whole buffers)
	};
	std::vector<Lane> lanes;
	std::deque<Job> jobs;          // unfinished or unreported, in ticket order
	std::map<uint64_t, int> failed;  // finished jobs that failed, by ticket
	uint64_t next_ticket = 1, seq = 0;
};

namespace {

using Pipe = fdb_crc32c_pipeline;

int hip_fail(const char* what, hipError_t e) { return set_error(FDB_CRC32C_EHIP, what, e); }
int inval(const char* what) { return set_error(FDB_CRC32C_EINVAL, what, hipSuccess); }

bool is_pinned(const void* p) {
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	return a.type == hipMemoryTypeHost;
}

struct DeviceScope {  // run on the pipeline's device, restore the caller's
	int prev = -1, want;
	explicit DeviceScope(int dev) : want(dev) {
		(void)hipGetDevice(&prev);
		if (prev != want) (void)hipSetDevice(want);
	}
	~DeviceScope() {
		if (prev != want && prev >= 0) (void)hipSetDevice(prev);
	}
};

Job* find_job(Pipe* p, uint64_t ticket) {
	if (p->jobs.empty() || ticket < p->jobs.front().ticket) return nullptr;
	const uint64_t k = ticket - p->jobs.front().ticket;
	return k < p->jobs.size() ? &p->jobs[k] : nullptr;
}

// Copies a finished segment's results to the caller and frees the lane.
void retire(Pipe* p, Pipe::Lane& L, hipError_t status) {
	L.busy = false;
	Job* j = find_job(p, L.ticket);
	if (!j) return;
	--j->inflight;
	if (status != hipSuccess) {
		if (!j->rc) j->rc = hip_fail("pipeline segment", status);
	} else if (!j->rc && L.piece != ~0ull) {
		auto it = j->longs.find(L.start);
		if (it != j->longs.end()) {
			Job::Long& g = it->second;
			g.crc[L.piece] = L.h_res[0];
			if (--g.left == 0) {  // crc32c_append(seed, P0 || P1 || ...) from the pieces' checksums
				uint32_t c = g.crc[0];
				for (size_t k = 1; k < g.crc.size(); ++k) c = crc32c_combine(c, g.crc[k], g.len[k]);
				memcpy(j->out + L.start * 4, &c, 4);
				j->longs.erase(it);
			}
		}
	} else if (!j->rc) {
		memcpy(j->out + L.start * j->esize(), L.h_res, L.n * j->esize());
		if (j->kind == SQLITE || j->kind == DISKQUEUE) j->bad += *L.h_bad;
	}
	if (j->rc) j->longs.clear();
	if (j->finished() && !j->rc && j->bad_out) *j->bad_out = j->bad;
}

// Enqueues the next piece of buffer j.next (longer than a segment) on lane L:
// one segment-sized range through the device engine, its checksum D2H.
int issue_piece(Pipe* p, Pipe::Lane& L, Job& j, uint64_t off, uint64_t len) {
	const uint64_t i = j.next, k = j.piece;
	const uint64_t npieces = (len + p->seg_bytes - 1) / p->seg_bytes;
	if (k == 0) {
		Job::Long& g = j.longs[i];
		g.crc.assign(npieces, 0);
		g.len.assign(npieces, 0);
		g.left = npieces;
	}
	const uint64_t po = k * p->seg_bytes, pl = std::min(p->seg_bytes, len - po);
	j.longs[i].len[k] = pl;
	const uint8_t* src = j.base + off + po;
	hipError_t e = hipSuccess;
	if (!j.pinned) {
		if (!L.h_stage && (e = hipHostMalloc(&L.h_stage, p->seg_bytes, hipHostMallocDefault)) != hipSuccess)
			return set_error(FDB_CRC32C_ENOMEM, "pipeline: staging", e);
		memcpy(L.h_stage, src, pl);
		src = L.h_stage;
	}
	// the piece keeps its host alignment mod 16 (page-shaped pieces run the page kernel)
	const uint64_t h = reinterpret_cast<uintptr_t>(j.base + off + po) % 16;
	uint8_t* dst = L.d_data + h;
	if ((e = hipMemcpyAsync(dst, src, pl, hipMemcpyHostToDevice, L.stream)) != hipSuccess) return hip_fail("H2D data", e);
	const uint32_t seed = k ? 0u : (j.seeds ? j.seeds[i] : j.seed);
	if (int rc = crc32c_gpu_batch_fixed(dst, 0, pl, 1, seed, nullptr, L.d_res, L.stream)) return rc;
	if ((e = hipMemcpyAsync(L.h_res, L.d_res, 4, hipMemcpyDeviceToHost, L.stream)) != hipSuccess)
		return hip_fail("D2H results", e);
	if ((e = hipEventRecord(L.done, L.stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
	L.busy = true;
	L.ticket = j.ticket;
	L.start = i;
	L.n = 1;
	L.piece = k;
	L.seq = ++p->seq;
	++j.inflight;
	if (++j.piece == npieces) {
		j.piece = 0;
		j.next = i + 1;
	}
	return 0;
}

// Builds and enqueues the next segment of `j` on free lane L.
int issue(Pipe* p, Pipe::Lane& L, Job& j) {
	const uint64_t i = j.next;
	uint64_t n = 0, lo = 0, span = 0, h = 0;
	L.piece = ~0ull;
	if (j.kind == VARLEN) {
		if (j.lens[i] > p->seg_bytes) return issue_piece(p, L, j, j.offs[i], j.lens[i]);
		uint64_t a = ~0ull, b = 0;
		while (i + n < j.count && n < p->max_bufs) {
			const uint64_t o = j.offs[i + n], l = j.lens[i + n];
			if (l > p->seg_bytes) break;  // a long buffer starts the next segment
			const uint64_t na = l ? std::min(a, o) : a, nb = l ? std::max(b, o + l) : b;
			if (n && nb > na && nb - na > p->seg_bytes) break;
			a = na;
			b = nb;
			++n;
		}
		if (b < a) a = b = 0;  // all empty
		lo = a;
		span = b - a;
		for (uint64_t k = 0; k < n; ++k) {
			L.h_meta[k] = j.lens[i + k] ? j.offs[i + k] - lo : 0;
			L.h_meta[p->max_bufs + k] = j.lens[i + k];
		}
	} else {
		if (j.length > p->seg_bytes) {
			if (j.kind == FIXED) return issue_piece(p, L, j, i * j.stride, j.length);
			return inval("pipeline: page larger than the pipeline's segment");
		}
		n = std::min(j.count - i, p->max_bufs);
		if (j.stride) n = std::min(n, (p->seg_bytes - j.length) / j.stride + 1);
		lo = i * j.stride;
		span = (n - 1) * j.stride + j.length;
		if (j.kind == FIXED) h = reinterpret_cast<uintptr_t>(j.base + lo) % 16;
	}
	hipError_t e = hipSuccess;
	const uint8_t* src = j.base + lo;
	if (!j.pinned && span) {
		if (!L.h_stage && (e = hipHostMalloc(&L.h_stage, p->seg_bytes, hipHostMallocDefault)) != hipSuccess)
			return set_error(FDB_CRC32C_ENOMEM, "pipeline: staging", e);
		memcpy(L.h_stage, src, span);
		src = L.h_stage;
	}
	uint8_t* dst = L.d_data + h;
	if (span && (e = hipMemcpyAsync(dst, src, span, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
		return hip_fail("H2D data", e);
	if (j.kind == VARLEN &&
	    ((e = hipMemcpyAsync(L.d_meta, L.h_meta, 8 * n, hipMemcpyHostToDevice, L.stream)) != hipSuccess ||
	     (e = hipMemcpyAsync(L.d_meta + p->max_bufs, L.h_meta + p->max_bufs, 8 * n, hipMemcpyHostToDevice, L.stream)) !=
	         hipSuccess))
		return hip_fail("H2D metadata", e);
	const bool seeded = j.seeds && (j.kind == VARLEN || j.kind == FIXED);
	if (seeded) {
		memcpy(L.h_seeds, j.seeds + i, 4 * n);
		if ((e = hipMemcpyAsync(L.d_seeds, L.h_seeds, 4 * n, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
			return hip_fail("H2D seeds", e);
	}
	int rc = 0;
	switch (j.kind) {
	case VARLEN:
		rc = crc32c_gpu_batch_varlen_ws(dst, L.d_meta, L.d_meta + p->max_bufs, n, j.seed, seeded ? L.d_seeds : nullptr,
		                                L.d_res, L.d_ws, L.ws_bytes, L.stream);
		break;
	case FIXED:
		rc = crc32c_gpu_batch_fixed(dst, j.stride, j.length, n, j.seed, seeded ? L.d_seeds : nullptr, L.d_res, L.stream);
		break;
	case SQLITE:
		rc = fdb_sqlite_verify_pages_ws(dst, j.length, n, j.first_pgno + (uint32_t)i, reinterpret_cast<uint8_t*>(L.d_res),
		                                L.d_bad, L.d_ws, L.ws_bytes, L.stream);
		break;
	case DISKQUEUE:
		rc = fdb_diskqueue_check_pages_ws(dst, n, reinterpret_cast<uint8_t*>(L.d_res), L.d_bad, L.d_ws, L.ws_bytes,
		                                  L.stream);
		break;
	}
	if (rc) return rc;
	if ((e = hipMemcpyAsync(L.h_res, L.d_res, n * j.esize(), hipMemcpyDeviceToHost, L.stream)) != hipSuccess)
		return hip_fail("D2H results", e);
	if ((j.kind == SQLITE || j.kind == DISKQUEUE) &&
	    (e = hipMemcpyAsync(L.h_bad, L.d_bad, 8, hipMemcpyDeviceToHost, L.stream)) != hipSuccess)
		return hip_fail("D2H bad count", e);
	if ((e = hipEventRecord(L.done, L.stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
	L.busy = true;
	L.ticket = j.ticket;
	L.start = i;
	L.n = n;
	L.seq = ++p->seq;
	j.next = i + n;
	++j.inflight;
	return 0;
}

// Non-blocking progress: retire completed segments, fill free lanes from the
// oldest jobs, drop finished jobs from the front of the queue.
void pump(Pipe* p) {
	for (auto& L : p->lanes) {
		if (!L.busy) continue;
		hipError_t e = hipEventQuery(L.done);
		if (e == hipErrorNotReady) continue;
		retire(p, L, e);
	}
	for (auto& j : p->jobs) {
		if (j.rc || j.next >= j.count) continue;
		for (auto& L : p->lanes) {
			if (L.busy || j.rc || j.next >= j.count) continue;
			if (int rc = issue(p, L, j)) j.rc = rc;
		}
		if (!j.rc && j.next < j.count) break;  // no free lane left
	}
	while (!p->jobs.empty() && p->jobs.front().finished()) {
		if (p->jobs.front().rc) p->failed[p->jobs.front().ticket] = p->jobs.front().rc;
		p->jobs.pop_front();
	}
}

// 1 done, 0 pending, < 0 the job's error.  A failed job's error is kept for
// the pipeline's lifetime: every later poll/wait of its ticket reports it
// again (never a success for results that were not written).
int job_state(Pipe* p, uint64_t ticket) {
	if (ticket == 0 || ticket >= p->next_ticket) return inval("pipeline: unknown ticket");
	Job* j = find_job(p, ticket);
	if (j) return j->finished() ? (j->rc ? j->rc : 1) : 0;
	auto it = p->failed.find(ticket);
	return it == p->failed.end() ? 1 : it->second;
}

int submit(Pipe* p, Job j, uint64_t* ticket) {
	if (!p) return inval("pipeline: null pipeline");
	DeviceScope ds(p->device);
	j.ticket = p->next_ticket++;
	j.pinned = j.count ? is_pinned(j.base) : true;
	if (j.count == 0 && j.bad_out) *j.bad_out = 0;
	p->jobs.push_back(j);
	pump(p);
	if (ticket) *ticket = j.ticket;
	return 0;
}

int wait(Pipe* p, uint64_t ticket) {
	if (!p) return inval("pipeline: null pipeline");
	DeviceScope ds(p->device);
	for (;;) {
		pump(p);
		int st = job_state(p, ticket);
		if (st != 0) return st == 1 ? 0 : st;
		Pipe::Lane* oldest = nullptr;  // block on the oldest segment in flight
		for (auto& L : p->lanes)
			if (L.busy && (!oldest || L.seq < oldest->seq)) oldest = &L;
		if (!oldest) return set_error(FDB_CRC32C_EHIP, "pipeline: job pending with no segment in flight", hipSuccess);
		retire(p, *oldest, hipEventSynchronize(oldest->done));
	}
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
	if (!out || nstreams < 1 || nstreams > 16) return inval("pipeline_create: bad args");
	if (segment_bytes < (1u << 20)) segment_bytes = 1u << 20;
	const DevTables* tabs;
	int cus;
	if (int rc = device_tables(&tabs, &cus)) return rc;
	auto* p = new fdb_crc32c_pipeline;
	(void)hipGetDevice(&p->device);
	p->seg_bytes = segment_bytes;
	p->max_bufs = segment_bytes / 64 + 1024;  // >= 64 B average per buffer
	p->lanes.resize(nstreams);
	const uint64_t ws = std::max(crc32c_gpu_varlen_workspace_bytes(p->max_bufs), fdb_pagecheck_workspace_bytes(p->max_bufs));
	for (auto& L : p->lanes) {
		hipError_t e;
		if ((e = hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking)) != hipSuccess ||
		    (e = hipMalloc(&L.d_data, segment_bytes + 64)) != hipSuccess ||
		    (e = hipMalloc(&L.d_meta, 16 * p->max_bufs)) != hipSuccess ||
		    (e = hipMalloc(&L.d_seeds, 4 * p->max_bufs)) != hipSuccess ||
		    (e = hipMalloc(&L.d_res, 4 * p->max_bufs)) != hipSuccess ||
		    (e = hipMalloc(&L.d_bad, 8)) != hipSuccess ||
		    (e = hipMalloc(&L.d_ws, ws)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_meta, 16 * p->max_bufs, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_seeds, 4 * p->max_bufs, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_res, 4 * p->max_bufs, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipHostMalloc(&L.h_bad, 8, hipHostMallocDefault)) != hipSuccess ||
		    (e = hipEventCreateWithFlags(&L.done, hipEventDisableTiming)) != hipSuccess) {
			crc32c_pipeline_destroy(p);
			return set_error(FDB_CRC32C_ENOMEM, "pipeline_create: allocation", e);
		}
		L.ws_bytes = ws;
	}
	*out = p;
	return 0;
}

void crc32c_pipeline_destroy(fdb_crc32c_pipeline* p) {
	if (!p) return;
	DeviceScope ds(p->device);
	for (auto& L : p->lanes) {
		if (L.stream) {
			(void)hipStreamSynchronize(L.stream);
			(void)crc32c_gpu_release_stream(L.stream);
		}
		if (L.d_data) (void)hipFree(L.d_data);
		if (L.d_meta) (void)hipFree(L.d_meta);
		if (L.d_seeds) (void)hipFree(L.d_seeds);
		if (L.d_res) (void)hipFree(L.d_res);
		if (L.d_bad) (void)hipFree(L.d_bad);
		if (L.d_ws) (void)hipFree(L.d_ws);
		if (L.h_meta) (void)hipHostFree(L.h_meta);
		if (L.h_seeds) (void)hipHostFree(L.h_seeds);
		if (L.h_res) (void)hipHostFree(L.h_res);
		if (L.h_bad) (void)hipHostFree(L.h_bad);
		if (L.h_stage) (void)hipHostFree(L.h_stage);
		if (L.done) (void)hipEventDestroy(L.done);
		if (L.stream) (void)hipStreamDestroy(L.stream);
	}
	delete p;
}

int crc32c_pipeline_submit_varlen(fdb_crc32c_pipeline* p, const void* h_base, const uint64_t* h_offsets,
                                  const uint64_t* h_lengths, uint64_t count, uint32_t seed, const uint32_t* h_seeds,
                                  uint32_t* h_out, uint64_t* ticket) {
	if (count && (!h_base || !h_offsets || !h_lengths || !h_out)) return inval("pipeline_varlen: null pointer");
	Job j;
	j.kind = VARLEN;
	j.base = static_cast<const uint8_t*>(h_base);
	j.offs = h_offsets;
	j.lens = h_lengths;
	j.count = count;
	j.seed = seed;
	j.seeds = h_seeds;
	j.out = reinterpret_cast<uint8_t*>(h_out);
	return submit(p, j, ticket);
}

int crc32c_pipeline_submit_fixed(fdb_crc32c_pipeline* p, const void* h_base, uint64_t stride, uint64_t length,
                                 uint64_t count, uint32_t seed, const uint32_t* h_seeds, uint32_t* h_out,
                                 uint64_t* ticket) {
	if (count && (!h_out || (!h_base && length))) return inval("pipeline_fixed: null pointer");
	Job j;
	j.kind = FIXED;
	j.base = static_cast<const uint8_t*>(h_base);
	j.stride = stride;
	j.length = length;
	j.count = count;
	j.seed = seed;
	j.seeds = h_seeds;
	j.out = reinterpret_cast<uint8_t*>(h_out);
	return submit(p, j, ticket);
}

int crc32c_pipeline_poll(fdb_crc32c_pipeline* p, uint64_t ticket) {
	if (!p) return inval("pipeline: null pipeline");
	DeviceScope ds(p->device);
	pump(p);
	return job_state(p, ticket);
}

int crc32c_pipeline_wait(fdb_crc32c_pipeline* p, uint64_t ticket) { return wait(p, ticket); }

int crc32c_pipeline_varlen(fdb_crc32c_pipeline* p, const void* h_base, const uint64_t* h_offsets,
                           const uint64_t* h_lengths, uint64_t count, uint32_t seed, const uint32_t* h_seeds,
                           uint32_t* h_out) {
	uint64_t t = 0;
	if (int rc = crc32c_pipeline_submit_varlen(p, h_base, h_offsets, h_lengths, count, seed, h_seeds, h_out, &t))
		return rc;
	return wait(p, t);
}

int crc32c_pipeline_fixed(fdb_crc32c_pipeline* p, const void* h_base, uint64_t stride, uint64_t length,
                          uint64_t count, uint32_t seed, const uint32_t* h_seeds, uint32_t* h_out) {
	uint64_t t = 0;
	if (int rc = crc32c_pipeline_submit_fixed(p, h_base, stride, length, count, seed, h_seeds, h_out, &t)) return rc;
	return wait(p, t);
}

// ---- host-resident page verifiers (include/fdb_pagecheck.h) -----------------

int fdb_sqlite_verify_pages_host_submit(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t page_size,
                                        uint64_t count, uint32_t first_pgno, uint8_t* h_status, uint64_t* h_bad,
                                        uint64_t* ticket) {
	if (count && (!h_pages || !h_status)) return inval("fdb_sqlite_verify_pages_host: null pointer");
	if (page_size % 16 || page_size <= 248 || page_size >= (1ull << 31))
		return inval("page_size must be a multiple of 16 in (248, 2^31)");
	if (count >= (1ull << 32)) return inval("count must be < 2^32");
	Job j;
	j.kind = SQLITE;
	j.base = static_cast<const uint8_t*>(h_pages);
	j.stride = j.length = page_size;
	j.count = count;
	j.first_pgno = first_pgno;
	j.out = h_status;
	j.bad_out = h_bad;
	return submit(p, j, ticket);
}

int fdb_sqlite_verify_pages_host(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t page_size, uint64_t count,
                                 uint32_t first_pgno, uint8_t* h_status, uint64_t* h_bad) {
	uint64_t t = 0;
	if (int rc = fdb_sqlite_verify_pages_host_submit(p, h_pages, page_size, count, first_pgno, h_status, h_bad, &t))
		return rc;
	return wait(p, t);
}

int fdb_diskqueue_check_pages_host_submit(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t count, uint8_t* h_ok,
                                          uint64_t* h_bad, uint64_t* ticket) {
	if (count && (!h_pages || !h_ok)) return inval("fdb_diskqueue_check_pages_host: null pointer");
	if (count >= (1ull << 32)) return inval("count must be < 2^32");
	Job j;
	j.kind = DISKQUEUE;
	j.base = static_cast<const uint8_t*>(h_pages);
	j.stride = j.length = 4096;
	j.count = count;
	j.out = h_ok;
	j.bad_out = h_bad;
	return submit(p, j, ticket);
}

int fdb_diskqueue_check_pages_host(fdb_crc32c_pipeline* p, const void* h_pages, uint64_t count, uint8_t* h_ok,
                                   uint64_t* h_bad) {
	uint64_t t = 0;
	if (int rc = fdb_diskqueue_check_pages_host_submit(p, h_pages, count, h_ok, h_bad, &t)) return rc;
	return wait(p, t);
}

}  // extern "C"
