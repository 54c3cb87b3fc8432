// C ABI for the batched engine (declarations and contracts: include/fdb_crc32c.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>
#include <new>
#include <mutex>
#include <string>

#include "../../include/fdb_crc32c.h"
#include "../../include/fdb_packets.h"
#include "../../include/fdb_pagecheck.h"
#include "../../include/fdb_redwood.h"
#include "../../include/fdb_xxh3.h"
#include "crc32c_device.h"
#include "packets.h"
#include "pagecheck.h"
#include "redwood.h"
#include "xxh3_device.h"

namespace fdbcrc {
namespace {

constexpr int kMaxDevices = 64;
constexpr int kHstatErr = 6;  // u64 word of the stream's host-mapped block holding its refusal flag
constexpr int kHstatXxhNeed = 7;  // ... the long-buffer blocks of its last XXH3 varlen batch (split route room)

// Library-owned state of one (device, stream).  `mu` is held from the
// workspace lookup through the enqueue of the kernels that use it, so a
// thread that grows (frees and reallocates) the workspace can never free a
// buffer another thread has been handed but not yet launched on.
struct StreamState {
	std::mutex mu;
	void* ws = nullptr;  // planning workspace (varlen, XXH3 varlen, verifiers)
	uint64_t ws_bytes = 0;
	uint32_t* ctr = nullptr;  // page-kernel grab counters
	uint64_t ctr_bytes = 0;
	uint64_t* aux = nullptr;  // the verifiers' counters (stream_aux)
	// held from a call's stream_aux lookup through its last launch: the counters
	// are shared by every call on the stream, so two host threads' calls must
	// not interleave their kernels on it (taken after `mu`, never before it)
	std::mutex aux_mu;
	uint64_t* hst_h = nullptr;  // varlen route statistics of the stream's last batch (host-mapped)
	uint64_t* hst_d = nullptr;  // ... its device address
	// extent route state (crc32c_extent.hip): grown to the batches seen
	void* xmem = nullptr;
	uint64_t xcount = 0;            // buffers it holds
	uint32_t xepoch = 0;            // launches on the extent route (epoch tags, never 0)
	// the prep-free block route's part accumulators (kNPAccBytes, zero between launches)
	uint32_t* bacc = nullptr;
};

struct DeviceState {
	DevTables* tables = nullptr;  // device copy
	int num_cus = 0;
	bool ready = false;
	std::map<hipStream_t, std::unique_ptr<StreamState>> streams;  // guarded by g_mu
};

std::mutex g_mu;
DeviceState g_dev[kMaxDevices];
thread_local std::string t_err;

int fail(int code, const char* what, hipError_t e = hipSuccess) {
	char buf[256];
	if (e != hipSuccess)
		snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
	else
		snprintf(buf, sizeof buf, "%s", what);
	t_err = buf;
	return code;
}

// Returns 0 and fills *st for the current device.
int device_state(DeviceState** st) {
	int dev = -1;
	hipError_t e = hipGetDevice(&dev);
	if (e != hipSuccess) return fail(FDB_CRC32C_ENODEV, "hipGetDevice", e);
	if (dev < 0 || dev >= kMaxDevices) return fail(FDB_CRC32C_ENODEV, "device ordinal out of range");
	DeviceState& d = g_dev[dev];
	std::lock_guard<std::mutex> lock(g_mu);
	if (!d.ready) {
		int cus = 0;
		e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
		if (e != hipSuccess) return fail(FDB_CRC32C_ENODEV, "hipDeviceGetAttribute", e);
		// ~1.3 MB: built on the heap, since the first call may come from a
		// thread with a small stack (SQLite readers, Flow's network thread)
		std::unique_ptr<DevTables> host(new (std::nothrow) DevTables);
		if (!host) return fail(FDB_CRC32C_ENOMEM, "host tables");
		build_dev_tables(host.get());
		DevTables* dt = nullptr;
		e = hipMalloc(reinterpret_cast<void**>(&dt), sizeof(DevTables));
		if (e != hipSuccess) return fail(FDB_CRC32C_ENOMEM, "hipMalloc(tables)", e);
		e = hipMemcpy(dt, host.get(), sizeof(DevTables), hipMemcpyHostToDevice);
		if (e != hipSuccess) {
			(void)hipFree(dt);
			return fail(FDB_CRC32C_EHIP, "hipMemcpy(tables)", e);
		}
		d.tables = dt;
		d.num_cus = cus > 0 ? cus : 256;
		d.ready = true;
	}
	*st = &d;
	return 0;
}

StreamState* stream_state(DeviceState* st, hipStream_t s) {
	std::lock_guard<std::mutex> lock(g_mu);
	auto& p = st->streams[s];
	if (!p) p.reset(new StreamState);
	return p.get();
}

// Planning workspace owned by the library for the convenience entry points,
// one per (device, stream) so concurrent streams never share it.  On success
// `hold` owns the stream's lock: keep it until the kernels using *ws are
// enqueued.  Growing synchronises the stream once (the old buffer may still be
// in use by launches already enqueued).
int stream_workspace(DeviceState* st, hipStream_t s, uint64_t need, void** ws, uint64_t* have,
                     std::unique_lock<std::mutex>* hold) {
	StreamState* ss = stream_state(st, s);
	std::unique_lock<std::mutex> lock(ss->mu);
	if (ss->ws_bytes < need) {
		if (ss->ws) {
			hipError_t e = hipStreamSynchronize(s);
			if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, "hipStreamSynchronize(workspace)", e);
			(void)hipFree(ss->ws);
			ss->ws = nullptr;
			ss->ws_bytes = 0;
		}
		uint64_t sz = need < (1u << 20) ? (1u << 20) : need * 2;
		void* p = nullptr;
		hipError_t e = hipMalloc(&p, sz);
		if (e != hipSuccess) return fail(FDB_CRC32C_ENOMEM, "hipMalloc(workspace)", e);
		ss->ws = p;
		ss->ws_bytes = sz;
	}
	*ws = ss->ws;
	*have = ss->ws_bytes;
	*hold = std::move(lock);
	return 0;
}

// The stream's host-mapped words: [0..2] route statistics of its last varlen
// batch, [kHstatErr] its sticky refusal flag (crc32c_gpu_stream_status).
bool stream_mapped(StreamState* ss) {
	if (ss->hst_h) return true;
	void* h = nullptr;
	void* d = nullptr;
	if (hipHostMalloc(&h, 64, hipHostMallocMapped) != hipSuccess) return false;
	memset(h, 0, 64);
	if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
		(void)hipHostFree(h);
		return false;
	}
	ss->hst_h = static_cast<uint64_t*>(h);
	ss->hst_d = static_cast<uint64_t*>(d);
	return true;
}

uint32_t* stream_err(DeviceState* st, hipStream_t s) {
	StreamState* ss = stream_state(st, s);
	std::lock_guard<std::mutex> lock(g_mu);
	return stream_mapped(ss) ? reinterpret_cast<uint32_t*>(ss->hst_d + kHstatErr) : nullptr;
}

// Route of the stream's next varlen batch from the span statistics its last
// batch left (prep writes them into host-mapped memory; read without any
// synchronisation: a stale or torn value only costs speed, never
// correctness).  Caller holds the stream's lock.  Falls back to kRouteBoth.
int stream_route(DeviceState* st, hipStream_t s, uint64_t** hstat) {
	StreamState* ss = stream_state(st, s);
	bool mapped;
	{
		std::lock_guard<std::mutex> lock(g_mu);
		mapped = stream_mapped(ss);
	}
	if (!mapped) {
		*hstat = nullptr;
		return kRouteBoth;
	}
	*hstat = ss->hst_d;
	static const int forced = [] {  // development: FDBCRC_ROUTE=0|1|2|3 pins the route
		const char* e = getenv("FDBCRC_ROUTE");
		return e ? atoi(e) : -1;
	}();
	if (forced >= kRouteBoth && forced <= kRouteExtent) return forced;
	return route_for_stats(ss->hst_h);
}

// The stream's extent-route state for a batch of `count` buffers (caller
// holds the stream's lock): per-buffer point values and per-wave aggregates,
// grown to the largest batch seen.  false: no state (allocation failed): the
// caller routes to the window engine.
bool stream_extent(DeviceState* st, hipStream_t s, uint64_t count, XState* xs) {
	StreamState* ss = stream_state(st, s);
	if (!ss->xmem || count > ss->xcount) {
		if (ss->xmem) {
			if (hipStreamSynchronize(s) != hipSuccess) return false;
			(void)hipFree(ss->xmem);
			ss->xmem = nullptr;
		}
		const uint64_t nc = count + count / 4;
		void* m = nullptr;
		const uint64_t bytes = extent_state_bytes(nc, kXGrabCap, st->num_cus);
		if (hipMalloc(&m, bytes) != hipSuccess) {
			(void)hipGetLastError();
			ss->xcount = 0;
			return false;
		}
		if (hipMemsetAsync(m, 0, 256, s) != hipSuccess) {  // the epoch-tagged flags
			(void)hipFree(m);
			return false;
		}
		ss->xmem = m;
		ss->xcount = nc;
	}
	extent_state_carve(ss->xmem, ss->xcount, kXGrabCap, st->num_cus, xs);
	// the dynamic stream kernel's grab counters (development: FDBCRC_XSTATIC=1
	// streams with static per-wave ranges instead)
	static const bool stat = getenv("FDBCRC_XSTATIC") && atoi(getenv("FDBCRC_XSTATIC")) == 1;
	xs->ctr = nullptr;
	if (!stat && page_counters(s, st->num_cus, &xs->ctr)) xs->ctr = nullptr;
	if (++ss->xepoch == 0) ++ss->xepoch;
	xs->epoch = ss->xepoch;
	return true;
}

// The prep-free block route's accumulators of `s` (caller holds the stream's
// lock): allocated and zeroed on the stream at first use, left zero by every
// launch.  nullptr: none (the route keeps its prep).
uint32_t* stream_blocks_acc(DeviceState* st, hipStream_t s) {
	StreamState* ss = stream_state(st, s);
	if (!ss->bacc) {
		void* m = nullptr;
		if (hipMalloc(&m, kNPAccBytes) != hipSuccess) {
			(void)hipGetLastError();
			return nullptr;
		}
		if (hipMemsetAsync(m, 0, kNPAccBytes, s) != hipSuccess) {
			(void)hipFree(m);
			return nullptr;
		}
		ss->bacc = static_cast<uint32_t*>(m);
	}
	return ss->bacc;
}

int check_launch(const char* what) {
	hipError_t e = hipGetLastError();
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, what, e);
	return 0;
}

}  // namespace

// Grab counters of the page kernels for `stream` on the current device:
// zeroed once here, left at zero by every page launch.
// The zeroing is enqueued on `stream` itself, ahead of the first page launch.
// (Allocation happens under g_mu, not the stream lock: the verifiers launch
// page kernels while holding their stream's workspace lock.)
// The first use of a stream allocates and zeroes its counters: that cannot be
// recorded into a graph (hipMalloc invalidates a capture, and the zeroing
// would only run at replay), so it is refused while the stream captures.
static bool capturing(hipStream_t s) {
	hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
	return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

int page_counters(hipStream_t stream, int num_cus, uint32_t** ctr) {
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	StreamState* ss = stream_state(st, stream);
	std::lock_guard<std::mutex> lock(g_mu);
	if (!ss->ctr) {
		if (capturing(stream))
			return fail(FDB_CRC32C_EINVAL, "first use of a stream inside a stream capture: run one call on it "
			                               "outside the capture first (its counters are allocated then)");
		const size_t bytes = (size_t)(num_cus > st->num_cus ? num_cus : st->num_cus) * kPageCtrWords * 4;
		uint32_t* q = nullptr;
		hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), bytes);
		if (e != hipSuccess) return fail(FDB_CRC32C_ENOMEM, "hipMalloc(page counters)", e);
		e = hipMemsetAsync(q, 0, bytes, stream);
		if (e != hipSuccess) {
			(void)hipFree(q);
			return fail(FDB_CRC32C_EHIP, "hipMemsetAsync(page counters)", e);
		}
		ss->ctr = q;
		ss->ctr_bytes = bytes;
	}
	*ctr = ss->ctr;
	return 0;
}

// The stream's counter words of the page verifiers, the seal passes and the
// packet verifier (kAux* in crc32c_device.h): zeroed once here, on `stream`
// ahead of their first use, and put back to zero by the last kernel of every
// call that uses them, so no call starts with a memset (and a captured graph
// of a call replays correctly: it ends with them at zero too).  Per stream,
// not in the workspace: the convenience entry points share one workspace per
// stream between every API, and a caller's workspace is not ours to keep.
int stream_aux(hipStream_t stream, uint64_t** aux, std::unique_lock<std::mutex>* hold) {
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	StreamState* ss = stream_state(st, stream);
	std::unique_lock<std::mutex> alock(ss->aux_mu);
	std::lock_guard<std::mutex> lock(g_mu);
	if (!ss->aux) {
		if (capturing(stream))
			return fail(FDB_CRC32C_EINVAL, "first use of a stream inside a stream capture: run one call on it "
			                               "outside the capture first (its counters are allocated then)");
		uint64_t* q = nullptr;
		hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), kAuxBytes);
		if (e != hipSuccess) return fail(FDB_CRC32C_ENOMEM, "hipMalloc(stream counters)", e);
		e = hipMemsetAsync(q, 0, kAuxBytes, stream);
		if (e != hipSuccess) {
			(void)hipFree(q);
			return fail(FDB_CRC32C_EHIP, "hipMemsetAsync(stream counters)", e);
		}
		ss->aux = q;
	}
	*aux = ss->aux;
	if (hold) *hold = std::move(alock);
	return 0;
}

// Frees what the library holds for `stream` on the current device.
int release_stream(hipStream_t stream) {
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	std::unique_ptr<StreamState> ss;
	{
		std::lock_guard<std::mutex> lock(g_mu);
		auto it = st->streams.find(stream);
		if (it == st->streams.end()) return 0;
		ss = std::move(it->second);
		st->streams.erase(it);
	}
	std::lock_guard<std::mutex> lock(ss->mu);  // wait for an enqueue in progress
	hipError_t e = hipStreamSynchronize(stream);
	if (ss->ws) (void)hipFree(ss->ws);
	if (ss->ctr) (void)hipFree(ss->ctr);
	if (ss->aux) (void)hipFree(ss->aux);
	if (ss->hst_h) (void)hipHostFree(ss->hst_h);
	if (ss->xmem) (void)hipFree(ss->xmem);
	if (ss->bacc) (void)hipFree(ss->bacc);
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, "hipStreamSynchronize(release)", e);
	return 0;
}

uint64_t stream_bytes(hipStream_t stream) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	std::lock_guard<std::mutex> lock(g_mu);
	auto it = st->streams.find(stream);
	if (it == st->streams.end()) return 0;
	return it->second->ws_bytes + it->second->ctr_bytes +
	       (it->second->xmem ? extent_state_bytes(it->second->xcount, kXGrabCap, st->num_cus) : 0) +
	       (it->second->bacc ? kNPAccBytes : 0);
}

// used by the host pipeline (crc32c_pipeline.cpp)
int device_tables(const DevTables** tabs, int* num_cus) {
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	*tabs = st->tables;
	*num_cus = st->num_cus;
	return 0;
}
int set_error(int code, const char* what, hipError_t e) { return fail(code, what, e); }

}  // namespace fdbcrc

using namespace fdbcrc;

#ifdef FDBCRC_DEBUG
// Debug builds: every varlen/general launch first sets the allowed data window
// (computed on the host from the batch description) and afterwards reports
// bounds violations instead of faulting.
extern "C" int crc32c_debug_bounds(uint64_t lo, uint64_t hi);
extern "C" int crc32c_debug_read(uint64_t* d_out8);
namespace {
void debug_report(const char* what) {
	uint64_t* d = nullptr;
	uint64_t h[8] = {0};
	if (hipMalloc(&d, 64) != hipSuccess) return;
	crc32c_debug_read(d);
	(void)hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
	(void)hipFree(d);
	if (h[2]) fprintf(stderr, "[fdbcrc debug] %s: %llu violations, first bad 0x%llx at site %llu (window 0x%llx..0x%llx)\n",
	                  what, (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4],
	                  (unsigned long long)h[0], (unsigned long long)h[1]);
	crc32c_debug_bounds(0, 0);  // page kernels launched later are not checked against this batch's window
}
void debug_window_varlen(const void* base, const uint64_t* d_off, const uint64_t* d_len, uint64_t n) {
	uint64_t lo = ~0ull, hi = 0;
	uint64_t* ho = (uint64_t*)malloc(8 * n);
	uint64_t* hl = (uint64_t*)malloc(8 * n);
	(void)hipDeviceSynchronize();
	(void)hipMemcpy(ho, d_off, 8 * n, hipMemcpyDeviceToHost);
	(void)hipMemcpy(hl, d_len, 8 * n, hipMemcpyDeviceToHost);
	for (uint64_t i = 0; i < n; ++i) {
		if (!hl[i]) continue;
		const uint64_t a = (uint64_t)base + ho[i];
		if (a < lo) lo = a;
		if (a + hl[i] > hi) hi = a + hl[i];
	}
	free(ho);
	free(hl);
	if (hi == 0) lo = hi = 1;
	crc32c_debug_bounds(lo, hi);
}
}  // namespace
#endif


extern "C" {

int crc32c_gpu_init(void) {
	DeviceState* st = nullptr;
	return device_state(&st);
}

int crc32c_gpu_batch_fixed(const void* d_base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                           const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || (!d_base && length)) return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_fixed: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	const uint8_t* base = static_cast<const uint8_t*>(d_base);
	const uint64_t blocks = length / 4096;
	const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && (stride % 16 == 0) && length % 4096 == 0 &&
	                     (blocks == 1 || blocks == 2);
	// a window [h, 4096 - t) of 16-byte aligned 4 KiB pages (h, t < 16): the
	// SQLite (4088 B at +0) and DiskQueue (4092 B at +4) checksum layouts
	const uint64_t h = reinterpret_cast<uintptr_t>(base) % 16;
	const bool window = !aligned && length > 0 && stride % 16 == 0 && h + length <= 4096 && h + length + 16 > 4096;
	int rc;
	if (length == 0)
		rc = launch_fill_seeds(count, seed, d_seeds, d_out, s);
	else if (aligned)
		rc = launch_pages((int)blocks, base, stride, count, seed, d_seeds, d_out, st->tables, st->num_cus, s);
	else if (window)
		rc = launch_pages_window(base - h, stride, count, (uint32_t)h, (uint32_t)(4096 - h - length), seed, d_seeds,
		                         d_out, st->tables, st->num_cus, s);
	else {
		// the varlen engine numbers 1 KiB windows with 32-bit slot indices
		const uint64_t wpb = (length + 30) / 1024 + 1;  // windows per buffer, an upper bound
		if (count >= (1ull << 32) / wpb)
			return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_fixed: batch covers 2^32 or more 1 KiB windows");
#ifdef FDBCRC_DEBUG
		crc32c_debug_bounds((uint64_t)base, (uint64_t)base + (count - 1) * stride + length);
#endif
		void* ws = nullptr;
		uint64_t have = 0;
		std::unique_lock<std::mutex> hold;
		if (int wrc = stream_workspace(st, s, varlen_workspace_bytes(count, (uint64_t)st->num_cus * 16), &ws, &have,
		                               &hold))
			return wrc;
		rc = launch_fixed_general(base, stride, length, count, seed, d_seeds, d_out, st->tables, st->num_cus, ws, s);
#ifdef FDBCRC_DEBUG
		(void)hipDeviceSynchronize();
		debug_report("batch_fixed(general)");
#endif
	}
	if (rc) return fail(FDB_CRC32C_EHIP, "crc32c_gpu_batch_fixed: launch setup failed");
	return check_launch("crc32c_gpu_batch_fixed launch");
}

uint64_t crc32c_gpu_varlen_workspace_bytes(uint64_t count) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return varlen_workspace_bytes(count, (uint64_t)st->num_cus * 16);
}

// d_base may be null (the reference accepts any pointer for length 0, and
// d_base = 0 makes the offsets absolute device addresses).
static int batch_varlen_impl(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                             uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace,
                             uint64_t workspace_bytes, void* stream, int route, uint64_t* hstat,
                             const XState* xs = nullptr, uint32_t* bacc = nullptr, uint32_t* pctr = nullptr) {
	if (count == 0) return 0;
	if (!d_out || !d_offsets || !d_lengths)
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_varlen: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const uint64_t need = varlen_workspace_bytes(count, (uint64_t)st->num_cus * 16);
	if (!d_workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_varlen: workspace too small or misaligned");
#ifdef FDBCRC_DEBUG
	debug_window_varlen(d_base, d_offsets, d_lengths, count);
#endif
	launch_varlen(static_cast<const uint8_t*>(d_base), d_offsets, d_lengths, count, seed, d_seeds, d_out, st->tables,
	              st->num_cus, d_workspace, reinterpret_cast<hipStream_t>(stream), route, hstat,
	              hstat ? reinterpret_cast<uint32_t*>(hstat + kHstatErr) : nullptr, xs, bacc, pctr);
#ifdef FDBCRC_DEBUG
	(void)hipDeviceSynchronize();
	debug_report("batch_varlen");
#endif
	return check_launch("crc32c_gpu_batch_varlen launch");
}

// Caller-owned workspace: no library state, so both routes run.
int crc32c_gpu_batch_varlen_ws(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                               uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace,
                               uint64_t workspace_bytes, void* stream) {
	return batch_varlen_impl(d_base, d_offsets, d_lengths, count, seed, d_seeds, d_out, d_workspace, workspace_bytes,
	                         stream, kRouteBoth, nullptr);
}

int crc32c_gpu_batch_varlen(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                            uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || !d_offsets || !d_lengths)
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_varlen: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
	                              varlen_workspace_bytes(count, (uint64_t)st->num_cus * 16), &ws, &have, &hold))
		return rc;
	uint64_t* hstat = nullptr;
	int route = stream_route(st, reinterpret_cast<hipStream_t>(stream), &hstat);
	XState xs;
	const bool ext = route == kRouteExtent && stream_extent(st, reinterpret_cast<hipStream_t>(stream), count, &xs);
	if (route == kRouteExtent && !ext) route = kRouteWindows;
	// the block route alone over a small enough batch: no prep (k_bigblocks
	// plans its own blocks), with the stream's accumulators and grab counters
	uint32_t* bacc = nullptr;
	uint32_t* pctr = nullptr;
	if (route == kRouteBlocks && count <= kNPMax && !capturing(reinterpret_cast<hipStream_t>(stream))) {
		bacc = stream_blocks_acc(st, reinterpret_cast<hipStream_t>(stream));
		if (bacc && page_counters(reinterpret_cast<hipStream_t>(stream), st->num_cus, &pctr)) pctr = nullptr;
	}
	return batch_varlen_impl(d_base, d_offsets, d_lengths, count, seed, d_seeds, d_out, ws, have, stream, route, hstat,
	                         ext ? &xs : nullptr, bacc, pctr);
}

// ---- grouped chains ------------------------------------------------------------

static uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

uint64_t crc32c_gpu_chained_workspace_bytes(uint64_t nsegs) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return align16(varlen_workspace_bytes(nsegs ? nsegs : 1, (uint64_t)st->num_cus * 16)) + align16(4 * nsegs + 4);
}

static int batch_chained_impl(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                              uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint32_t seed,
                              const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace, uint64_t workspace_bytes,
                              void* stream, uint32_t* err) {
	if (nchains == 0) return 0;
	if (!d_out || !d_chain_starts || (nsegs && (!d_seg_offsets || !d_seg_lengths)))
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_chained: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const uint64_t vws = align16(varlen_workspace_bytes(nsegs ? nsegs : 1, (uint64_t)st->num_cus * 16));
	if (!d_workspace || workspace_bytes < vws + align16(4 * nsegs + 4) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_chained: workspace too small or misaligned");
	hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	uint32_t* segcrc = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_workspace) + vws);
	if (nsegs)  // raw(0, M_j) of every segment: seed 0xffffffff
		launch_varlen(static_cast<const uint8_t*>(d_base), d_seg_offsets, d_seg_lengths, nsegs, 0xffffffffu, nullptr,
		              segcrc, st->tables, st->num_cus, d_workspace, s, kRouteBoth, nullptr, err);
	launch_chain_fold(d_chain_starts, nchains, d_seg_lengths, segcrc, seed, d_seeds, d_out, st->tables, st->num_cus, s);
	return check_launch("crc32c_gpu_batch_chained launch");
}

int crc32c_gpu_batch_chained_ws(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                                uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint32_t seed,
                                const uint32_t* d_seeds, uint32_t* d_out, void* d_workspace, uint64_t workspace_bytes,
                                void* stream) {
	return batch_chained_impl(d_base, d_seg_offsets, d_seg_lengths, nsegs, d_chain_starts, nchains, seed, d_seeds, d_out,
	                          d_workspace, workspace_bytes, stream, nullptr);
}

int crc32c_gpu_batch_chained(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                             uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint32_t seed,
                             const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
	if (nchains == 0) return 0;
	if (!d_out || !d_chain_starts || (nsegs && (!d_seg_offsets || !d_seg_lengths)))
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_chained: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), crc32c_gpu_chained_workspace_bytes(nsegs),
	                              &ws, &have, &hold))
		return rc;
	return batch_chained_impl(d_base, d_seg_offsets, d_seg_lengths, nsegs, d_chain_starts, nchains, seed, d_seeds, d_out,
	                          ws, have, stream, stream_err(st, reinterpret_cast<hipStream_t>(stream)));
}

// ---- XXH3-64 (include/fdb_xxh3.h) -------------------------------------------

int xxh3_gpu_batch_fixed(const void* d_base, uint64_t stride, uint64_t length, uint64_t count, uint64_t seed,
                         const uint64_t* d_seeds, uint64_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || (!d_base && length)) return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_fixed: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	fdbxxh::XxhParams P{};
	P.base = static_cast<const uint8_t*>(d_base);
	P.stride = stride;
	P.length = length;
	P.count = count;
	P.seed = seed;
	P.seeds = d_seeds;
	P.out = d_out;
	if (length > fdbxxh::kXSplitMin) {
		// long buffers: the split route (every 1 KiB block of the batch in
		// parallel), planned in the stream's workspace
		const uint64_t nw = fdbxxh::xxh3_nwave(st->num_cus);
		const uint64_t nb = count * (((length - 1) >> 10) + 1);
		void* ws = nullptr;
		uint64_t have = 0;
		std::unique_lock<std::mutex> hold;
		if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
		                              fdbxxh::xxh3_workspace_bytes_for(count, nw, nb), &ws, &have, &hold))
			return rc;
		P.ws_bytes = have;
		if (fdbxxh::launch_xxh3(P, st->num_cus, ws, reinterpret_cast<hipStream_t>(stream)))
			return fail(FDB_CRC32C_EHIP, "xxh3_gpu_batch_fixed: launch setup failed");
		return check_launch("xxh3_gpu_batch_fixed launch");
	}
	if (fdbxxh::launch_xxh3(P, st->num_cus, nullptr, reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "xxh3_gpu_batch_fixed: launch setup failed");
	return check_launch("xxh3_gpu_batch_fixed launch");
}

uint64_t xxh3_gpu_varlen_workspace_bytes(uint64_t count) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return fdbxxh::xxh3_workspace_bytes(count, fdbxxh::xxh3_nwave(st->num_cus));
}

uint64_t xxh3_gpu_varlen_workspace_bytes_for(uint64_t count, uint64_t total_bytes) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return fdbxxh::xxh3_workspace_bytes_for(count, fdbxxh::xxh3_nwave(st->num_cus),
	                                        fdbxxh::xxh3_long_blocks_bound(total_bytes));
}

static int xxh3_varlen_impl(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                            uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* d_workspace,
                            uint64_t workspace_bytes, void* stream, uint64_t* hneed, uint32_t* err = nullptr) {
	if (count == 0) return 0;
	if (!d_out || !d_offsets || !d_lengths || !d_base)
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_varlen: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const uint64_t need = fdbxxh::xxh3_workspace_bytes(count, fdbxxh::xxh3_nwave(st->num_cus));
	if (!d_workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_varlen: workspace too small or misaligned");
	fdbxxh::XxhParams P{};
	P.base = static_cast<const uint8_t*>(d_base);
	P.offsets = d_offsets;
	P.lengths = d_lengths;
	P.count = count;
	P.seed = seed;
	P.seeds = d_seeds;
	P.out = d_out;
	P.ws_bytes = workspace_bytes;
	P.hneed = hneed;
	P.err = err;
	if (fdbxxh::launch_xxh3(P, st->num_cus, d_workspace, reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "xxh3_gpu_batch_varlen: launch setup failed");
	return check_launch("xxh3_gpu_batch_varlen launch");
}

int xxh3_gpu_batch_varlen_ws(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                             uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* d_workspace,
                             uint64_t workspace_bytes, void* stream) {
	return xxh3_varlen_impl(d_base, d_offsets, d_lengths, count, seed, d_seeds, d_out, d_workspace, workspace_bytes,
	                        stream, nullptr);
}

// The library's workspace for the stream: the planner's arrays plus room for
// the split route sized from the long blocks the stream's last batch needed
// (recorded by the device in host-mapped memory; a batch needing more than
// the room runs its long buffers on the row kernel, and the next call grows).
int xxh3_gpu_batch_varlen(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                          uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || !d_offsets || !d_lengths || !d_base)
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_varlen: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	StreamState* ss = stream_state(st, s);
	bool mapped;
	{
		std::lock_guard<std::mutex> lock(g_mu);
		mapped = stream_mapped(ss);
	}
	const uint64_t last = mapped ? *reinterpret_cast<volatile uint64_t*>(ss->hst_h + kHstatXxhNeed) : 0;
	const uint64_t room = last + last / 4;
	const uint64_t want = fdbxxh::xxh3_workspace_bytes_for(count, fdbxxh::xxh3_nwave(st->num_cus), room);
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, s, want, &ws, &have, &hold)) return rc;
	// (the room asked for, not the whole workspace: no long buffers last time, no split launches now)
	return xxh3_varlen_impl(d_base, d_offsets, d_lengths, count, seed, d_seeds, d_out, ws, want < have ? want : have,
	                        stream, mapped ? ss->hst_d + kHstatXxhNeed : nullptr,
	                        mapped ? reinterpret_cast<uint32_t*>(ss->hst_d + kHstatErr) : nullptr);
}

uint64_t xxh3_gpu_chained_workspace_bytes(uint64_t nsegs, uint64_t nchains, uint64_t total_bytes) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return fdbxxh::xxh3_chain_workspace_bytes(nsegs, nchains, total_bytes, fdbxxh::xxh3_nwave(st->num_cus));
}

int xxh3_gpu_batch_chained_ws(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                              uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint64_t total_bytes,
                              uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* d_workspace,
                              uint64_t workspace_bytes, void* stream) {
	if (nchains == 0) return 0;
	if (!d_out || !d_chain_starts || (nsegs && (!d_base || !d_seg_offsets || !d_seg_lengths)))
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_chained: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const uint64_t need = fdbxxh::xxh3_chain_workspace_bytes(nsegs, nchains, total_bytes, fdbxxh::xxh3_nwave(st->num_cus));
	if (!d_workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_chained: workspace too small or misaligned");
	if (fdbxxh::launch_xxh3_chained(static_cast<const uint8_t*>(d_base), d_seg_offsets, d_seg_lengths, nsegs,
	                                d_chain_starts, nchains, total_bytes, seed, d_seeds, d_out, st->num_cus, d_workspace,
	                                reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "xxh3_gpu_batch_chained: launch setup failed");
	return check_launch("xxh3_gpu_batch_chained launch");
}

int xxh3_gpu_batch_chained(const void* d_base, const uint64_t* d_seg_offsets, const uint64_t* d_seg_lengths,
                           uint64_t nsegs, const uint64_t* d_chain_starts, uint64_t nchains, uint64_t total_bytes,
                           uint64_t seed, const uint64_t* d_seeds, uint64_t* d_out, void* stream) {
	if (nchains == 0) return 0;
	if (!d_out || !d_chain_starts || (nsegs && (!d_base || !d_seg_offsets || !d_seg_lengths)))
		return fail(FDB_CRC32C_EINVAL, "xxh3_gpu_batch_chained: null pointer");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
	                              fdbxxh::xxh3_chain_workspace_bytes(nsegs, nchains, total_bytes,
	                                                                 fdbxxh::xxh3_nwave(st->num_cus)),
	                              &ws, &have, &hold))
		return rc;
	return xxh3_gpu_batch_chained_ws(d_base, d_seg_offsets, d_seg_lengths, nsegs, d_chain_starts, nchains, total_bytes,
	                                 seed, d_seeds, d_out, ws, have, stream);
}

// ---- page verifiers (include/fdb_pagecheck.h) ---------------------------------

uint64_t fdb_pagecheck_workspace_bytes(uint64_t count) { return fdbpc::workspace_bytes(count); }

static int pages_ok(const void* d_pages, uint64_t page_size, uint64_t count, const void* d_out, const char* who) {
	if (!d_pages || !d_out) return fail(FDB_CRC32C_EINVAL, who);
	if (reinterpret_cast<uintptr_t>(d_pages) % 16) return fail(FDB_CRC32C_EINVAL, "pages must be 16-byte aligned");
	// multiples of 16: every page then starts 16-byte aligned, as the kernels'
	// 16-byte vector loads require (SQLite page sizes are powers of two >= 512)
	if (page_size % 16 || page_size <= 248 || page_size >= (1ull << 31))
		return fail(FDB_CRC32C_EINVAL, "page_size must be a multiple of 16 in (248, 2^31)");
	if (count >= (1ull << 32)) return fail(FDB_CRC32C_EINVAL, "count must be < 2^32");
	return 0;
}

int fdb_sqlite_verify_pages_ws(const void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno,
                               uint8_t* d_status, uint64_t* d_bad, void* d_workspace, uint64_t workspace_bytes,
                               void* stream) {
	if (count == 0) {
		if (d_bad) (void)hipMemsetAsync(d_bad, 0, 8, reinterpret_cast<hipStream_t>(stream));
		return 0;
	}
	if (int rc = pages_ok(d_pages, page_size, count, d_status, "fdb_sqlite_verify_pages: null pointer")) return rc;
	if (!d_workspace || workspace_bytes < fdbpc::workspace_bytes(count) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_sqlite_verify_pages: workspace too small or misaligned");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	uint64_t* aux = nullptr;
	std::unique_lock<std::mutex> aux_hold;  // until the call's last launch
	if (int rc = stream_aux(reinterpret_cast<hipStream_t>(stream), &aux, &aux_hold)) return rc;
	if (fdbpc::sqlite_verify(static_cast<const uint8_t*>(d_pages), page_size, count, first_pgno, d_status, d_bad,
	                         st->tables, st->num_cus, d_workspace,
	                         reinterpret_cast<unsigned long long*>(aux + kAuxPageCtr),
	                         reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_sqlite_verify_pages: launch setup failed");
	return check_launch("fdb_sqlite_verify_pages launch");
}

int fdb_sqlite_verify_pages(const void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno,
                            uint8_t* d_status, uint64_t* d_bad, void* stream) {
	if (count == 0) return fdb_sqlite_verify_pages_ws(d_pages, page_size, 0, first_pgno, d_status, d_bad, nullptr, 0,
	                                                  stream);
	if (int rc = pages_ok(d_pages, page_size, count, d_status, "fdb_sqlite_verify_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), fdbpc::workspace_bytes(count), &ws, &have,
	                              &hold))
		return rc;
	return fdb_sqlite_verify_pages_ws(d_pages, page_size, count, first_pgno, d_status, d_bad, ws, have, stream);
}

int fdb_diskqueue_check_pages_ws(const void* d_pages, uint64_t count, uint8_t* d_ok, uint64_t* d_bad,
                                 void* d_workspace, uint64_t workspace_bytes, void* stream) {
	if (count == 0) {
		if (d_bad) (void)hipMemsetAsync(d_bad, 0, 8, reinterpret_cast<hipStream_t>(stream));
		return 0;
	}
	if (int rc = pages_ok(d_pages, 4096, count, d_ok, "fdb_diskqueue_check_pages: null pointer")) return rc;
	if (!d_workspace || workspace_bytes < fdbpc::workspace_bytes(count) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_diskqueue_check_pages: workspace too small or misaligned");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	uint64_t* aux = nullptr;
	std::unique_lock<std::mutex> aux_hold;  // until the call's last launch
	if (int rc = stream_aux(reinterpret_cast<hipStream_t>(stream), &aux, &aux_hold)) return rc;
	if (fdbpc::diskqueue_check(static_cast<const uint8_t*>(d_pages), count, d_ok, d_bad, st->tables, st->num_cus,
	                           d_workspace, reinterpret_cast<unsigned long long*>(aux + kAuxPageCtr),
	                           reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_diskqueue_check_pages: launch setup failed");
	return check_launch("fdb_diskqueue_check_pages launch");
}

int fdb_diskqueue_check_pages(const void* d_pages, uint64_t count, uint8_t* d_ok, uint64_t* d_bad, void* stream) {
	if (count == 0) return fdb_diskqueue_check_pages_ws(d_pages, 0, d_ok, d_bad, nullptr, 0, stream);
	if (int rc = pages_ok(d_pages, 4096, count, d_ok, "fdb_diskqueue_check_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), fdbpc::workspace_bytes(count), &ws, &have,
	                              &hold))
		return rc;
	return fdb_diskqueue_check_pages_ws(d_pages, count, d_ok, d_bad, ws, have, stream);
}

// ---- the write side: sealing pages in place ----------------------------------
int fdb_sqlite_seal_pages_ws(void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno, void* d_workspace,
                             uint64_t workspace_bytes, void* stream) {
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, page_size, count, d_pages, "fdb_sqlite_seal_pages: null pointer")) return rc;
	if (!d_workspace || workspace_bytes < fdbpc::workspace_bytes(count) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_sqlite_seal_pages: workspace too small or misaligned");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	if (fdbpc::sqlite_seal(static_cast<uint8_t*>(d_pages), page_size, count, first_pgno, st->num_cus, d_workspace,
	                       reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_sqlite_seal_pages: launch setup failed");
	return check_launch("fdb_sqlite_seal_pages launch");
}

int fdb_sqlite_seal_pages(void* d_pages, uint64_t page_size, uint64_t count, uint32_t first_pgno, void* stream) {
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, page_size, count, d_pages, "fdb_sqlite_seal_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), fdbpc::workspace_bytes(count), &ws, &have,
	                              &hold))
		return rc;
	return fdb_sqlite_seal_pages_ws(d_pages, page_size, count, first_pgno, ws, have, stream);
}

// ---- the pager's codec hook over a batch (PageChecksumCodec::codec) ----------
int fdb_sqlite_codec_pages_ws(void* d_pages, uint64_t page_size, uint32_t reserve_size, uint64_t count,
                              uint32_t first_pgno, int op, uint8_t* d_status, void* d_workspace,
                              uint64_t workspace_bytes, void* stream) {
	// KeyValueStoreSQLite.cpp:206-208: writes are ops 6 (db page) and 7 (journal page); anything else must be 3
	if (op != 3 && op != 6 && op != 7)
		return fail(FDB_CRC32C_EINVAL, "fdb_sqlite_codec_pages: op must be 3 (read), 6 or 7 (write)");
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, page_size, count, d_status, "fdb_sqlite_codec_pages: null pointer")) return rc;
	if (!d_workspace || workspace_bytes < fdbpc::workspace_bytes(count) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_sqlite_codec_pages: workspace too small or misaligned");
	const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	const bool write = op != 3;
	auto seal_status = [&](uint8_t* st, uint64_t n) -> int {  // a sealed page: codec() returns it (XXH3 trailer)
		hipError_t e = hipMemsetAsync(st, 2, n, s);
		return e == hipSuccess ? 0 : fail(FDB_CRC32C_EHIP, "fdb_sqlite_codec_pages: hipMemsetAsync", e);
	};
	if (reserve_size == 8) {  // sizeof(SumType): every page goes through checksum()
		if (write) {
			if (int rc = fdb_sqlite_seal_pages_ws(d_pages, page_size, count, first_pgno, d_workspace, workspace_bytes,
			                                      stream))
				return rc;
			return seal_status(d_status, count);
		}
		return fdb_sqlite_verify_pages_ws(d_pages, page_size, count, first_pgno, d_status, nullptr, d_workspace,
		                                  workspace_bytes, stream);
	}
	// any other reserve size: codec() returns nullptr for every page but page 1
	// and leaves it untouched (:225-237); page 1 is checksummed as usual
	hipError_t e = hipMemsetAsync(d_status, 0, count, s);
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, "fdb_sqlite_codec_pages: hipMemsetAsync", e);
	const uint64_t i1 = (uint32_t)(1u - first_pgno);
	if (i1 >= count) return 0;
	uint8_t* p1 = static_cast<uint8_t*>(d_pages) + i1 * page_size;
	if (write) {
		if (int rc = fdb_sqlite_seal_pages_ws(p1, page_size, 1, 1, d_workspace, workspace_bytes, stream)) return rc;
		return seal_status(d_status + i1, 1);
	}
	return fdb_sqlite_verify_pages_ws(p1, page_size, 1, 1, d_status + i1, nullptr, d_workspace, workspace_bytes, stream);
}

int fdb_sqlite_codec_pages(void* d_pages, uint64_t page_size, uint32_t reserve_size, uint64_t count,
                           uint32_t first_pgno, int op, uint8_t* d_status, void* stream) {
	if (op != 3 && op != 6 && op != 7)
		return fail(FDB_CRC32C_EINVAL, "fdb_sqlite_codec_pages: op must be 3 (read), 6 or 7 (write)");
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, page_size, count, d_status, "fdb_sqlite_codec_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), fdbpc::workspace_bytes(count), &ws, &have,
	                              &hold))
		return rc;
	return fdb_sqlite_codec_pages_ws(d_pages, page_size, reserve_size, count, first_pgno, op, d_status, ws, have, stream);
}

int fdb_diskqueue_seal_pages_ws(void* d_pages, uint64_t count, void* d_workspace, uint64_t workspace_bytes,
                                void* stream) {
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, 4096, count, d_pages, "fdb_diskqueue_seal_pages: null pointer")) return rc;
	if (!d_workspace || workspace_bytes < fdbpc::workspace_bytes(count) || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_diskqueue_seal_pages: workspace too small or misaligned");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	uint64_t* aux = nullptr;
	std::unique_lock<std::mutex> aux_hold;  // until the call's last launch
	if (int rc = stream_aux(reinterpret_cast<hipStream_t>(stream), &aux, &aux_hold)) return rc;
	if (fdbpc::diskqueue_seal(static_cast<uint8_t*>(d_pages), count, st->tables, st->num_cus, d_workspace,
	                          reinterpret_cast<unsigned long long*>(aux + kAuxPageCtr),
	                          reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_diskqueue_seal_pages: launch setup failed");
	return check_launch("fdb_diskqueue_seal_pages launch");
}

int fdb_diskqueue_seal_pages(void* d_pages, uint64_t count, void* stream) {
	if (count == 0) return 0;
	if (int rc = pages_ok(d_pages, 4096, count, d_pages, "fdb_diskqueue_seal_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream), fdbpc::workspace_bytes(count), &ws, &have,
	                              &hold))
		return rc;
	return fdb_diskqueue_seal_pages_ws(d_pages, count, ws, have, stream);
}

// ---- Redwood pages (include/fdb_redwood.h) ----------------------------------
static int redwood_args(const void* d_pages, uint64_t page_size, uint64_t count, const char* who) {
	if (!d_pages) return fail(FDB_CRC32C_EINVAL, who);
	if (page_size % 16 || page_size < 512 || page_size >= (1ull << 31))
		return fail(FDB_CRC32C_EINVAL, "redwood pages: page_size must be a multiple of 16 in [512, 2^31)");
	if (reinterpret_cast<uintptr_t>(d_pages) % 16) return fail(FDB_CRC32C_EINVAL, "redwood pages: pages not 16-byte aligned");
	if (count > 0xFFFFFFFFull) return fail(FDB_CRC32C_EINVAL, "redwood pages: more than 2^32 - 1 pages");
	return 0;
}

uint64_t fdb_redwood_workspace_bytes(uint64_t count, uint64_t page_size) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return fdbrw::workspace_bytes(count, page_size, st->num_cus);
}

int fdb_redwood_verify_pages_ws(const void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                                uint32_t first_page_id, uint8_t* d_status, uint64_t* d_bad, void* d_workspace,
                                uint64_t workspace_bytes, void* stream) {
	const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	if (count == 0) {
		if (d_bad) (void)hipMemsetAsync(d_bad, 0, 8, s);
		return 0;
	}
	if (int rc = redwood_args(d_pages, page_size, count, "fdb_redwood_verify_pages: null pointer")) return rc;
	if (!d_status) return fail(FDB_CRC32C_EINVAL, "fdb_redwood_verify_pages: null status");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	if (!d_workspace || workspace_bytes < fdbrw::workspace_bytes(count, page_size, st->num_cus) ||
	    reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_redwood_verify_pages: workspace too small or misaligned");
	if (fdbrw::verify(static_cast<const uint8_t*>(d_pages), page_size, count, d_page_ids, first_page_id, d_status,
	                  d_bad, st->num_cus, d_workspace, workspace_bytes, s))
		return fail(FDB_CRC32C_EHIP, "fdb_redwood_verify_pages: launch setup failed");
	return check_launch("fdb_redwood_verify_pages launch");
}

int fdb_redwood_verify_pages(const void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                             uint32_t first_page_id, uint8_t* d_status, uint64_t* d_bad, void* stream) {
	if (count == 0)
		return fdb_redwood_verify_pages_ws(d_pages, page_size, 0, d_page_ids, first_page_id, d_status, d_bad, nullptr,
		                                   0, stream);
	if (int rc = redwood_args(d_pages, page_size, count, "fdb_redwood_verify_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
	                              fdbrw::workspace_bytes(count, page_size, st->num_cus), &ws, &have, &hold))
		return rc;
	return fdb_redwood_verify_pages_ws(d_pages, page_size, count, d_page_ids, first_page_id, d_status, d_bad, ws, have,
	                                   stream);
}

int fdb_redwood_seal_pages_ws(void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                              uint32_t first_page_id, uint8_t* d_status, void* d_workspace, uint64_t workspace_bytes,
                              void* stream) {
	if (count == 0) return 0;
	if (int rc = redwood_args(d_pages, page_size, count, "fdb_redwood_seal_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	if (!d_workspace || workspace_bytes < fdbrw::workspace_bytes(count, page_size, st->num_cus) ||
	    reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_redwood_seal_pages: workspace too small or misaligned");
	if (fdbrw::seal(static_cast<uint8_t*>(d_pages), page_size, count, d_page_ids, first_page_id, d_status, st->num_cus,
	                d_workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_redwood_seal_pages: launch setup failed");
	return check_launch("fdb_redwood_seal_pages launch");
}

int fdb_redwood_seal_pages(void* d_pages, uint64_t page_size, uint64_t count, const uint32_t* d_page_ids,
                           uint32_t first_page_id, uint8_t* d_status, void* stream) {
	if (count == 0) return 0;
	if (int rc = redwood_args(d_pages, page_size, count, "fdb_redwood_seal_pages: null pointer")) return rc;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
	                              fdbrw::workspace_bytes(count, page_size, st->num_cus), &ws, &have, &hold))
		return rc;
	return fdb_redwood_seal_pages_ws(d_pages, page_size, count, d_page_ids, first_page_id, d_status, ws, have, stream);
}

// ---- FlowTransport receive verification (include/fdb_packets.h) ------------

uint64_t fdb_packets_workspace_bytes(uint64_t nbuf, uint64_t max_frames, uint64_t total_bytes) {
	DeviceState* st = nullptr;
	if (device_state(&st)) return 0;
	return fdbpkt::workspace_bytes(nbuf, max_frames, total_bytes, st->num_cus);
}

int fdb_packets_verify_ws(const void* d_base, const uint64_t* d_buf_offsets, const uint64_t* d_buf_lengths,
                          uint64_t nbuf, uint64_t total_bytes, int checksum_enabled, uint32_t packet_limit,
                          uint64_t max_frames, fdb_packet_result* d_results, void* d_workspace,
                          uint64_t workspace_bytes, void* stream) {
	if (nbuf == 0) return 0;
	if (!d_base || !d_buf_offsets || !d_buf_lengths || !d_results)
		return fail(FDB_CRC32C_EINVAL, "fdb_packets_verify: null pointer");
	if (nbuf >= 0xFFFFFFFFull || max_frames >= 0xFFFFFFFFull)
		return fail(FDB_CRC32C_EINVAL, "fdb_packets_verify: nbuf and max_frames must be below 2^32");
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	const uint64_t need = fdbpkt::workspace_bytes(nbuf, max_frames, total_bytes, st->num_cus);
	if (!d_workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(d_workspace) % 16)
		return fail(FDB_CRC32C_EINVAL, "fdb_packets_verify: workspace too small or misaligned");
	const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	uint64_t* aux = nullptr;
	std::unique_lock<std::mutex> aux_hold;  // until the call's last launch
	if (int rc = stream_aux(s, &aux, &aux_hold)) return rc;
	// the split route's room from the long frames the stream's last batch
	// needed (host-mapped, no synchronisation; a stale hint costs speed only:
	// long frames past the room are hashed by the row kernel, and the next call
	// grows the room)
	StreamState* ss = stream_state(st, s);
	bool mapped;
	{
		std::lock_guard<std::mutex> lock(g_mu);
		mapped = stream_mapped(ss);
	}
	const uint64_t last = mapped ? *reinterpret_cast<volatile uint64_t*>(ss->hst_h + kHstatXxhNeed) : ~0ull;
	const uint64_t room = mapped ? last + last / 4 : ~0ull;
	if (fdbpkt::launch_verify(static_cast<const uint8_t*>(d_base), d_buf_offsets, d_buf_lengths, nbuf,
	                          checksum_enabled ? 1 : 0, packet_limit, max_frames, d_results, d_workspace,
	                          workspace_bytes, st->num_cus, aux + kAuxPktFrames, room,
	                          mapped ? ss->hst_d + kHstatXxhNeed : nullptr, s))
		return fail(FDB_CRC32C_EHIP, "fdb_packets_verify: launch setup failed");
	return check_launch("fdb_packets_verify launch");
}

int fdb_packets_verify(const void* d_base, const uint64_t* d_buf_offsets, const uint64_t* d_buf_lengths,
                       uint64_t nbuf, uint64_t total_bytes, int checksum_enabled, uint32_t packet_limit,
                       uint64_t max_frames, fdb_packet_result* d_results, void* stream) {
	if (nbuf == 0) return 0;
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	void* ws = nullptr;
	uint64_t have = 0;
	std::unique_lock<std::mutex> hold;
	if (int rc = stream_workspace(st, reinterpret_cast<hipStream_t>(stream),
	                              fdbpkt::workspace_bytes(nbuf, max_frames, total_bytes, st->num_cus), &ws, &have,
	                              &hold))
		return rc;
	return fdb_packets_verify_ws(d_base, d_buf_offsets, d_buf_lengths, nbuf, total_bytes, checksum_enabled,
	                             packet_limit, max_frames, d_results, ws, have, stream);
}

int fdb_packets_frames(const void* d_workspace, uint64_t nbuf, uint64_t max_frames, fdb_packet_frame* d_frames,
                       uint64_t capacity, uint64_t* d_nframes, void* stream) {
	if (!d_workspace || (capacity && !d_frames)) return fail(FDB_CRC32C_EINVAL, "fdb_packets_frames: null pointer");
	void* xws = nullptr;
	uint64_t xb = 0;
	const fdbpkt::Ws w = fdbpkt::carve(const_cast<void*>(d_workspace), nbuf, max_frames, ~0ull >> 1, &xws, &xb);
	if (fdbpkt::launch_frames(w, nbuf, d_frames, capacity, d_nframes, reinterpret_cast<hipStream_t>(stream)))
		return fail(FDB_CRC32C_EHIP, "fdb_packets_frames: launch setup failed");
	return check_launch("fdb_packets_frames launch");
}

int crc32c_gpu_release_stream(void* stream) { return release_stream(reinterpret_cast<hipStream_t>(stream)); }

int crc32c_gpu_stream_status(void* stream) {
	DeviceState* st = nullptr;
	if (int rc = device_state(&st)) return rc;
	hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	hipError_t e = hipStreamSynchronize(s);
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, "crc32c_gpu_stream_status: hipStreamSynchronize", e);
	StreamState* ss = stream_state(st, s);
	std::lock_guard<std::mutex> lock(g_mu);
	if (!ss->hst_h) return 0;
	volatile uint32_t* w = reinterpret_cast<volatile uint32_t*>(ss->hst_h + kHstatErr);
	const uint32_t v = *w;
	if (!v) return 0;
	*w = 0;
	if (v == fdbxxh::kErrXxhStall)
		return fail(FDB_CRC32C_EHIP, "an XXH3 batch on this stream stalled on the device (a long-route wait ran out); "
		                             "some of its digests were not written");
	return fail(FDB_CRC32C_EINVAL, "a variable-length batch on this stream was refused: it covered 2^32 - 1 or more "
	                               "1 KiB windows (or 4 KiB blocks); its checksums are undefined");
}

int crc32c_gpu_workspace_status(const void* d_workspace, void* stream) {
	if (!d_workspace) return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_workspace_status: null workspace");
	uint64_t flag = 0;
	hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	hipError_t e = hipMemcpyAsync(&flag, varlen_refused_word(d_workspace), 8, hipMemcpyDeviceToHost, s);
	if (e == hipSuccess) e = hipStreamSynchronize(s);
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, "crc32c_gpu_workspace_status", e);
	if (flag != 1) return 0;
	return fail(FDB_CRC32C_EINVAL, "the last variable-length batch in this workspace was refused: it covered 2^32 - 1 "
	                               "or more 1 KiB windows (or 4 KiB blocks); its checksums are undefined");
}

uint64_t crc32c_gpu_stream_bytes(void* stream) { return stream_bytes(reinterpret_cast<hipStream_t>(stream)); }

const char* crc32c_gpu_last_error(void) { return t_err.c_str(); }

const char* crc32c_gpu_version(void) { return "fdb_crc32c 0.1 gfx950"; }



}  // extern "C"
