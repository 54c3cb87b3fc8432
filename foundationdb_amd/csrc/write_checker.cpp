// Batched lost-write checker (include/fdb_writechecker.h).
//
// The history bookkeeping restates fdbrpc/AsyncFileWriteChecker.h; every rule
// below cites the lines it follows.  The checksums of all full pages of one
// I/O are computed as one batch by the engine (host CRC, the pinned GPU
// pipeline, or an asynchronous device batch), then applied to the history in
// submission order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <deque>
#include <map>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fdb_crc32c.h"
#include "../../include/fdb_writechecker.h"

namespace fdbcrc {
int set_error(int code, const char* what, hipError_t e);
}

namespace {

constexpr int64_t kPage = 4096;             // checksumHistoryPageSize
constexpr uint32_t kSeed = 0xab12fd93u;     // AsyncFileWriteChecker.h:298

// The process-wide history budget (AsyncFileWriteChecker.h:222-227): set by
// the first checker, shared by all.
std::mutex g_budget_mu;
bool g_budget_set = false;
int64_t g_budget = 0;

struct WriteInfo {
	uint32_t checksum = 0;
	uint64_t timestamp = 0;
};

// AsyncFileWriteChecker.h:107-194, same containers and the same behaviour
// (truncate() leaves pageContents behind; only keyToStep decides existence).
class LRU {
public:
	void update(uint32_t page, WriteInfo info) {
		auto it = keyToStep.find(page);
		if (it != keyToStep.end()) stepToKey.erase(it->second);
		keyToStep[page] = step;
		stepToKey[step] = page;
		pageContents[page] = info;
		++step;
	}
	void truncate(uint32_t page) {
		for (auto it = keyToStep.lower_bound(page); it != keyToStep.end();) {
			stepToKey.erase(it->second);
			it = keyToStep.erase(it);
		}
	}
	int64_t size() const { return (int64_t)keyToStep.size(); }
	bool exist(uint32_t page) const { return keyToStep.count(page) != 0; }
	WriteInfo find(uint32_t page) {
		if (!exist(page)) return WriteInfo();
		return pageContents[page];
	}
	void remove(uint32_t page) {
		auto it = keyToStep.find(page);
		if (it == keyToStep.end()) return;
		pageContents.erase(page);
		stepToKey.erase(it->second);
		keyToStep.erase(it);
	}
	// Pages from the least recently used on (leastRecentlyUsedPage, :168-173,
	// walked forward), stopping before the first page `stop` rejects.
	template <class Stop>
	uint64_t lru_order(uint32_t* out, uint64_t cap, Stop stop) const {
		uint64_t n = 0;
		for (auto it = stepToKey.begin(); it != stepToKey.end() && n < cap; ++it) {
			if (stop(it->second)) break;
			out[n++] = it->second;
		}
		return n;
	}

private:
	uint64_t step = 0;
	std::map<uint64_t, uint32_t> stepToKey;
	std::map<uint32_t, uint64_t> keyToStep;
	std::unordered_map<uint32_t, WriteInfo> pageContents;
};

// Full pages of [offset, offset+len) as updateChecksumHistory numbers them
// (:287-297): first page number, bytes to skip in the buffer, and the
// exclusive end page number (the reference's `pageEnd`, which leaves out the
// last full page).
struct Span {
	uint32_t page, end;
	int64_t skip;
	uint64_t count() const { return end > page ? end - page : 0; }
};
Span span_of(int64_t offset, int64_t len) {
	Span s;
	s.page = (uint32_t)(offset / kPage + 1);
	const int64_t slack = offset % kPage;
	s.skip = 0;
	if (slack != 0) {
		++s.page;
		s.skip = kPage - slack;
	}
	s.end = (uint32_t)((offset + len) / kPage);
	return s;
}

struct Scratch {  // device + pinned result buffers of one queued batch
	uint32_t* d = nullptr;
	uint32_t* h = nullptr;
	uint64_t cap = 0;
	hipEvent_t ev = nullptr;
};

struct Op {
	enum Kind { kWrite, kRead } kind;
	Span sp;
	uint64_t now_ms;
	uint64_t ticket;
	Scratch sc;
	bool device;
};

}  // namespace

struct fdb_write_checker {
	LRU lru;
	std::unordered_set<uint32_t> writing;
	uint64_t synced = 0;  // syncedTime
	uint64_t succeed = 0, failed = 0;
	uint64_t gpu_threshold = 64;
	fdb_crc32c_pipeline* pipe = nullptr;
	hipStream_t stream = nullptr;
	std::deque<Op> queue;
	std::vector<Scratch> pool;
	uint64_t next_ticket = 1, applied = 0;
	std::vector<uint32_t> crcs;

	// ---- history rules --------------------------------------------------
	// updateChecksumHistory(true, ...), :299-324
	void apply_write(const Span& sp, const uint32_t* c, uint64_t now_ms, std::vector<uint32_t>* pages) {
		uint64_t k = 0;
		for (uint32_t p = sp.page; p < sp.end; ++p, ++k) {
			writing.insert(p);
			if (pages) pages->push_back(p);
			if (!lru.exist(p)) {
				std::lock_guard<std::mutex> g(g_budget_mu);
				if (g_budget > 0)
					g_budget -= 1;
				else
					break;  // SkippedPagesDuringUpdateChecksum
			}
			WriteInfo w;
			w.timestamp = now_ms;
			w.checksum = c[k];
			lru.update(p, w);
		}
	}
	// verifyChecksum, :244-275
	int verify(uint32_t p, uint32_t checksum, uint64_t* fails) {
		if (!lru.exist(p)) return 1;
		const WriteInfo h = lru.find(p);
		if (h.timestamp < synced) {
			if (h.checksum != checksum) {
				++failed;  // AsyncFileLostWriteDetected
				if (fails) ++*fails;
			} else {
				{
					std::lock_guard<std::mutex> g(g_budget_mu);
					g_budget += 1;
				}
				lru.remove(p);
				++succeed;
			}
			return 1;
		}
		return 0;
	}
	// updateChecksumHistory(false, ...), :325-330
	void apply_read(const Span& sp, const uint32_t* c, uint64_t* fails) {
		uint64_t k = 0;
		for (uint32_t p = sp.page; p < sp.end; ++p, ++k)
			if (!verify(p, c[k], fails)) break;
	}

	// ---- checksum batches ------------------------------------------------
	int host_crcs(const void* buf, const Span& sp) {
		const uint64_t n = sp.count();
		crcs.resize(n);
		if (!n) return 0;
		const uint8_t* base = static_cast<const uint8_t*>(buf) + sp.skip;
		if (gpu_threshold && n >= gpu_threshold) {
			if (!pipe)
				if (int rc = crc32c_pipeline_create(&pipe, 16u << 20, 2)) return rc;
			return crc32c_pipeline_fixed(pipe, base, kPage, kPage, n, kSeed, nullptr, crcs.data());
		}
		for (uint64_t i = 0; i < n; ++i) crcs[i] = crc32c_append(kSeed, base + i * kPage, (size_t)kPage);
		return 0;
	}

	int scratch(uint64_t n, Scratch* out) {
		for (size_t i = 0; i < pool.size(); ++i)
			if (pool[i].cap >= n) {
				*out = pool[i];
				pool.erase(pool.begin() + i);
				return 0;
			}
		Scratch s;
		s.cap = n < 1024 ? 1024 : n;
		hipError_t e = hipMalloc(reinterpret_cast<void**>(&s.d), 4 * s.cap);
		if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.h), 4 * s.cap, hipHostMallocDefault);
		if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming);
		if (e != hipSuccess) return fdbcrc::set_error(FDB_CRC32C_ENOMEM, "write checker scratch", e);
		*out = s;
		return 0;
	}

	int submit_device(Op::Kind kind, const void* d_buf, int64_t length, int64_t offset, uint64_t now_ms,
	                  uint64_t* ticket) {
		if (!stream) {
			hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
			if (e != hipSuccess) return fdbcrc::set_error(FDB_CRC32C_EHIP, "write checker stream", e);
		}
		Op op;
		op.kind = kind;
		op.sp = span_of(offset, length);
		op.now_ms = now_ms;
		op.device = true;
		const uint64_t n = op.sp.count();
		if (n) {
			if (int rc = scratch(n, &op.sc)) return rc;
			const uint8_t* base = static_cast<const uint8_t*>(d_buf) + op.sp.skip;
			if (int rc = crc32c_gpu_batch_fixed(base, kPage, kPage, n, kSeed, nullptr, op.sc.d, stream)) return rc;
			hipError_t e = hipMemcpyAsync(op.sc.h, op.sc.d, 4 * n, hipMemcpyDeviceToHost, stream);
			if (e == hipSuccess) e = hipEventRecord(op.sc.ev, stream);
			if (e != hipSuccess) return fdbcrc::set_error(FDB_CRC32C_EHIP, "write checker D2H", e);
		}
		op.ticket = next_ticket++;
		if (ticket) *ticket = op.ticket;
		queue.push_back(op);
		return 0;
	}

	void apply_front() {
		Op op = queue.front();
		queue.pop_front();
		const uint32_t* c = op.sc.h;
		if (op.kind == Op::kWrite)
			apply_write(op.sp, c, op.now_ms, nullptr);
		else
			apply_read(op.sp, c, nullptr);
		if (op.sc.cap) pool.push_back(op.sc);
		applied = op.ticket;
	}

	int poll() {
		while (!queue.empty()) {
			const Op& f = queue.front();
			if (f.sp.count()) {
				const hipError_t e = hipEventQuery(f.sc.ev);
				if (e == hipErrorNotReady) return 0;
				if (e != hipSuccess) return fdbcrc::set_error(FDB_CRC32C_EHIP, "write checker poll", e);
			}
			apply_front();
		}
		return 0;
	}

	int wait(uint64_t ticket) {
		while (!queue.empty() && applied < ticket) {
			const Op& f = queue.front();
			if (f.sp.count()) {
				const hipError_t e = hipEventSynchronize(f.sc.ev);
				if (e != hipSuccess) return fdbcrc::set_error(FDB_CRC32C_EHIP, "write checker wait", e);
			}
			apply_front();
		}
		return 0;
	}
	int drain() { return wait(~uint64_t(0)); }

	~fdb_write_checker() {
		(void)drain();
		for (auto& s : pool) {
			(void)hipFree(s.d);
			(void)hipHostFree(s.h);
			(void)hipEventDestroy(s.ev);
		}
		if (stream) {
			(void)crc32c_gpu_release_stream(stream);
			(void)hipStreamDestroy(stream);
		}
		if (pipe) crc32c_pipeline_destroy(pipe);
	}
};

extern "C" {

int fdb_wc_create(fdb_write_checker** out, int64_t history_budget) {
	if (!out) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_create: null", hipSuccess);
	{
		std::lock_guard<std::mutex> g(g_budget_mu);
		if (!g_budget_set) {
			g_budget = history_budget;
			g_budget_set = true;
		}
	}
	*out = new fdb_write_checker();
	return 0;
}

void fdb_wc_destroy(fdb_write_checker* wc) {
	if (!wc) return;
	(void)wc->drain();
	{
		std::lock_guard<std::mutex> g(g_budget_mu);
		g_budget += wc->lru.size();  // ~AsyncFileWriteChecker, :205-208
	}
	delete wc;
}

void fdb_wc_reset_budget(void) {
	std::lock_guard<std::mutex> g(g_budget_mu);
	g_budget_set = false;
	g_budget = 0;
}

int64_t fdb_wc_budget(void) {
	std::lock_guard<std::mutex> g(g_budget_mu);
	return g_budget;
}

int fdb_wc_set_gpu_threshold(fdb_write_checker* wc, uint64_t pages) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	wc->gpu_threshold = pages;
	return 0;
}

int fdb_wc_write(fdb_write_checker* wc, const void* buf, int64_t length, int64_t offset, uint64_t now_ms,
                 uint32_t* pages_out, uint64_t cap, uint64_t* n_pages) {
	if (!wc || (!buf && length > 0) || length < 0 || offset < 0)
		return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_write: bad arguments", hipSuccess);
	if (int rc = wc->drain()) return rc;
	const Span sp = span_of(offset, length);
	if (int rc = wc->host_crcs(buf, sp)) return rc;
	std::vector<uint32_t> pages;
	wc->apply_write(sp, wc->crcs.data(), now_ms, &pages);
	if (n_pages) *n_pages = pages.size();
	if (pages_out)
		for (uint64_t i = 0; i < pages.size() && i < cap; ++i) pages_out[i] = pages[i];
	return 0;
}

int fdb_wc_write_done(fdb_write_checker* wc, const uint32_t* pages, uint64_t n) {
	if (!wc || (!pages && n)) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_write_done: bad arguments", hipSuccess);
	for (uint64_t i = 0; i < n; ++i) wc->writing.erase(pages[i]);
	return 0;
}

int fdb_wc_read(fdb_write_checker* wc, const void* buf, int64_t length, int64_t offset, uint64_t* failures) {
	if (!wc || (!buf && length > 0) || length < 0 || offset < 0)
		return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_read: bad arguments", hipSuccess);
	if (int rc = wc->drain()) return rc;
	const Span sp = span_of(offset, length);
	if (int rc = wc->host_crcs(buf, sp)) return rc;
	uint64_t f = 0;
	wc->apply_read(sp, wc->crcs.data(), &f);
	if (failures) *failures = f;
	return 0;
}

int fdb_wc_sync(fdb_write_checker* wc, uint64_t now_ms) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	if (int rc = wc->drain()) return rc;
	wc->synced = now_ms;  // :87-92
	return 0;
}

int fdb_wc_truncate(fdb_write_checker* wc, int64_t size) {
	if (!wc || size < 0) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_truncate: bad arguments", hipSuccess);
	if (int rc = wc->drain()) return rc;
	const int max_full_page = (int)(size / kPage);  // :76-84
	const int64_t old = wc->lru.size();
	wc->lru.truncate((uint32_t)max_full_page);
	std::lock_guard<std::mutex> g(g_budget_mu);
	g_budget += old - wc->lru.size();
	return 0;
}

int fdb_wc_write_device(fdb_write_checker* wc, const void* d_buf, int64_t length, int64_t offset, uint64_t now_ms,
                        uint64_t* ticket) {
	if (!wc || (!d_buf && length > 0) || length < 0 || offset < 0)
		return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_write_device: bad arguments", hipSuccess);
	return wc->submit_device(Op::kWrite, d_buf, length, offset, now_ms, ticket);
}

int fdb_wc_read_device(fdb_write_checker* wc, const void* d_buf, int64_t length, int64_t offset, uint64_t* ticket) {
	if (!wc || (!d_buf && length > 0) || length < 0 || offset < 0)
		return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc_read_device: bad arguments", hipSuccess);
	return wc->submit_device(Op::kRead, d_buf, length, offset, 0, ticket);
}

int fdb_wc_poll(fdb_write_checker* wc, uint64_t* applied) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	const int rc = wc->poll();
	if (applied) *applied = wc->applied;
	return rc;
}

int fdb_wc_wait(fdb_write_checker* wc, uint64_t ticket) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	return wc->wait(ticket);
}

int fdb_wc_stats(fdb_write_checker* wc, uint64_t* checked_succeed, uint64_t* checked_fail, uint64_t* history_size,
                 uint64_t* writing) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	if (checked_succeed) *checked_succeed = wc->succeed;
	if (checked_fail) *checked_fail = wc->failed;
	if (history_size) *history_size = (uint64_t)wc->lru.size();
	if (writing) *writing = wc->writing.size();
	return 0;
}

// The batched form of the reference's sweep actor (AsyncFileWriteChecker.h:218-232),
// which re-reads the least recently used page and waits while it is being
// written: the next pages it would visit, in that order, up to the first page
// being written.
int fdb_wc_sweep_pages(fdb_write_checker* wc, uint32_t* pages_out, uint64_t cap, uint64_t* n) {
	if (!wc || !n || (cap && !pages_out)) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null argument", hipSuccess);
	if (int rc = wc->drain()) return rc;
	*n = wc->lru.lru_order(pages_out, cap, [&](uint32_t p) { return wc->writing.count(p) != 0; });
	return 0;
}

int fdb_wc_history(fdb_write_checker* wc, uint32_t page, uint32_t* checksum, uint64_t* timestamp_ms) {
	if (!wc) return fdbcrc::set_error(FDB_CRC32C_EINVAL, "fdb_wc: null checker", hipSuccess);
	if (!wc->lru.exist(page)) return 0;
	const WriteInfo w = wc->lru.find(page);
	if (checksum) *checksum = w.checksum;
	if (timestamp_ms) *timestamp_ms = w.timestamp;
	return 1;
}

}  // extern "C"
