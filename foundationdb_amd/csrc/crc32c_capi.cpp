// C ABI for the batched engine (declarations and contracts: include/fdb_crc32c.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#include "../../include/fdb_crc32c.h"
#include "crc32c_device.h"

namespace fdbcrc {
namespace {

constexpr int kMaxDevices = 64;

struct DeviceState {
	DevTables* tables = nullptr;  // device copy
	int num_cus = 0;
	bool ready = false;
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
		DevTables host;
		build_dev_tables(&host);
		DevTables* dt = nullptr;
		e = hipMalloc(reinterpret_cast<void**>(&dt), sizeof(DevTables));
		if (e != hipSuccess) return fail(FDB_CRC32C_ENOMEM, "hipMalloc(tables)", e);
		e = hipMemcpy(dt, &host, sizeof(DevTables), hipMemcpyHostToDevice);
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

int check_launch(const char* what) {
	hipError_t e = hipGetLastError();
	if (e != hipSuccess) return fail(FDB_CRC32C_EHIP, what, e);
	return 0;
}

}  // namespace
}  // namespace fdbcrc

using namespace fdbcrc;

extern "C" {

int crc32c_gpu_init(void) {
	DeviceState* st;
	return device_state(&st);
}

int crc32c_gpu_batch_fixed(const void* d_base, uint64_t stride, uint64_t length, uint64_t count, uint32_t seed,
                           const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || (!d_base && length)) return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_fixed: null pointer");
	DeviceState* st;
	if (int rc = device_state(&st)) return rc;
	hipStream_t s = reinterpret_cast<hipStream_t>(stream);
	const uint8_t* base = static_cast<const uint8_t*>(d_base);
	const uint64_t blocks = length / 4096;
	const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && (stride % 16 == 0) && length % 4096 == 0 &&
	                     (blocks == 1 || blocks == 2);
	if (aligned) {
		launch_pages((int)blocks, base, stride, count, seed, d_seeds, d_out, st->tables, st->num_cus, s);
	} else {
		launch_general(base, stride, length, nullptr, nullptr, count, seed, d_seeds, d_out, st->tables, st->num_cus,
		               s);
	}
	return check_launch("crc32c_gpu_batch_fixed launch");
}

int crc32c_gpu_batch_varlen(const void* d_base, const uint64_t* d_offsets, const uint64_t* d_lengths, uint64_t count,
                            uint32_t seed, const uint32_t* d_seeds, uint32_t* d_out, void* stream) {
	if (count == 0) return 0;
	if (!d_out || !d_offsets || !d_lengths || !d_base)
		return fail(FDB_CRC32C_EINVAL, "crc32c_gpu_batch_varlen: null pointer");
	DeviceState* st;
	if (int rc = device_state(&st)) return rc;
	launch_general(static_cast<const uint8_t*>(d_base), 0, 0, d_offsets, d_lengths, count, seed, d_seeds, d_out,
	               st->tables, st->num_cus, reinterpret_cast<hipStream_t>(stream));
	return check_launch("crc32c_gpu_batch_varlen launch");
}

const char* crc32c_gpu_last_error(void) { return t_err.c_str(); }

const char* crc32c_gpu_version(void) { return "fdb_crc32c 0.1 gfx950"; }

}  // extern "C"
