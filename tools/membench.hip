// Access-pattern microbenchmark (design exploration, not product code).
// Measures device read bandwidth for the lane layouts considered for the
// batched CRC32C page kernel: coalesced rows vs per-lane contiguous segments.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef unsigned int u32;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// LANE_BYTES: contiguous bytes per lane per page-group; lanes per page = 4096/LANE_BYTES
template <int LANE_BYTES, int LDS_KB>
__global__ __launch_bounds__(1024) void rd(const u32x4* __restrict__ src, size_t npages, u32* __restrict__ out) {
  extern __shared__ u32 lds[];
  constexpr int LPP = 4096 / LANE_BYTES;           // lanes per page
  constexpr int PPW = 64 / LPP;                    // pages per wave
  constexpr int NCH = LANE_BYTES / 16;             // 16B chunks per lane
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  size_t gw = (size_t)blockIdx.x * wpb + wave;
  size_t nw = (size_t)gridDim.x * wpb;
  if (LDS_KB) { if (threadIdx.x == 0) lds[0] = 0; }
  const int pg = lane / LPP, li = lane % LPP;
  for (size_t g = gw; g * PPW < npages; g += nw) {
    size_t page = g * PPW + pg;
    const u32x4* p = src + page * 256 + li * NCH;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc ^= __builtin_nontemporal_load(p + c);
    u32 x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x12345678u) out[page] = x;   // practically never stores
  }
}

// coalesced: lane reads 16B at lane*16 for each of 4 rows of a page (wave per page)
__global__ __launch_bounds__(1024) void rd_coal(const u32x4* __restrict__ src, size_t npages, u32* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  size_t gw = (size_t)blockIdx.x * wpb + wave;
  size_t nw = (size_t)gridDim.x * wpb;
  for (size_t page = gw; page < npages; page += nw) {
    const u32x4* p = src + page * 256 + lane;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c) acc ^= __builtin_nontemporal_load(p + 64 * c);
    u32 x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x12345678u) out[page] = x;
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  size_t npages = 1 << 20;
  size_t bytes = npages * 4096;
  u32x4* d; u32* o;
  CHECK(hipMalloc(&d, bytes)); CHECK(hipMalloc(&o, npages * 4));
  CHECK(hipMemset(d, 0x5a, bytes));
  int reps = 20;
  auto report = [&](const char* name, int threads, int blocks, float ms) {
    printf("%-28s thr=%4d blk=%5d  %.3f ms  %.1f GB/s\n", name, threads, blocks, ms, bytes / ms / 1e6);
  };
  for (int threads : {256, 512, 1024}) {
    for (int bpc : {1, 2, 4, 8}) {
      int blocks = 256 * bpc;
      if (threads * bpc > 2048) continue;
      report("coalesced", threads, blocks, timeit([&] { rd_coal<<<blocks, threads>>>(d, npages, o); }, reps));
      report("lane64B", threads, blocks, timeit([&] { rd<64, 0><<<blocks, threads>>>(d, npages, o); }, reps));
      report("lane256B", threads, blocks, timeit([&] { rd<256, 0><<<blocks, threads>>>(d, npages, o); }, reps));
      report("lane1KiB", threads, blocks, timeit([&] { rd<1024, 0><<<blocks, threads>>>(d, npages, o); }, reps));
    }
  }
  CHECK(hipFuncSetAttribute((const void*)rd<64, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  CHECK(hipFuncSetAttribute((const void*)rd<256, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  // with a big LDS allocation (1 WG per CU) as the CRC kernel will have
  for (int threads : {512, 1024}) {
    int blocks = 256;
    report("lane64B+128KiB LDS", threads, blocks, timeit([&] { rd<64, 128><<<blocks, threads, 128 * 1024>>>(d, npages, o); }, reps));
    report("lane256B+128KiB LDS", threads, blocks, timeit([&] { rd<256, 128><<<blocks, threads, 128 * 1024>>>(d, npages, o); }, reps));
  }
  CHECK(hipFree(d)); CHECK(hipFree(o));
  return 0;
}
