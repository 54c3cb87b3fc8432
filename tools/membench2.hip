// Access-order microbenchmark (design exploration): does the ORDER in which
// waves walk 4 KiB pages matter?  contiguous run per wave vs grid-stride.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// mode 0: grid-stride pages; mode 1: contiguous run of pages per wave; mode 2: contiguous run of 8 KiB units
template <int MODE, int UNITPAGES>
__global__ __launch_bounds__(1024) void rd(const u32x4* __restrict__ src, size_t npages, u32* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  u32x4 acc = {0, 0, 0, 0};
  if (MODE == 0) {
    for (size_t pg = wave * UNITPAGES; pg < npages; pg += nw * UNITPAGES) {
#pragma unroll
      for (int j = 0; j < UNITPAGES; ++j) {
        const u32x4* p = src + (pg + j) * 256 + lane;
#pragma unroll
        for (int c = 0; c < 4; ++c) acc ^= __builtin_nontemporal_load(p + 64 * c);
      }
    }
  } else {
    size_t per = (npages + nw - 1) / nw;
    size_t b = wave * per, e = b + per < npages ? b + per : npages;
    for (size_t pg = b; pg < e; pg += UNITPAGES) {
#pragma unroll
      for (int j = 0; j < UNITPAGES; ++j) {
        const u32x4* p = src + (pg + j) * 256 + lane;
#pragma unroll
        for (int c = 0; c < 4; ++c) acc ^= __builtin_nontemporal_load(p + 64 * c);
      }
    }
  }
  u32 x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x12345678u) out[wave] = x;
}

template <typename F> float timeit(F f, int reps) {
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f(); CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a)); for (int i = 0; i < reps; ++i) f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main() {
  size_t npages = 1 << 20, bytes = npages * 4096;
  u32x4* d; u32* o;
  CHECK(hipMalloc(&d, bytes)); CHECK(hipMalloc(&o, 1 << 20));
  CHECK(hipMemset(d, 0x5a, bytes));
  auto rep = [&](const char* n, float ms) { printf("%-34s %.4f ms %.1f GB/s\n", n, ms, bytes / ms / 1e6); };
  for (int blk : {256, 512}) {
    printf("grid %d x 1024\n", blk);
    rep("grid-stride pages", timeit([&] { rd<0, 1><<<blk, 1024>>>(d, npages, o); }, 20));
    rep("grid-stride 2-page units", timeit([&] { rd<0, 2><<<blk, 1024>>>(d, npages, o); }, 20));
    rep("contiguous run, 1 page at a time", timeit([&] { rd<1, 1><<<blk, 1024>>>(d, npages, o); }, 20));
    rep("contiguous run, 2-page units", timeit([&] { rd<1, 2><<<blk, 1024>>>(d, npages, o); }, 20));
  }
  return 0;
}
