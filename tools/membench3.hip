// Access-pattern microbenchmark (design exploration, not product code).
// Page-kernel-shaped streaming (1024-thread workgroups, one per CU with the
// 160 KiB LDS image, two 4 KiB pages per unit, the next unit in flight) with
// two load shapes per wave-instruction:
//   coal:  one contiguous KiB (8 whole 128-B lines)
//   half:  16 half-lines of 64 B at a 128-B stride (the partner instruction
//          of the unit reads the other halves) -- the shape a 32-lane page
//          with 128-byte lane spans needs from permlane swaps alone
//   dword: 16 global_load_dword per page, lane l reading bytes 4l + 256k
//          (256 contiguous bytes per instruction)
//   dx2:   8 global_load_dwordx2 per page, lane l reading 8l + 512k
//   u8/u1: coal's shape shifted by 8 / 1 bytes (unaligned dwordx4; the
//          DiskQueue V2 XXH3 region at +8, packet payloads at any offset)
//   dq2:   coal's shape at +8 as two dwordx2 per 16 bytes (the current
//          8-byte-aligned XXH3 row form)
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench3.hip -o tools/membench3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef unsigned int u32;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((address_space(1))) const u32x4 g4;
typedef __attribute__((address_space(1))) const u32x2 g2;
typedef __attribute__((address_space(1))) const u32 g1;

__device__ __forceinline__ u32x4 ld(const unsigned char* p) { return __builtin_nontemporal_load((g4*)(uintptr_t)p); }

// MODE 2 / 3: a page as 16 dwords / 8 dword pairs per lane
template <int MODE>
__global__ __launch_bounds__(1024) void rdw(const unsigned char* __restrict__ src, size_t npages, u32* __restrict__ out) {
  __shared__ u32 lds[160 * 256];
  const u32 lane = threadIdx.x & 63;
  if (threadIdx.x < 64) lds[threadIdx.x * 640] = lane;
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const size_t per = (npages / 2 + nw - 1) / nw * 2;
  size_t p0 = w * per, p1 = p0 + per < npages ? p0 + per : npages;
  if (p0 >= p1) return;
  u32 a[32], b[32];
  auto load = [&](u32 (&u)[32], size_t p) {
    p = p < p1 ? p : p1 - 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned char* pg = src + (p + j) * 4096;
      if (MODE == 2) {
#pragma unroll
        for (int k = 0; k < 16; ++k) u[16 * j + k] = __builtin_nontemporal_load((g1*)(uintptr_t)(pg + 4 * lane + 256 * k));
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const u32x2 v = __builtin_nontemporal_load((g2*)(uintptr_t)(pg + 8 * lane + 512 * k));
          u[16 * j + 2 * k] = v.x;
          u[16 * j + 2 * k + 1] = v.y;
        }
      }
    }
  };
  u32 acc = 0;
  load(a, p0);
  for (size_t p = p0; p < p1; p += 4) {
    load(b, p + 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= a[i];
    __builtin_amdgcn_sched_barrier(0);
    load(a, p + 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= b[i];
    __builtin_amdgcn_sched_barrier(0);
  }
  u32 x = acc ^ lds[(lane * 37) & 1023];
  if (x == 0x12345678u) out[w] = x;
}

typedef __attribute__((ext_vector_type(4), aligned(1))) unsigned int u32x4u;
typedef __attribute__((address_space(1))) const u32x4u g4u;
template <int HALF, int SHIFT = 0>
__global__ __launch_bounds__(1024) void rd(const unsigned char* __restrict__ src, size_t npages, u32* __restrict__ out) {
  __shared__ u32 lds[160 * 256];
  const u32 lane = threadIdx.x & 63;
  if (threadIdx.x < 64) lds[threadIdx.x * 640] = lane;
  // byte offset of load k (0..3) of a page for this lane
  u32 off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (HALF == 1) {  // k = 2A + B: bytes 2048A + 128r + 64B + 16(lane & 3), r = lane >> 2
      off[k] = 2048u * (k >> 1) + 128u * (lane >> 2) + 64u * (k & 1) + 16u * (lane & 3);
    } else {
      off[k] = 1024u * k + 16u * lane;
    }
  }
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const size_t per = (npages / 2 + nw - 1) / nw * 2;
  size_t p0 = w * per, p1 = p0 + per < npages ? p0 + per : npages;
  if (p0 >= p1) return;
  u32x4 a[8], b[8];
  auto load = [&](u32x4 (&u)[8], size_t p) {
    p = p < p1 ? p : p1 - 2;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned char* a = src + (p + j) * 4096 + off[k] + SHIFT;
        if (SHIFT == 0) {
          u[4 * j + k] = ld(a);
        } else if (HALF == 2) {  // two dwordx2 per 16 B (8-byte aligned)
          const u32x2 x = __builtin_nontemporal_load((g2*)(uintptr_t)a), y = __builtin_nontemporal_load((g2*)(uintptr_t)(a + 8));
          u[4 * j + k] = u32x4{x.x, x.y, y.x, y.y};
        } else {
          const u32x4u v = __builtin_nontemporal_load((g4u*)(uintptr_t)a);
          u[4 * j + k] = u32x4{v.x, v.y, v.z, v.w};
        }
      }
  };
  u32x4 acc = {0, 0, 0, 0};
  load(a, p0);
  for (size_t p = p0; p < p1; p += 4) {
    load(b, p + 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= a[i];
    __builtin_amdgcn_sched_barrier(0);
    load(a, p + 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= b[i];
    __builtin_amdgcn_sched_barrier(0);
  }
  u32 x = acc.x ^ acc.y ^ acc.z ^ acc.w ^ lds[(lane * 37) & 1023];
  if (x == 0x12345678u) out[w] = x;
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
  unsigned char* d; u32* o;
  CHECK(hipMalloc(&d, bytes)); CHECK(hipMalloc(&o, 1 << 20));
  CHECK(hipMemset(d, 0x5a, bytes));
  int cus = 256;
  for (int rep = 0; rep < 3; ++rep) {
    float c = timeit([&] { rd<0><<<cus, 1024>>>(d, npages, o); }, 30);
    float h = timeit([&] { rd<1><<<cus, 1024>>>(d, npages, o); }, 30);
    float w1 = timeit([&] { rdw<2><<<cus, 1024>>>(d, npages, o); }, 30);
    float w2 = timeit([&] { rdw<3><<<cus, 1024>>>(d, npages, o); }, 30);
    float u8 = timeit([&] { rd<0, 8><<<cus, 1024>>>(d, npages - 2, o); }, 30);
    float u1 = timeit([&] { rd<0, 1><<<cus, 1024>>>(d, npages - 2, o); }, 30);
    float q2 = timeit([&] { rd<2, 8><<<cus, 1024>>>(d, npages - 2, o); }, 30);
    printf("coal %.1f  half %.1f  dword %.1f  dx2 %.1f  u8 %.1f  u1 %.1f  dq2 %.1f GB/s\n", bytes / c / 1e6,
           bytes / h / 1e6, bytes / w1 / 1e6, bytes / w2 / 1e6, bytes / u8 / 1e6, bytes / u1 / 1e6, bytes / q2 / 1e6);
  }
  CHECK(hipFree(d)); CHECK(hipFree(o));
  return 0;
}
