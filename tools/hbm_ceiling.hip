// HBM stream ceilings on one MI355X for the byte mixes the keyed step's kernels run:
// read-only, write-only (plain and nontemporal 16-B stores, as K7's flush), copy
// (1 read : 1 write) and 1 read : 3 writes (K7 reads 5.5 GB and writes 17.3 GB per
// C4k launch).  Grid-stride 16-B accesses, 256-thread workgroups, hipEvent timing,
// best of 10 launches after 3 warmups.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_ceiling tools/hbm_ceiling.hip && /tmp/hbm_ceiling [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t n, u32x4* __restrict__ sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) acc ^= a[i];
  if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc;  // keeps the loads
}

template <bool kNt>
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ b, size_t n) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const u32x4 v = {uint32_t(i), uint32_t(i >> 32), 1u, 2u};
    if (kNt) __builtin_nontemporal_store(v, b + i);
    else b[i] = v;
  }
}

// W writes of 16 B per 16 B read: dst holds W rows of n chunks
template <int W, bool kNt>
__global__ __launch_bounds__(256) void k_mix(const u32x4* __restrict__ a, size_t n, u32x4* __restrict__ b) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const u32x4 v = a[i];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const u32x4 x = v + u32x4{uint32_t(w), 0u, 0u, 0u};
      if (kNt) __builtin_nontemporal_store(x, b + size_t(w) * n + i);
      else b[size_t(w) * n + i] = x;
    }
  }
}

template <class F>
static float best_ms(F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 10; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;  // bytes read per test (writes: x W)
  const size_t n = size_t(gib * (1ull << 30)) / 16;
  u32x4 *a, *b, *sink;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, 3 * n * 16));
  CK(hipMalloc(&sink, 16));
  CK(hipMemset(a, 1, n * 16));
  CK(hipMemset(b, 0, 3 * n * 16));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = unsigned(cus) * 8;  // 8 workgroups of 256 per CU, grid-stride
  const double GB = 1e9;
  auto rep = [&](const char* name, double bytes, float ms) {
    printf("{\"test\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"TBps\": %.3f}\n", name, bytes, ms, bytes / (ms * 1e-3) / (1e3 * GB));
  };
  const double B = double(n) * 16;
  rep("read", B, best_ms([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, sink); }));
  rep("write_plain", 3 * B, best_ms([&] { hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, b, 3 * n); }));
  rep("write_nt", 3 * B, best_ms([&] { hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, b, 3 * n); }));
  rep("copy_plain", 2 * B, best_ms([&] { hipLaunchKernelGGL((k_mix<1, false>), dim3(grid), dim3(256), 0, 0, a, n, b); }));
  rep("copy_nt", 2 * B, best_ms([&] { hipLaunchKernelGGL((k_mix<1, true>), dim3(grid), dim3(256), 0, 0, a, n, b); }));
  rep("read1_write3_plain", 4 * B, best_ms([&] { hipLaunchKernelGGL((k_mix<3, false>), dim3(grid), dim3(256), 0, 0, a, n, b); }));
  rep("read1_write3_nt", 4 * B, best_ms([&] { hipLaunchKernelGGL((k_mix<3, true>), dim3(grid), dim3(256), 0, 0, a, n, b); }));
  CK(hipGetLastError());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
