// HBM stream ceilings on one MI355X for the read/write mixes the step's kernels run:
// read-only, write-only, copy (1 read : 1 write), 1 : 3 (K7 reads 5.5 GB and writes
// 17.3 GB per C4k launch) and 3 : 1 (the keyed K2: 4.8 GB read, 1.4 GB written).
// Each thread moves U 16-byte chunks per array per trip (all loads issued before the
// stores), R source arrays and W destination arrays of n chunks each, grid-stride;
// plain or nontemporal loads / stores; 256-thread workgroups, G per CU.  hipEvent
// timing, best of 10 launches after 3 warmups; one JSON line per configuration.
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

struct Bufs {
  const u32x4* src[3];
  u32x4* dst[3];
  u32x4* sink;
};

template <int R, int W, int U, bool kNtL, bool kNtS>
__global__ __launch_bounds__(256) void k_stream(Bufs b, size_t n) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i0 = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i0 < n; i0 += stride * U) {
    u32x4 v[R > 0 ? R : 1][U];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t i = i0 + size_t(u) * stride;
        v[r][u] = i < n ? (kNtL ? __builtin_nontemporal_load(b.src[r] + i) : b.src[r][i]) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t i = i0 + size_t(u) * stride;
        u32x4 x = u32x4{uint32_t(i), uint32_t(w), 1u, 2u};
#pragma unroll
        for (int r = 0; r < R; ++r) x += v[r][u];
        if (i < n) {
          if (kNtS) __builtin_nontemporal_store(x, b.dst[w] + i);
          else b.dst[w][i] = x;
        }
      }
    if (W == 0)
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[0][u];
  }
  if (W == 0 && (acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) b.sink[0] = acc;  // keeps the loads
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

static Bufs g_b;
static size_t g_n;
static int g_cus;

template <int R, int W, int U, bool kNtL, bool kNtS>
static void run(const char* mix, int per_cu) {
  const unsigned grid = unsigned(g_cus * per_cu);
  const float ms = best_ms([&] { hipLaunchKernelGGL((k_stream<R, W, U, kNtL, kNtS>), dim3(grid), dim3(256), 0, 0, g_b, g_n); });
  CK(hipGetLastError());
  const double bytes = double(g_n) * 16 * (R + W);
  printf("{\"test\": \"%s\", \"unroll\": %d, \"nt_load\": %d, \"nt_store\": %d, \"wg_per_cu\": %d, \"bytes\": %.0f, "
         "\"ms\": %.4f, \"TBps\": %.3f}\n",
         mix, U, int(kNtL), int(kNtS), per_cu, bytes, ms, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

template <int R, int W>
static void sweep(const char* mix) {
  for (int g : {4, 8}) {
    run<R, W, 1, false, false>(mix, g);
    run<R, W, 4, false, false>(mix, g);
    run<R, W, 4, true, false>(mix, g);
    if (W) run<R, W, 4, true, true>(mix, g);
  }
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;  // bytes per array
  g_n = size_t(gib * (1ull << 30)) / 16;
  for (int k = 0; k < 3; ++k) {
    u32x4 *s, *d;
    CK(hipMalloc(&s, g_n * 16));
    CK(hipMalloc(&d, g_n * 16));
    CK(hipMemset(s, 1 + k, g_n * 16));
    CK(hipMemset(d, 0, g_n * 16));
    g_b.src[k] = s;
    g_b.dst[k] = d;
  }
  CK(hipMalloc(&g_b.sink, 16));
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  sweep<1, 0>("read");
  sweep<0, 1>("write");
  sweep<1, 1>("copy");
  sweep<1, 3>("read1_write3");
  sweep<3, 1>("read3_write1");
  for (int k = 0; k < 3; ++k) {
    CK(hipFree(const_cast<u32x4*>(g_b.src[k])));
    CK(hipFree(g_b.dst[k]));
  }
  CK(hipFree(g_b.sink));
  return 0;
}
