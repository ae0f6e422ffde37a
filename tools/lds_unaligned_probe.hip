// Probe: do unaligned 8-byte LDS stores / loads work on gfx950 (byte-exact), and
// what do they cost against aligned ones?  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

struct __attribute__((packed)) U64u { uint64_t v; };
typedef __attribute__((address_space(3))) U64u* lds_u64u;
typedef __attribute__((address_space(3))) uint8_t* lds_b;

__global__ void k_pattern(uint8_t* out) {
  __shared__ uint64_t img[64 * 16 / 8 + 2];
  uint8_t* b = reinterpret_cast<uint8_t*>(img);
  for (int i = threadIdx.x; i < 64 * 16 + 16; i += 64) b[i] = 0xEE;
  __syncthreads();
  // lane l writes 8 bytes (l, l+1, ..., l+7) at byte 16*l + (l % 8)
  const uint32_t l = threadIdx.x;
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) v |= uint64_t(uint8_t(l + k)) << (8 * k);
  ((lds_u64u)((lds_b)(b) + 16 * l + (l % 8)))->v = v;
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 16; i += 64) out[i] = b[i];
  // and an unaligned load back
  const uint64_t r = ((lds_u64u)((lds_b)(b) + 16 * l + (l % 8)))->v;
  reinterpret_cast<uint64_t*>(out + 64 * 16)[l] = r;
}

template <bool UNAL>
__global__ void k_bw(uint64_t* sink, int iters) {
  __shared__ uint64_t img[4096 / 8 + 2];
  uint8_t* b = reinterpret_cast<uint8_t*>(img);
  const uint32_t l = threadIdx.x;
  uint32_t p = (UNAL ? 3u : 0u) + 8u * (l & 63) + 512u * (l >> 6);
  uint64_t acc = l;
  for (int it = 0; it < iters; ++it) {
    ((lds_u64u)((lds_b)(b) + (p & 4095)))->v = acc;
    p += UNAL ? 13 : 8 * 64;
    acc += 0x9E3779B97F4A7C15ull;
  }
  __syncthreads();
  sink[blockIdx.x * blockDim.x + l] = img[l % 512];
}

int main() {
  uint8_t* d;
  hipMalloc(&d, 64 * 16 + 64 * 8);
  hipLaunchKernelGGL(k_pattern, dim3(1), dim3(64), 0, 0, d);
  std::vector<uint8_t> h(64 * 16 + 64 * 8);
  hipMemcpy(h.data(), d, h.size(), hipMemcpyDeviceToHost);
  int bad = 0;
  for (uint32_t l = 0; l < 64; ++l) {
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t s = l % 8;
      const uint8_t want = (i >= s && i < s + 8) ? uint8_t(l + i - s) : 0xEE;
      if (h[16 * l + i] != want) ++bad;
    }
    uint64_t r;
    std::memcpy(&r, &h[64 * 16 + 8 * l], 8);
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v |= uint64_t(uint8_t(l + k)) << (8 * k);
    if (r != v) ++bad;
  }
  printf("unaligned LDS b64 store/load: %s (%d bad bytes)\n", bad ? "WRONG" : "exact", bad);
  uint64_t* s;
  hipMalloc(&s, 8 * 256 * 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int u = 0; u < 2; ++u) {
      hipEventRecord(e0);
      if (u) hipLaunchKernelGGL(k_bw<true>, dim3(4096), dim3(256), 0, 0, s, 4096);
      else hipLaunchKernelGGL(k_bw<false>, dim3(4096), dim3(256), 0, 0, s, 4096);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s b64 LDS stores: %.3f ms (%.1f G stores/s)\n", u ? "unaligned" : "aligned", ms,
             4096.0 * 256 * 4096 / ms / 1e6);
    }
  }
  return bad ? 1 : 0;
}
