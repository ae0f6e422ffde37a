// VALU throughput probe (gfx950): issue cost of the instructions the SHA-512
// compression is made of, to price K4's VALU roofline.  Each lane runs 8
// independent chains of one instruction kind (inline asm, so the compiler cannot
// rewrite it); the host times the launch and converts to cycles per
// wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/valu_probe.hip -o tools/_valu_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CH 8

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(uint64_t* out, int iters, uint32_t seed) {
  uint64_t x[CH];
  uint32_t y[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    x[c] = (uint64_t(threadIdx.x) << 32) ^ (seed + c * 0x9E37u);
    y[c] = uint32_t(x[c]) * 3u + c;
  }
  const uint64_t k = 0x428a2f98d728ae22ull ^ seed;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (KIND == 0) {  // v_lshl_add_u64 (64-bit add)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[c]) : "v"(k));
      } else if constexpr (KIND == 1) {  // 64-bit add as v_add_co_u32 + v_addc_co_u32
        uint32_t lo = uint32_t(x[c]), hi = uint32_t(x[c] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                     : "+v"(lo), "+v"(hi) : "v"(uint32_t(k)), "v"(uint32_t(k >> 32)) : "vcc");
        x[c] = (uint64_t(hi) << 32) | lo;
      } else if constexpr (KIND == 2) {  // v_alignbit_b32
        asm volatile("v_alignbit_b32 %0, %0, %1, 14" : "+v"(y[c]) : "v"(y[(c + 1) % CH]));
      } else if constexpr (KIND == 3) {  // v_bitop3_b32
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(y[c]) : "v"(y[(c + 1) % CH]),
                     "v"(y[(c + 2) % CH]));
      } else if constexpr (KIND == 4) {  // v_xor_b32
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(y[c]) : "v"(y[(c + 3) % CH]));
      } else if constexpr (KIND == 5) {  // v_add_u32 (32-bit, for reference)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(y[c]) : "v"(y[(c + 3) % CH]));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c] + y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

extern "C" int valu_probe(int kind, void* out, int blocks, int iters, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint64_t* o = static_cast<uint64_t*>(out);
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
    case 1: hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
    case 2: hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
    case 3: hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
    case 4: hipLaunchKernelGGL(k_probe<4>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
    default: hipLaunchKernelGGL(k_probe<5>, dim3(blocks), dim3(256), 0, s, o, iters, 7u); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
