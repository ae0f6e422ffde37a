// Chained look-back probe (gfx950): which cross-workgroup publish / poll forms
// make a decoupled look-back complete, and how fast.  Each workgroup takes a
// ticket, "works" for a while, publishes its aggregate, looks back over the
// tickets before it (64 per wave step, as K0's avdb_vcf_tokenize does), checks
// its exclusive prefix (= ticket * 3) and publishes the inclusive one.
//   hipcc --offload-arch=gfx950 -O3 -o handoff_probe tools/handoff_probe.hip
//   ./handoff_probe [tickets] [grid]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62;
constexpr uint32_t kLimit = 1u << 16;

template <int MODE>
__device__ __forceinline__ uint64_t rd(uint64_t* p) {
  if constexpr (MODE == 0) {  // CAS 0 -> 0, agent
    uint64_t e = 0;
    __hip_atomic_compare_exchange_strong(p, &e, 0ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return e;
  } else if constexpr (MODE == 1) {  // relaxed agent load (sc1)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == 2) {  // acquire agent load
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  } else {  // relaxed system load
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
template <int MODE>
__device__ __forceinline__ void wr(uint64_t* p, uint64_t v) {
  if constexpr (MODE == 0) {
    (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == 1) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == 2) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ uint64_t wsum(uint64_t v) {
  for (int d = 32; d > 0; d >>= 1)
    v += (uint64_t(uint32_t(__shfl_xor(uint32_t(v >> 32), d, 64))) << 32) | uint32_t(__shfl_xor(uint32_t(v), d, 64));
  return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_chain(unsigned* ticket, uint64_t* st, uint64_t* pre, uint32_t n,
                                              unsigned long long* err, unsigned* seen, uint32_t work) {
  __shared__ uint32_t s_t;
  for (;;) {
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t c = s_t;
    __syncthreads();
    if (c >= n) return;
    if (threadIdx.x == 0) atomicAdd(seen + c, 1u);
    // some work: a dependent ALU chain whose length varies by ticket
    uint32_t x = c;
    for (uint32_t k = 0; k < work + (c * 2654435761u >> 24); ++k) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) err[2] = x;  // keep the chain
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint32_t lane = threadIdx.x;
      uint64_t s = 0;
      if (c > 0) {
        if (lane == 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          wr<MODE>(st + c, kAgg | 3u);
        }
        int64_t base = int64_t(c) - 1;
        uint32_t spins = 0;
        while (true) {
          const int64_t j = base - int64_t(lane);
          uint64_t v = kInc;
          bool ready = true;
          if (j >= 0) {
            v = rd<MODE>(st + j);
            ready = (v >> 62) != 0;
          }
          while (!__all(ready)) {
            __builtin_amdgcn_s_sleep(2);
            if (!ready) {
              v = rd<MODE>(st + j);
              ready = (v >> 62) != 0;
            }
            if (++spins > kLimit) {
              if (lane == 0) atomicAdd(err, 1ull);
              if (!ready) v = kInc;
              ready = true;
            }
          }
          const uint64_t f = v >> 62;
          const uint64_t pm = __ballot(f == 2);
          const uint32_t l = pm ? uint32_t(__ffsll((unsigned long long)pm)) - 1 : 64u;
          uint64_t a = 0;
          if (lane < l) a = v & 0xFFFFFull;
          else if (lane == l && j >= 0) a = rd<MODE>(pre + j);
          s += wsum(a);
          if (pm) break;
          base -= 64;
        }
      }
      if (lane == 0) {
        if (s != uint64_t(c) * 3) atomicAdd(err + 1, 1ull);
        wr<MODE>(pre + c, s + 3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wr<MODE>(st + c, kInc);
      }
    }
    __syncthreads();
  }
}

template <int MODE>
static void run(uint32_t n, uint32_t grid, uint32_t work) {
  unsigned* ticket;
  uint64_t *st, *pre;
  unsigned long long* err;
  unsigned* seen;
  hipMalloc(&ticket, 256);
  hipMalloc(&st, 8ull * n);
  hipMalloc(&pre, 8ull * n);
  hipMalloc(&err, 64);
  hipMalloc(&seen, 4ull * n);
  float best = 1e30f;
  unsigned long long e[3] = {0, 0, 0};
  unsigned dup = 0, miss = 0;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(ticket, 0, 256);
    hipMemset(st, 0, 8ull * n);
    hipMemset(err, 0, 64);
    hipMemset(seen, 0, 4ull * n);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_chain<MODE>, dim3(grid), dim3(256), 0, 0, ticket, st, pre, n, err, seen, work);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
    unsigned long long h[3];
    hipMemcpy(h, err, 24, hipMemcpyDeviceToHost);
    unsigned* sv = (unsigned*)malloc(4ull * n);
    hipMemcpy(sv, seen, 4ull * n, hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < n; ++i) {
      dup += sv[i] > 1;
      miss += sv[i] == 0;
    }
    free(sv);
    e[0] += h[0];
    e[1] += h[1];
  }
  printf("{\"mode\": %d, \"tickets\": %u, \"grid\": %u, \"work\": %u, \"best_ms\": %.4f, \"gave_up\": %llu, "
         "\"wrong_prefix\": %llu, \"dup_tickets\": %u, \"missed\": %u}\n",
         MODE, n, grid, work, best, e[0], e[1], dup, miss);
  fflush(stdout);
  hipFree(ticket);
  hipFree(st);
  hipFree(pre);
  hipFree(err);
  hipFree(seen);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
  const uint32_t grid = argc > 2 ? atoi(argv[2]) : 1024;
  const uint32_t work = argc > 3 ? atoi(argv[3]) : 2000;
  run<1>(n, grid, work);
  run<2>(n, grid, work);
  run<0>(n, grid, work);
  run<3>(n, grid, work);
  run<1>(64, 64, work);
  run<0>(64, 64, work);
  return 0;
}
