// Device-wide exclusive prefix sum (u64 out, u64 or u16 in; in place allowed) for
// the per-line / per-record size arrays of K0 (record and heap offsets), K5 (COPY
// and .mapping offsets), K7's two-call form (key and path offsets) and K9 (a
// rank's line bytes).  Reduce-then-scan over 1,024-element tiles in three short
// launches — tile sums, one workgroup scanning the tile sums, then each tile
// scanned again with its base — no look-back across workgroups and no library.
// Traffic is 2 reads + 1 write of the array (8.4 M u64: ~0.2 GB).
#pragma once

#include "avdb_internal.hpp"

namespace avdb {
namespace scan {

constexpr uint32_t kThreads = 256;
// elements per thread (contiguous): 4 u64 are two 16-byte loads per lane, so a
// wave's load instruction covers 2 KB of whole 64-byte halves of lines (16 per
// thread measured 61 us per 8.4 M-element pass: each instruction touched 64 lines)
constexpr uint32_t kPer = 4;
constexpr uint32_t kTile = kThreads * kPer;      // 1,024 elements per workgroup
constexpr uint32_t kSumThreads = 1024;           // the tile-sum scan's one workgroup

inline size_t tiles(size_t n) { return (n + kTile - 1) / kTile; }
// workspace bytes for n elements: one u64 per tile (+ alignment slack)
inline size_t workspace_bytes(size_t n) { return 8 * tiles(n) + 256; }

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t(uint32_t(__shfl_up(uint32_t(v >> 32), d, kWave))) << 32) | uint32_t(__shfl_up(uint32_t(v), d, kWave));
}

// exclusive block scan of one u64 per thread over kThreads threads; *total = sum
__device__ __forceinline__ uint64_t block_excl(uint64_t v, uint64_t* s_w, uint64_t* total) {
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t u = shfl_up64(x, d);
    if (lane >= uint32_t(d)) x += u;
  }
  if (lane == kWave - 1) s_w[wv] = x;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kThreads / kWave; ++w) {
    const uint64_t t = s_w[w];
    if (w < wv) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

template <class T>
__device__ __forceinline__ void load_run(const T* in, size_t n, size_t i0, uint64_t (&v)[kPer]) {
  if (i0 + kPer <= n) {  // (the unguarded loads vectorise)
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) v[k] = uint64_t(in[i0 + k]);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) v[k] = i0 + k < n ? uint64_t(in[i0 + k]) : 0ull;
  }
}

template <class T>
__global__ __launch_bounds__(kThreads) void k_tile_sums(const T* __restrict__ in, size_t n, uint64_t* __restrict__ sums) {
  __shared__ uint64_t s_w[kThreads / kWave];
  uint64_t v[kPer];
  load_run(in, n, size_t(blockIdx.x) * kTile + size_t(threadIdx.x) * kPer, v);
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) s += v[k];
  uint64_t tot;
  (void)block_excl(s, s_w, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of the tile sums in place (one workgroup, sequential chunks);
// a template so that every translation unit including this header may define it
template <int = 0>
__global__ __launch_bounds__(kSumThreads) void k_scan_sums(uint64_t* __restrict__ sums, size_t nt) {
  __shared__ uint64_t s_w[kSumThreads / kWave];
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  uint64_t run = 0;
  for (size_t c0 = 0; c0 < nt; c0 += kSumThreads) {
    const size_t i = c0 + threadIdx.x;
    const uint64_t v = i < nt ? sums[i] : 0ull;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint64_t u = shfl_up64(x, d);
      if (lane >= uint32_t(d)) x += u;
    }
    if (lane == kWave - 1) s_w[wv] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
    for (uint32_t w = 0; w < kSumThreads / kWave; ++w) {
      if (w < wv) base += s_w[w];
      tot += s_w[w];
    }
    if (i < nt) sums[i] = run + base + x - v;
    run += tot;
    __syncthreads();
  }
}

template <class T>
__global__ __launch_bounds__(kThreads) void k_tile_scan(const T* in, size_t n,
                                                         const uint64_t* __restrict__ base,
                                                         uint64_t* out) {  // (in may alias out)
  __shared__ uint64_t s_w[kThreads / kWave];
  const size_t i0 = size_t(blockIdx.x) * kTile + size_t(threadIdx.x) * kPer;
  uint64_t v[kPer];
  load_run(in, n, i0, v);
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) s += v[k];
  uint64_t tot;
  uint64_t run = base[blockIdx.x] + block_excl(s, s_w, &tot);
  if (i0 + kPer <= n) {
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      out[i0 + k] = run;
      run += v[k];
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      if (i0 + k < n) out[i0 + k] = run;
      run += v[k];
    }
  }
}

// out[i] = in[0] + ... + in[i-1] for i < n (in may alias out).  workspace:
// workspace_bytes(n), 8-byte aligned.
template <class T>
inline int exclusive_u64(const T* in, void* out_u64, size_t n, void* workspace, size_t workspace_size,
                         hipStream_t s) {
  static_assert(sizeof(T) <= 8, "u16 .. u64 inputs");
  auto* out = static_cast<uint64_t*>(out_u64);
  if (n == 0) return AVDB_OK;
  if (!workspace || workspace_size < workspace_bytes(n) || reinterpret_cast<uintptr_t>(workspace) % 8) {
    avdb_set_error("exclusive scan: 8-byte aligned workspace of %zu bytes required", workspace_bytes(n));
    return AVDB_ERANGE;
  }
  const size_t nt = tiles(n);
  auto* sums = static_cast<uint64_t*>(workspace);
  hipLaunchKernelGGL(k_tile_sums<T>, dim3(unsigned(nt)), dim3(kThreads), 0, s, in, n, sums);
  AVDB_LAUNCH_CHECK("scan::k_tile_sums");
  hipLaunchKernelGGL(k_scan_sums<>, dim3(1), dim3(kSumThreads), 0, s, sums, nt);
  AVDB_LAUNCH_CHECK("scan::k_scan_sums");
  hipLaunchKernelGGL(k_tile_scan<T>, dim3(unsigned(nt)), dim3(kThreads), 0, s, in, n, sums, out);
  AVDB_LAUNCH_CHECK("scan::k_tile_scan");
  return AVDB_OK;
}

}  // namespace scan
}  // namespace avdb
