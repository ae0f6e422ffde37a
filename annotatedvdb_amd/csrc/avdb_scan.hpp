// Device-wide exclusive prefix sum (u64 out, u64 or u16 in; in place allowed) for
// the per-line / per-record size arrays of K0 (record and heap offsets), K5 (COPY
// and .mapping offsets), K7's two-call form (key and path offsets) and K9 (a
// rank's line bytes).  Reduce-then-scan over 1,024-element tiles in three short
// launches — tile sums, one workgroup scanning the tile sums, then each tile
// scanned again with its base — no look-back across workgroups and no library.
// Two arrays of the same length (K0's record and heap counts, K5's COPY and
// .mapping sizes) are scanned by the same three launches (exclusive_u64_pair).
// Traffic is 2 reads + 1 write of each array (8.4 M u64: ~0.2 GB).
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
constexpr uint32_t kSumPer = 8;                  // tile sums per thread of that workgroup

inline size_t tiles(size_t n) { return (n + kTile - 1) / kTile; }
// workspace bytes for n elements of na arrays: one u64 per tile and array (+ slack)
inline size_t workspace_bytes(size_t n, int na = 1) { return 8 * size_t(na) * tiles(n) + 256; }

template <class T, int NA>
struct Arrays {
  const T* in[NA];
  uint64_t* out[NA];  // (may alias in)
};

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t(uint32_t(__shfl_up(uint32_t(v >> 32), d, kWave))) << 32) | uint32_t(__shfl_up(uint32_t(v), d, kWave));
}

// exclusive scan of one u64 per thread over the NT threads of the workgroup;
// *total = sum.  s_w holds NT / kWave words.
template <uint32_t NT>
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
  for (uint32_t w = 0; w < NT / kWave; ++w) {
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

// sums[NA * tile + a] = sum of array a over the tile
template <class T, int NA>
__global__ __launch_bounds__(kThreads) void k_tile_sums(Arrays<T, NA> A, size_t n, uint64_t* __restrict__ sums) {
  __shared__ uint64_t s_w[kThreads / kWave];
  const size_t i0 = size_t(blockIdx.x) * kTile + size_t(threadIdx.x) * kPer;
  uint64_t v[NA][kPer];
#pragma unroll
  for (int a = 0; a < NA; ++a) load_run(A.in[a], n, i0, v[a]);
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) s += v[a][k];
    uint64_t tot;
    (void)block_excl<kThreads>(s, s_w, &tot);
    if (threadIdx.x == 0) sums[NA * size_t(blockIdx.x) + a] = tot;
  }
}

// exclusive scan of each array's tile sums in place (one workgroup; kSumPer
// consecutive tiles per thread, so up to 8,192 tiles = 8.4 M elements in one
// trip); a template, so every translation unit including this header may define it
template <int NA>
__global__ __launch_bounds__(kSumThreads) void k_scan_sums(uint64_t* __restrict__ sums, size_t nt) {
  __shared__ uint64_t s_w[kSumThreads / kWave];
  uint64_t run[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) run[a] = 0;
  for (size_t c0 = 0; c0 < nt; c0 += size_t(kSumThreads) * kSumPer) {
    const size_t t0 = c0 + size_t(threadIdx.x) * kSumPer;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      uint64_t v[kSumPer], s = 0;
#pragma unroll
      for (uint32_t k = 0; k < kSumPer; ++k) {
        v[k] = t0 + k < nt ? sums[NA * (t0 + k) + a] : 0ull;
        s += v[k];
      }
      uint64_t tot;
      uint64_t x = run[a] + block_excl<kSumThreads>(s, s_w, &tot);
#pragma unroll
      for (uint32_t k = 0; k < kSumPer; ++k) {
        if (t0 + k < nt) sums[NA * (t0 + k) + a] = x;
        x += v[k];
      }
      run[a] += tot;
    }
  }
}

template <class T, int NA>
__global__ __launch_bounds__(kThreads) void k_tile_scan(Arrays<T, NA> A, size_t n, const uint64_t* __restrict__ base) {
  __shared__ uint64_t s_w[kThreads / kWave];
  const size_t i0 = size_t(blockIdx.x) * kTile + size_t(threadIdx.x) * kPer;
  uint64_t v[NA][kPer];
#pragma unroll
  for (int a = 0; a < NA; ++a) load_run(A.in[a], n, i0, v[a]);
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) s += v[a][k];
    uint64_t tot;
    uint64_t run = base[NA * size_t(blockIdx.x) + a] + block_excl<kThreads>(s, s_w, &tot);
    uint64_t* out = A.out[a];
    if (i0 + kPer <= n) {
#pragma unroll
      for (uint32_t k = 0; k < kPer; ++k) {
        out[i0 + k] = run;
        run += v[a][k];
      }
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kPer; ++k) {
        if (i0 + k < n) out[i0 + k] = run;
        run += v[a][k];
      }
    }
  }
}

template <class T, int NA>
inline int exclusive_n(const Arrays<T, NA>& A, size_t n, void* workspace, size_t workspace_size, hipStream_t s) {
  static_assert(sizeof(T) <= 8, "u16 .. u64 inputs");
  if (n == 0) return AVDB_OK;
  if (!workspace || workspace_size < workspace_bytes(n, NA) || reinterpret_cast<uintptr_t>(workspace) % 8) {
    avdb_set_error("exclusive scan: 8-byte aligned workspace of %zu bytes required", workspace_bytes(n, NA));
    return AVDB_ERANGE;
  }
  const size_t nt = tiles(n);
  auto* sums = static_cast<uint64_t*>(workspace);
  hipLaunchKernelGGL((k_tile_sums<T, NA>), dim3(unsigned(nt)), dim3(kThreads), 0, s, A, n, sums);
  AVDB_LAUNCH_CHECK("scan::k_tile_sums");
  hipLaunchKernelGGL(k_scan_sums<NA>, dim3(1), dim3(kSumThreads), 0, s, sums, nt);
  AVDB_LAUNCH_CHECK("scan::k_scan_sums");
  hipLaunchKernelGGL((k_tile_scan<T, NA>), dim3(unsigned(nt)), dim3(kThreads), 0, s, A, n, sums);
  AVDB_LAUNCH_CHECK("scan::k_tile_scan");
  return AVDB_OK;
}

// out[i] = in[0] + ... + in[i-1] for i < n (in may alias out).  workspace:
// workspace_bytes(n), 8-byte aligned.
template <class T>
inline int exclusive_u64(const T* in, void* out_u64, size_t n, void* workspace, size_t workspace_size,
                         hipStream_t s) {
  Arrays<T, 1> A{{in}, {static_cast<uint64_t*>(out_u64)}};
  return exclusive_n(A, n, workspace, workspace_size, s);
}

// two arrays of n elements in the same three launches.  workspace:
// workspace_bytes(n, 2), 8-byte aligned.
template <class T>
inline int exclusive_u64_pair(const T* in0, void* out0, const T* in1, void* out1, size_t n, void* workspace,
                              size_t workspace_size, hipStream_t s) {
  Arrays<T, 2> A{{in0, in1}, {static_cast<uint64_t*>(out0), static_cast<uint64_t*>(out1)}};
  return exclusive_n(A, n, workspace, workspace_size, s);
}

}  // namespace scan
}  // namespace avdb
