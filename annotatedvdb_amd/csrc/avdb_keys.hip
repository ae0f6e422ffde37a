// K5a avdb_display_attributes (display-attribute JSON of a record batch) and K7
// avdb_primary_keys (primary keys + ltree bin paths of a record batch) (gfx950).
#include "avdb_fmt.hpp"

#include "avdb_scan.hpp"
#include <string.h>

namespace avdb {

// ---------------------------------------------------------------------------
// K5a: display attributes of a record batch (allele heap); one lane per record
// ---------------------------------------------------------------------------
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_display(const uint8_t* __restrict__ chrom,
                                                    const uint32_t* __restrict__ pos,
                                                    const uint32_t* __restrict__ end,
                                                    const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ rl,
                                                    const uint32_t* __restrict__ al,
                                                    const uint8_t* __restrict__ heap, size_t heap_bytes,
                                                    size_t n, uint64_t* __restrict__ out_off,
                                                    uint8_t* __restrict__ out, uint8_t* __restrict__ state) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const uint64_t o = off[i];
    const uint32_t r = rl[i], a = al[i];
    if constexpr (WRITE) {
      if (state[i]) continue;
      Out<true> w(out, out_off[i]);
      w = display_json<true>(w, chrom[i], pos[i], end[i], (glb_cp)(heap + o), r, (glb_cp)(heap + o + r), a);
      w.finish();
    } else {
      uint8_t st = o + r + a > heap_bytes ? 2 : 0;
      for (uint32_t k = 0; k < r + a && !st; ++k)
        if (heap[o + k] & 0x80) st = 1;  // non-ASCII alleles: outside the contract
      state[i] = st;
      uint64_t len = 0;
      if (!st) {
        len = display_json<true>(Out<false>(nullptr, 0), chrom[i], pos[i], end[i], (glb_cp)(heap + o), r,
                                 (glb_cp)(heap + o + r), a).size();
      }
      out_off[i] = len;
    }
  }
}


// ---------------------------------------------------------------------------
// K7: primary keys (+ ltree bin paths) of a record batch as text.
//   key  = label ':' pos ':' ref ':' alt [':rs' id]     (primary_key_generator.py:106-122)
//          label ':' pos ':' <32 digest chars> [':rs' id]  (ref_len + alt_len > max_seq_len)
//   path = generate_bin_index_references.py's ltree label of the record's bin
// The batch is cut into scan groups of 64 or 256 records.  Each group's (keys,
// paths) byte total comes from the keyed K2 (avdb_record_prep_keyed) or from
// k_key_group_totals; k_key_group_scan scans them per block of 4,096 groups; the
// write pass (k_record_keys_v2) recomputes each record's sizes from the SoA it
// reads anyway, scans them over the wave, writes the u64 offsets itself and
// renders the text.  A device-wide decoupled look-back over 64-record tiles was
// built first: the agent-scope status loads of each look-back window cost more
// than the tile (168 ms for C4k's 1.25e8 records), so the scan runs over group
// totals instead.
// ---------------------------------------------------------------------------
struct KeyArgs {
  const uint8_t* chrom;
  const uint32_t* pos;
  const uint64_t* off;
  const uint32_t* rl;
  const uint32_t* al;
  const uint8_t* heap;
  const uint64_t* ext;
  const uint32_t* code;   // nullable: no paths
  const char* digest;     // nullable: long records get state NEED_DIGEST (or DIGEST_PENDING)
  size_t heap_bytes, n, key_cap, path_cap;
  uint32_t max_seq_len;
  int32_t n_chrom;
  uint32_t defer;         // AVDB_KEYS_DIGEST_DEFERRED: long keys laid out, their 32 chars left for the fill pass
  uint64_t* key_off;
  uint64_t* path_off;
  uint8_t* key_out;
  uint8_t* path_out;
  uint8_t* state;
  // per group the (keys, paths) offset of its first record =
  // blk_pre[2*(g / kGroupsPerBlock) + {0,1}] + grp_pre[g].{x,y}
  const uint2* grp_pre;
  const uint64_t* blk_pre;
  uint32_t group_log2;  // records per scan group = 64 << group_log2 (tiles per group = 1 << group_log2)
  uint32_t blk_raw;     // blk_pre holds each block's totals, not their exclusive scan
  uint32_t off32;       // AVDB_KEYS_OFF32: key_off / path_off in the narrow layout (off32_store)
};

// AVDB_KEYS_OFF32 (avdb.h): an offset array of n + 1 entries as u32 low words
// (offset mod 2^32), then, from the next 8-byte boundary, a u64 base for every
// kOff32Span records (the full offset of record k * kOff32Span): 4 bytes per record
// written instead of 8.  Full offset of i = base[i / kOff32Span] +
// (uint32_t)(low[i] - (uint32_t)base[i / kOff32Span]) — a span's text is < 4 GB.
constexpr uint32_t kOff32Log2 = 12, kOff32Span = 1u << kOff32Log2;
__host__ __device__ inline size_t off32_low_bytes(size_t n) { return (4 * (n + 1) + 7) & ~size_t(7); }
__host__ __device__ inline size_t off32_bytes(size_t n) { return off32_low_bytes(n) + 8 * ((n >> kOff32Log2) + 1); }
template <bool NARROW>
__device__ __forceinline__ void off_store(uint64_t* off, size_t n, size_t i, uint64_t v) {
  if constexpr (!NARROW) {
    off[i] = v;
    return;
  }
  reinterpret_cast<uint32_t*>(off)[i] = uint32_t(v);
  if (!(i & (kOff32Span - 1)))
    reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(off) + off32_low_bytes(n))[i >> kOff32Log2] = v;
}

#ifndef AVDB_K7_GRID
#define AVDB_K7_GRID 16384u  // write-pass waves / 4 (C4k K7 5.14 -> 5.00 ms against 4,096; with one-wave workgroups the grid is 4x this)
#endif
// (A periodic-span flush for tiles whose 64 records share one bin — the path
// rendered once, each chunk read from it at its phase — measured no faster:
// 10.21 vs 10.19 ms on C4k keys + paths; not kept.)
constexpr uint32_t kKeyWave = 2560;
constexpr uint32_t kPathWave = 5632;

constexpr uint32_t kWavesPerBlock = kBlock / kWave;

// the wave's LDS writes (lanes OR into words their neighbours share) are complete
// and visible to all its lanes before it reads them back: DS instructions of one
// wave execute in order; the fences keep the compiler from moving LDS accesses
// across this point
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Records per scan group: 256 (4 tiles of 64, one wave renders them in turn)
// for large batches; 64 (one tile) below kSmallGroupN records, where a wave per
// tile gives the launch 4x the waves (C1, 1.1 M records: one generation of waves).
constexpr uint32_t kGroupLog2 = 2;
#ifndef AVDB_K7_SMALL_GROUP_N
#define AVDB_K7_SMALL_GROUP_N (size_t(4) << 20)
#endif
constexpr size_t kSmallGroupN = AVDB_K7_SMALL_GROUP_N;
constexpr uint32_t kGroupsPerBlock = 4096;    // groups per block of the local scan
constexpr uint32_t kScanThreads = 1024;       // 4 groups per thread
// up to ctx->k7_raw_blocks (256) blocks of groups, the write pass sums the block
// totals before its group itself (<= 4 loads per lane at a group's start) instead
// of a separate one-workgroup scan launch

// the sizes the write pass gives record j (SoA-decidable key state only)
__device__ __forceinline__ void record_sizes(const KeyArgs& A, uint32_t c, uint32_t p, uint32_t r, uint32_t a,
                                             uint64_t e, uint32_t cd, uint32_t* ks, uint32_t* ps) {
  key_path_sizes(c, p, r, a, e, cd, A.max_seq_len, uint32_t(A.n_chrom), A.digest != nullptr || A.defer,
                 A.code != nullptr, ks, ps);
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1)
    v += (uint64_t(uint32_t(__shfl_xor(uint32_t(v >> 32), d, kWave))) << 32) | uint32_t(__shfl_xor(uint32_t(v), d, kWave));
  return v;
}

// the (keys, paths) bytes of group g (records (g << group_log2 + k) * 64 + lane),
// summed over the wave
__device__ __forceinline__ uint2 group_total(const KeyArgs& A, size_t g, uint32_t lane) {
  const uint32_t tpg = 1u << A.group_log2;
  uint32_t K = 0, P = 0;
#pragma unroll 4
  for (uint32_t k = 0; k < tpg; ++k) {
    const size_t j = ((g << A.group_log2) + k) * kWave + lane;
    if (j < A.n) {
      uint32_t ks, ps;
      record_sizes(A, A.chrom[j], A.pos[j], A.rl[j], A.al[j], A.ext ? A.ext[j] : 0ull,
                   A.code ? A.code[j] : AVDB_BIN_NONE, &ks, &ps);
      K += ks;
      P += ps;
    }
  }
  return make_uint2(wave_sum32(K), wave_sum32(P));
}

// group totals: one wave per group of 64 << group_log2 records
__global__ __launch_bounds__(kBlock) void k_key_group_totals(KeyArgs A, uint2* __restrict__ tot, size_t n_groups,
                                                              size_t g_begin) {
  const uint32_t lane = __lane_id();
  const size_t w0 = g_begin + (size_t(blockIdx.x) * blockDim.x + threadIdx.x) / kWave;
  const size_t nw = size_t(gridDim.x) * blockDim.x / kWave;
  for (size_t g = w0; g < n_groups; g += nw) {
    const uint2 t = group_total(A, g, lane);
    if (lane == 0) tot[g] = t;
  }
}

// exclusive scan of the group totals inside each block of 4,096 groups (u32: a
// block's text is < 4 GB) and the block totals.  redo_last: the totals came from
// the keyed K2, whose vector form may leave the last group's final < 4 records to
// a scalar tail — the last block's first wave sums that group again here.
__global__ __launch_bounds__(kScanThreads) void k_key_group_scan(const uint2* __restrict__ tot, size_t n_groups,
                                                                  uint2* __restrict__ pre, uint64_t* __restrict__ btot,
                                                                  KeyArgs A, int redo_last) {
  __shared__ uint32_t s_k[kScanThreads / kWave], s_p[kScanThreads / kWave];
  __shared__ uint2 s_last;
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  const bool redo = redo_last && blockIdx.x == gridDim.x - 1;  // (block-uniform)
  if (redo) {
    if (wv == 0) {
      const uint2 t = group_total(A, n_groups - 1, lane);
      if (lane == 0) s_last = t;
    }
    __syncthreads();
  }
  const size_t g0 = size_t(blockIdx.x) * kGroupsPerBlock + 4 * threadIdx.x;
  uint2 v[4];
  uint32_t k = 0, p = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = g0 + q < n_groups ? (redo && g0 + q == n_groups - 1 ? s_last : tot[g0 + q]) : make_uint2(0, 0);
    k += v[q].x;
    p += v[q].y;
  }
  uint32_t xk = k, xp = p;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t uk = __shfl_up(xk, d, kWave), up = __shfl_up(xp, d, kWave);
    if (lane >= uint32_t(d)) {
      xk += uk;
      xp += up;
    }
  }
  if (lane == kWave - 1) {
    s_k[wv] = xk;
    s_p[wv] = xp;
  }
  __syncthreads();
  uint32_t bk = 0, bp = 0, tk = 0, tp = 0;
  for (uint32_t w = 0; w < kScanThreads / kWave; ++w) {
    if (w < wv) {
      bk += s_k[w];
      bp += s_p[w];
    }
    tk += s_k[w];
    tp += s_p[w];
  }
  uint32_t ek = bk + xk - k, ep = bp + xp - p;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (g0 + q < n_groups) pre[g0 + q] = make_uint2(ek, ep);
    ek += v[q].x;
    ep += v[q].y;
  }
  if (threadIdx.x == 0) {
    btot[2 * blockIdx.x] = tk;
    btot[2 * blockIdx.x + 1] = tp;
  }
}

// exclusive scan of the block totals in place (one workgroup, sequential chunks),
// and the grand totals into key_off[n] / path_off[n]
__global__ __launch_bounds__(kScanThreads) void k_key_block_scan(uint64_t* __restrict__ b, size_t nb,
                                                                 uint64_t* __restrict__ key_off,
                                                                 uint64_t* __restrict__ path_off, size_t n,
                                                                 uint32_t off32) {
  __shared__ uint64_t s_k[kScanThreads / kWave], s_p[kScanThreads / kWave];
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  uint64_t run_k = 0, run_p = 0;
  for (size_t c0 = 0; c0 < nb; c0 += kScanThreads) {
    const size_t i = c0 + threadIdx.x;
    const uint64_t k = i < nb ? b[2 * i] : 0ull, p = i < nb ? b[2 * i + 1] : 0ull;
    uint64_t xk = k, xp = p;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint64_t uk = (uint64_t(uint32_t(__shfl_up(uint32_t(xk >> 32), d, kWave))) << 32) |
                          uint32_t(__shfl_up(uint32_t(xk), d, kWave));
      const uint64_t up = (uint64_t(uint32_t(__shfl_up(uint32_t(xp >> 32), d, kWave))) << 32) |
                          uint32_t(__shfl_up(uint32_t(xp), d, kWave));
      if (lane >= uint32_t(d)) {
        xk += uk;
        xp += up;
      }
    }
    if (lane == kWave - 1) {
      s_k[wv] = xk;
      s_p[wv] = xp;
    }
    __syncthreads();
    uint64_t bk = 0, bp = 0, tk = 0, tp = 0;
    for (uint32_t w = 0; w < kScanThreads / kWave; ++w) {
      if (w < wv) {
        bk += s_k[w];
        bp += s_p[w];
      }
      tk += s_k[w];
      tp += s_p[w];
    }
    if (i < nb) {
      b[2 * i] = run_k + bk + xk - k;
      b[2 * i + 1] = run_p + bp + xp - p;
    }
    run_k += tk;
    run_p += tp;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (off32) {
      off_store<true>(key_off, n, n, run_k);
      if (path_off) off_store<true>(path_off, n, n, run_p);
    } else {
      off_store<false>(key_off, n, n, run_k);
      if (path_off) off_store<false>(path_off, n, n, run_p);
    }
  }
}

// the two-call form's size pass (avdb_primary_keys with key_out == NULL): each
// record's key and path size in place in key_off / path_off, scanned afterwards
__global__ __launch_bounds__(kBlock) void k_key_sizes(KeyArgs A) {
  for (size_t j = size_t(blockIdx.x) * blockDim.x + threadIdx.x; j < A.n; j += size_t(gridDim.x) * blockDim.x) {
    uint32_t ks, ps;
    record_sizes(A, A.chrom[j], A.pos[j], A.rl[j], A.al[j], A.ext ? A.ext[j] : 0ull,
                 A.code ? A.code[j] : AVDB_BIN_NONE, &ks, &ps);
    A.key_off[j] = ks;
    if (A.code) A.path_off[j] = ps;
  }
}

// ---------------------------------------------------------------------------
// The write pass (k_record_keys_v2).  Each wave takes 256-record groups
// (grid-stride) and renders their four 64-record tiles in turn; each stream's
// span of a tile (the records' texts are adjacent) is staged in the wave's own
// LDS image when it fits (keys <= 40 B and ltree paths <= 87 B on average; else
// the lanes write global memory directly), then flushed by the same wave with
// coalesced 16-byte stores (a wave of per-lane 8-byte stores would touch 64
// partly written lines per instruction).  The flush zeroes what it read, which
// keeps the images zero between tiles (the sink ORs the words lanes share).
// Round 4 (the round-3 pass issued ~1,280 VALU wave-instructions per tile,
// profiles/pmc_k7.json, most of them in the key stream):
//  * a long record's digest row and a short record's ref are the same kind of
//    piece, a byte range of a register window, so one code path renders both;
//  * ref and alt come from two windows (each aligned at its own range), appended
//    as two ranges with the ':' between — no per-word colon shifting;
//  * a range loop stops when no lane of the wave has bytes left (the longest
//    range of the tile decides, not a fixed seven words), full words take the
//    constant-size append, and the ':' / non-ASCII test runs on the words as
//    they are appended;
//  * "label:pos:" and ":rs<id>" are assembled in two registers each and appended
//    as one or two pieces.
// A key that turns out HOST (':' or a non-ASCII byte) has its span written with
// its bytes: the span is reserved from the SoA either way, and a key's text is
// read only when its state is AVDB_KEY_OK.
// Deferred digests (A.defer, digest == NULL): a long record's key is laid out
// with its 32 digest characters as zero bytes and state AVDB_KEY_DIGEST_PENDING;
// avdb_primary_keys_fill_digests writes them once K4 is done.  K7 then does not
// wait for K4 (SHA-512, VALU-bound), so the two can share the chip.
// ---------------------------------------------------------------------------
constexpr uint32_t kWinWords = 7;  // a range of <= 49 bytes at byte offset <= 7

// a tile's per-record inputs, loaded one tile ahead
struct KeyTileIn {
  uint32_t c, p, r, a, cd;
  uint64_t e, off;
};

// flush_span with 32-bit chunk indices (a tile's span is < 8 KB): one 64-bit
// address add per store instead of 64-bit index arithmetic
__device__ __forceinline__ void flush_span32(lds_u64* img, uint8_t* out, uint64_t g0, uint64_t g1, uint32_t lane) {
  const uint64_t a0 = g0 & ~uint64_t(15);
  const uint64_t f0 = (g0 + 15) & ~uint64_t(15), f1 = g1 & ~uint64_t(15);  // full chunks [f0, f1)
  u32x4* dst = reinterpret_cast<u32x4*>(out + a0);
  if (f1 > f0) {
    const uint32_t q1 = uint32_t(f1 - a0) >> 4;
    for (uint32_t q = (uint32_t(f0 - a0) >> 4) + lane; q < q1; q += kWave) {
      const uint64_t lo = img[2 * q], hi = img[2 * q + 1];
      img[2 * q] = 0;
      img[2 * q + 1] = 0;
      __builtin_nontemporal_store(u32x4{uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32)}, dst + q);
    }
  }
  const bool head = g0 != f0 || f1 < f0;
  const bool tail = (g1 & 15) && f1 >= f0 && (f1 != a0 || !head);
  if ((lane == 0 && head) || (lane == 1 && tail)) {
    const uint64_t a = lane == 0 ? a0 : f1;
    const uint32_t q = uint32_t(a - a0) >> 4;
    const uint64_t v0 = img[2 * q], v1 = img[2 * q + 1];
    img[2 * q] = 0;
    img[2 * q + 1] = 0;
    const uint32_t lo = a < g0 ? uint32_t(g0 - a) : 0u;
    const uint32_t hi = a + 16 > g1 ? uint32_t(g1 - a) : 16u;
    store_part16(out, a, lo, hi, v0, v1);
  }
}

// bit 7 of each byte of x that is ':' (metaseqId.split raises, primary_key_generator.py:106)
// or non-ASCII — exact as an any-test (x's bytes outside the range are zero)
__device__ __forceinline__ uint64_t key_bad(uint64_t x) {
  const uint64_t v = x ^ 0x3A3A3A3A3A3A3A3Aull;
  return (((v - 0x0101010101010101ull) & ~v) | x) & kHiBits;
}

// the window: words [aw, aw + 8 * kWinWords) of the range's aligned start, loaded
// only as far as some byte of the range needs (bytes outside [lo, hi) read as 0)
__device__ __forceinline__ void load_win(uint64_t (&W)[kWinWords], uintptr_t src, uint32_t n, const Heap& h) {
  const uintptr_t aw = src & ~uintptr_t(7);
  const uint32_t nw = (uint32_t(src & 7) + n + 7) >> 3;
  if (aw >= h.lo && aw + 8 * kWinWords <= h.hi) {
    // the whole window inside the allocation: all seven words, no per-word select
    // (words past the range are only ever read under a byte mask)
#pragma unroll
    for (uint32_t k = 0; k < kWinWords; ++k) W[k] = gptr<uint64_t>(aw)[k];
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kWinWords; ++k) W[k] = k < nw ? heap_word(aw + 8 * k, h) : 0ull;
  }
}

// bytes [m, m + n) of window W (m + n <= 56) to the sink, bad |= key_bad of them.
// The loop ends when no lane has bytes left (wave-uniform).
template <class O>
__device__ __forceinline__ void append_win(O& o, const uint64_t (&W)[kWinWords], uint32_t m, uint32_t n,
                                           uint64_t& bad) {
#pragma unroll
  for (uint32_t j = 0; j < kWinWords; ++j) {
    if (!__any(n > 8 * j)) break;
    if (n > 8 * j) {
      uint64_t x = W[j] >> (8 * m);
      if (j + 1 < kWinWords) x |= (W[j + 1] << (63 - 8 * m)) << 1;  // (m == 0: nothing)
      if (n - 8 * j >= 8) {
        bad |= key_bad(x);
        o.append(x, 8);
      } else {
        const uint32_t t = n - 8 * j;
        x &= low_bytes_mask(t);
        bad |= key_bad(x);
        o.append(x, t);
      }
    }
  }
}

// "label:pos:" (contigs 0..24) as up to 14 bytes in two words; returns its length
__device__ __forceinline__ uint32_t key_prefix(uint32_t c, const Dec& d, uint64_t* p0, uint64_t* p1) {
  const uint32_t L = key_label_width(c);
  const uint64_t lab = c < 9 ? uint64_t('1' + c)
                             : (c < 22 ? (uint64_t('0' + (c + 1) / 10u) | (uint64_t('0' + (c + 1) % 10u) << 8))
                                       : (c == 22 ? uint64_t('X') : (c == 23 ? uint64_t('Y') : uint64_t('M'))));
  const uint32_t sh = 8 * (L + 1);  // 16 or 24
  uint64_t a = lab | (0x3Aull << (8 * L)) | (d.lo << sh);
  uint64_t b = (d.lo >> (64 - sh)) | (d.hi << sh);
  const uint32_t cp = L + 1 + d.n;  // the second ':' (<= 13)
  if (cp < 8) a |= 0x3Aull << (8 * cp);
  else b |= 0x3Aull << (8 * (cp - 8));
  *p0 = a;
  *p1 = b;
  return cp + 1;
}

template <class O>
__device__ __forceinline__ void append2(O& o, uint64_t w0, uint64_t w1, uint32_t n) {  // n <= 16
  if (n >= 8) {
    o.append(w0, 8);
    if (n > 8) o.append(w1 & low_bytes_mask(n - 8), n - 8);
  } else {
    o.append(w0 & low_bytes_mask(n), n);
  }
}

// One 64-record tile of the write pass (K7's k_record_keys_v2 and the one-pass
// keyed prep k_keyed_onepass): the records' sizes scanned over the wave from
// run_k / run_p (advanced by the tile's totals), their offsets and states, the
// key and path text rendered into the wave's LDS images and flushed.  cur: record
// t0 + lane (live: t0 + lane < A.n).
template <bool NARROW = false>
__device__ __forceinline__ void key_tile(const KeyArgs& A, const KeyTileIn& cur, size_t t0, uint64_t& run_k,
                                         uint64_t& run_p, lds_u64* kimg, lds_u64* pimg, const Heap& hheap,
                                         uint32_t lane) {
  const size_t i = t0 + lane;
  const bool live = i < A.n;
  const uint32_t n_chrom = uint32_t(A.n_chrom);
  const bool has_digest = A.digest != nullptr || A.defer;  // long keys are laid out
  // the tile's sizes (SoA-decidable, as the group totals: key_path_sizes), from
  // the POS and refSNP digits the key renders anyway, scanned over the wave
  const Dec dp = dec_text(cur.p);
  const bool e32 = cur.e <= 0xFFFFFFFFull;
  const Dec de = dec_text(uint32_t(cur.e));
  uint32_t ksz = 0, psz = 0;
  if (live) {
    const bool lg = uint64_t(cur.r) + cur.a > A.max_seq_len;
    if (cur.c < uint32_t(A.n_chrom) && !(cur.e >> 63) && !(lg && !has_digest))
      ksz = key_label_width(cur.c) + 2u + dp.n + (lg ? uint32_t(AVDB_DIGEST_CHARS) : cur.r + 1u + cur.a) +
            (cur.e ? 3u + (e32 ? de.n : ndigits64(cur.e)) : 0u);
    if (A.code && cur.cd != AVDB_BIN_NONE && cur.c < uint32_t(A.n_chrom)) psz = bin_path_size(cur.c, cur.cd);
  }
  const uint32_t xk = wave_incl_sum(ksz), xp = wave_incl_sum(psz);
  const uint32_t K = __builtin_amdgcn_readlane(xk, kWave - 1), P = __builtin_amdgcn_readlane(xp, kWave - 1);
  const uint64_t gk0 = run_k, gk1 = run_k + K, gp0 = run_p, gp1 = run_p + P;
  const uint64_t ko = gk0 + xk - ksz, ko1 = gk0 + xk, po = gp0 + xp - psz, po1 = gp0 + xp;
  run_k = gk1;
  run_p = gp1;
  const uint32_t c = cur.c, r = cur.r, a = cur.a;
  const uint64_t e = cur.e;
  const bool lng = uint64_t(r) + a > A.max_seq_len;
  uint8_t st = AVDB_KEY_HOST;
  if (live) {
    off_store<NARROW>(A.key_off, A.n, i, ko);
    if (A.code) off_store<NARROW>(A.path_off, A.n, i, po);
    if (i + 1 == A.n) {
      off_store<NARROW>(A.key_off, A.n, A.n, ko1);
      if (A.code) off_store<NARROW>(A.path_off, A.n, A.n, po1);
    }
    st = AVDB_KEY_OK;
    if (c >= n_chrom || (e >> 63)) st = AVDB_KEY_HOST;  // no label / interned external id
    else if (lng && !A.digest) st = A.defer ? AVDB_KEY_DIGEST_PENDING : AVDB_KEY_NEED_DIGEST;
    else if (!lng && cur.off + r + a > A.heap_bytes) st = AVDB_KEY_HOST;
    if ((st == AVDB_KEY_OK || st == AVDB_KEY_DIGEST_PENDING) && ko1 > A.key_cap) st = AVDB_KEY_OVERFLOW;
  }
  // the body's two ranges: a long record's 32 digest characters, or ref then alt
  // (windows loaded up front, independent of each other); a pending digest is 32
  // zero bytes here
  const bool kok = st == AVDB_KEY_OK || st == AVDB_KEY_DIGEST_PENDING;
  uint64_t W1[kWinWords], W2[kWinWords];
  uint32_t m1 = 0, n1 = 0, m2 = 0, n2 = 0;
  bool wide = false;  // a range past the window (max_seq_len > 50): the per-piece path
#pragma unroll
  for (uint32_t k = 0; k < kWinWords; ++k) W1[k] = W2[k] = 0;
  if (kok) {
    if (lng) {
      n1 = AVDB_DIGEST_CHARS;
      if (A.digest) {
        const uintptr_t s1 = reinterpret_cast<uintptr_t>(A.digest) + 32 * i;
        m1 = uint32_t(s1 & 7);
        load_win(W1, s1, n1, Heap{s1, s1 + AVDB_DIGEST_CHARS});
      }
    } else {
      const uintptr_t s1 = reinterpret_cast<uintptr_t>(A.heap) + cur.off, s2 = s1 + r;
      n1 = r;
      n2 = a;
      m1 = uint32_t(s1 & 7);
      m2 = uint32_t(s2 & 7);
      wide = m1 + n1 > 8 * kWinWords || m2 + n2 > 8 * kWinWords;
      if (!wide) {
        load_win(W1, s1, n1, hheap);
        load_win(W2, s2, n2, hheap);
      }
    }
  }
  // stream 0: keys
  const bool kst = gk1 - (gk0 & ~uint64_t(15)) + 16 <= kKeyWave && gk1 <= A.key_cap;
  uint64_t bad = 0;
  auto render_key = [&](auto o) {  // primary_key_generator.py:106-122
    uint64_t q0, q1;
    const uint32_t lp = key_prefix(c, dp, &q0, &q1);
    append2(o, q0, q1, lp);
    if (!wide) {
      append_win(o, W1, m1, n1, bad);
      if (!lng) o.put(':');
      append_win(o, W2, m2, n2, bad);
    } else {
      const uint64_t off = cur.off;
      if (!key_allele_ok((glb_cp)(A.heap + off), r + a)) bad = kHiBits;
      o.bytes((glb_cp)(A.heap + off), r);
      o.put(':');
      o.bytes((glb_cp)(A.heap + off + r), a);
    }
    if (e) {  // ':rs' + the refSNP number (not interned: bit 63 clear)
      if (e32) {
        append2(o, 0x73723Aull | (de.lo << 24), (de.lo >> 40) | (de.hi << 24), 3 + de.n);
      } else {
        o.lit(":rs");
        o.u64v(e);
      }
    }
    return o;
  };
  if (kok) {
    if (kst) {
      Out<true, true> o(LdsImage{}, kimg, ko - (gk0 & ~uint64_t(15)));
      render_key(o).finish();
    } else {
      Out<true> o(A.key_out, ko);
      render_key(o).finish();
    }
    if (bad) st = AVDB_KEY_HOST;
  }
  // stream 1: ltree paths
  bool pst = false, path_over = false;
  if (A.code) {
    pst = gp1 - (gp0 & ~uint64_t(15)) + 16 <= kPathWave && gp1 <= A.path_cap;
    const uint32_t cd = live ? cur.cd : AVDB_BIN_NONE;
    const bool has_path = live && cd != AVDB_BIN_NONE && c < n_chrom;
    path_over = has_path && po1 > A.path_cap;
    if (has_path && !path_over) {
      if (pst) {
        Out<true, true> o(LdsImage{}, pimg, po - (gp0 & ~uint64_t(15)));
        bin_path<true>(o, c, cd).finish();
      } else {
        Out<true> o(A.path_out, po);
        bin_path<true>(o, c, cd).finish();
      }
    }
  }
  if (live) A.state[i] = st | (path_over ? AVDB_PATH_OVERFLOW : 0u);
  wave_lds_sync();
  if (kst) flush_span32(kimg, A.key_out, gk0, gk1, lane);
  if (pst) flush_span32(pimg, A.path_out, gp0, gp1, lane);
  wave_lds_sync();
}

#ifndef AVDB_K7_V2_BLOCK
#define AVDB_K7_V2_BLOCK 64  // write-pass workgroup size: one wave (waves share nothing; against 256 threads K7 -0.5 to -0.9 %, A/B knob)
#endif
constexpr uint32_t kV2Block = AVDB_K7_V2_BLOCK, kV2Waves = kV2Block / kWave;
#ifndef AVDB_K7_V2_WAVES
#define AVDB_K7_V2_WAVES 4
#endif
template <bool NARROW>
__global__ __launch_bounds__(kV2Block, AVDB_K7_V2_WAVES) void k_record_keys_v2(KeyArgs A) {
  __shared__ uint64_t s_kimg[kV2Waves * kKeyWave / 8];
  __shared__ uint64_t s_pimg[kV2Waves * kPathWave / 8];
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  lds_u64* kimg = (lds_u64*)s_kimg + wv * (kKeyWave / 8);
  lds_u64* pimg = (lds_u64*)s_pimg + wv * (kPathWave / 8);
  for (uint32_t q = lane; q < kKeyWave / 8; q += kWave) kimg[q] = 0;
  for (uint32_t q = lane; q < kPathWave / 8; q += kWave) pimg[q] = 0;
  wave_lds_sync();
  const Heap hheap = make_heap(A.heap, A.heap_bytes);
  auto load_in = [&](size_t t) {
    KeyTileIn v{};
    const size_t j = t + lane;
    if (j < A.n) {
      v.c = A.chrom[j];
      v.p = A.pos[j];
      v.r = A.rl[j];
      v.a = A.al[j];
      v.e = A.ext ? A.ext[j] : 0ull;
      v.off = A.off[j];
      if (A.code) v.cd = A.code[j];
    }
    return v;
  };
  const size_t gwave = size_t(blockIdx.x) * kV2Waves + wv, n_gw = size_t(gridDim.x) * kV2Waves;
  const uint32_t tpg = 1u << A.group_log2;
  size_t t0 = gwave * (size_t(kWave) << A.group_log2);
  KeyTileIn nx{};
  if (t0 < A.n) nx = load_in(t0);
  uint64_t run_k = 0, run_p = 0;
  for (size_t tn = 0; t0 < A.n; t0 = tn) {
    tn = ((t0 / kWave) & (tpg - 1)) != tpg - 1 ? t0 + kWave
                                               : t0 - size_t(tpg - 1) * kWave + n_gw * (size_t(kWave) << A.group_log2);
    const KeyTileIn cur = nx;
    if (tn < A.n) nx = load_in(tn);
    if (((t0 / kWave) & (tpg - 1)) == 0) {  // a new group: its scanned base
      const size_t g = (t0 / kWave) >> A.group_log2;
      const size_t b = g / kGroupsPerBlock;
      const uint2 gp = A.grp_pre[g];
      if (A.blk_raw) {
        uint64_t bk = 0, bp = 0;
        for (size_t q = lane; q < b; q += kWave) {
          bk += A.blk_pre[2 * q];
          bp += A.blk_pre[2 * q + 1];
        }
        run_k = wave_sum64(bk) + gp.x;
        run_p = wave_sum64(bp) + gp.y;
      } else {
        run_k = A.blk_pre[2 * b] + gp.x;
        run_p = A.blk_pre[2 * b + 1] + gp.y;
      }
    }
    key_tile<NARROW>(A, cur, t0, run_k, run_p, kimg, pimg, hheap, lane);
  }
}

// avdb_primary_keys_fill_digests: the 32 digest characters of every key K7 left
// pending, at key_off[i] + len("label:pos:"), then its state AVDB_KEY_OK.  A wave
// reads 1,024 states per step (16 per lane); the pending ones (the long records)
// load their digest row as two 16-byte loads and store it as four 8-byte stores.
__global__ __launch_bounds__(kBlock) void k_fill_digests(const uint8_t* __restrict__ chrom,
                                                         const uint32_t* __restrict__ pos, size_t n,
                                                         const char* __restrict__ digest,
                                                         const uint64_t* __restrict__ key_off,
                                                         uint8_t* __restrict__ key_out, uint8_t* __restrict__ state) {
  const size_t stride = size_t(gridDim.x) * blockDim.x * 16;
  for (size_t j0 = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) * 16; j0 < n; j0 += stride) {
    uint8_t st[16];
    if (j0 + 16 <= n) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(state + j0);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) st[k] = uint8_t(w[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) st[k] = j0 + k < n ? state[j0 + k] : uint8_t(0);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if ((st[k] & 0x0F) != AVDB_KEY_DIGEST_PENDING) continue;
      const size_t i = j0 + k;
      const uint32_t c = chrom[i];
      const uint64_t at = key_off[i] + key_body_at(c, pos[i]);  // (the layout key_prefix renders)
      const u32x4* d = reinterpret_cast<const u32x4*>(digest + 32 * i);
      const u32x4 d0 = d[0], d1 = d[1];
      gw_u64u q = reinterpret_cast<gw_u64u>((gbyte*)key_out + at);
      q[0].v = uint64_t(d0.x) | (uint64_t(d0.y) << 32);
      q[1].v = uint64_t(d0.z) | (uint64_t(d0.w) << 32);
      q[2].v = uint64_t(d1.x) | (uint64_t(d1.y) << 32);
      q[3].v = uint64_t(d1.z) | (uint64_t(d1.w) << 32);
      state[i] = uint8_t((st[k] & 0xF0) | AVDB_KEY_OK);
    }
  }
}

// ---------------------------------------------------------------------------
// The keyed step's record prep and its text in ONE pass (avdb_keyed_prep; the
// round-6 form of K2 + K7).  K2 (end, bin, status; K3's marks, K4's long codes,
// the L8 histogram and counters) and K7 (keys + ltree paths) both read the whole
// SoA; run as two kernels the SoA and the bin codes cross HBM twice (29 + 4 B per
// record, 4.2 GB of C4k's 34 GB).  Here a workgroup of four waves takes one group
// of 256 * kOpTpw records (kOpTpw 64-record tiles per wave, one record per lane
// per tile, held in registers from the K2 half to the K7 half):
//   1. SoA loads, heap peeks, end / bin / status, the marks and codes, and the
//      tile's key / path byte totals (key_path_sizes, what the keyed K2 summed);
//   2. a decoupled look-back over the groups for the group's text offsets:
//      a group (= workgroup index, dispatched in order) publishes its totals
//      first, then sums its predecessors' back to the nearest published
//      inclusive prefix (8-byte {flag, value} granules, agent-scope atomic
//      loads / stores: MI355X_MICROARCH.md's granule hand-off);
//   3. each wave renders its tile (key_tile, K7's write pass) from the registers
//      phase 1 loaded.
// The round-1 look-back over 64-record tiles polled with plain loads (168 ms for
// C4k); here a group is 1,024 records and every poll is an agent-scope load.
// Long records' keys are laid out with their digest pending (A.defer): K4 runs
// after this pass on the codes it wrote and writes the digests into the keys
// (avdb_vrs_digest_keys).  Measured slower than K2 then K7 (8.13 vs 6.0 ms on
// C4k: the look-back waits), so it is an opt-in layout.
// The histogram and counters go through per-group partials (k_keyed_stats), so no
// workgroup holds a 24 KB LDS histogram beside K7's 32 KB of text images.
// ---------------------------------------------------------------------------
#ifndef AVDB_OP_WAVES
#define AVDB_OP_WAVES 4  // waves per workgroup (a group: every wave's tiles; one look-back)
#endif
constexpr uint32_t kOpWaves = AVDB_OP_WAVES;
constexpr uint32_t kOpBlock = kOpWaves * kWave;
constexpr uint32_t kOpGroup = kOpWaves * kWave;      // records per group and tile of its waves
#ifndef AVDB_OP_TPW
#define AVDB_OP_TPW 4  // tiles per wave: a group is 256 * this records (one look-back each)
#endif
constexpr uint32_t kOpTpw = AVDB_OP_TPW;
constexpr uint32_t kOpGroupRecs = kOpGroup * kOpTpw;
constexpr uint64_t kLbAgg = uint64_t(1) << 62, kLbInc = uint64_t(2) << 62, kLbVal = kLbAgg - 1;
constexpr uint32_t kLbSpinCap = 1u << 22;            // polls before a (never expected) give-up
constexpr uint32_t kOpSlicesMax = 4096;              // K3 list slices (avdb_pk_dedup_ex's resolve grid)

struct PrepArgs {
  uint32_t* end;
  uint32_t* code;
  uint8_t* status;          // nullable
  uint8_t* keep;            // nullable: no K3 marks
  uint32_t* dd_counts;      // [slices], zeroed by k_keyed_init
  uint32_t* dd_list;        // slice s at dd_list + s * dd_slice
  size_t dd_slice;
  uint32_t dd_slices;
  uint8_t* long_codes;      // nullable: no K4 codes
  uint4* grp_stat;          // nullable: no histogram / counters; per group {key0, cnt0, key1, cnt1},
                            // {status 1, 2, 3 counts, 0}
  uint32_t* hist;           // nullable: waves of mixed L8 keys add here directly
  unsigned long long* lb;   // [2 * groups] look-back granules (keys, paths), zeroed by k_keyed_init
  uint32_t* hdr;            // [1] look-back give-ups (zeroed by k_keyed_init)
  size_t n_groups;
  uint32_t max_seq_len;
};

__device__ __forceinline__ void lb_store(unsigned long long* p, uint64_t v) {
  __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of group g: publish (agg_k, agg_p), look back, publish the inclusive
// prefixes; returns the exclusive ones (every lane).  A look-back step reads
// kLbPerLane groups per lane (256 per step): at C4k's rate (~25 groups of 1,024
// records per microsecond) an agent-scope round trip of a few microseconds then
// reaches the nearest published inclusive prefix in one step.
constexpr uint32_t kLbPerLane = 4;
__device__ __forceinline__ void group_lookback(unsigned long long* lb, uint32_t* hdr, size_t g, uint64_t agg_k,
                                               uint64_t agg_p, uint64_t* xk, uint64_t* xp) {
  const uint32_t lane = __lane_id();
  if (g == 0) {
    if (lane == 0) {
      lb_store(lb, kLbInc | agg_k);
      lb_store(lb + 1, kLbInc | agg_p);
    }
    *xk = *xp = 0;
    return;
  }
  if (lane == 0) {
    lb_store(lb + 2 * g, kLbAgg | agg_k);
    lb_store(lb + 2 * g + 1, kLbAgg | agg_p);
  }
  uint64_t ek = 0, ep = 0;
  bool gave_up = false;
  for (int64_t q0 = int64_t(g) - 1; q0 >= 0; q0 -= int64_t(kWave) * kLbPerLane) {
    uint64_t sk[kLbPerLane], sp[kLbPerLane];
#pragma unroll
    for (uint32_t j = 0; j < kLbPerLane; ++j) {
      const int64_t q = q0 - int64_t(kLbPerLane * lane + j);
      sk[j] = sp[j] = 0;
      if (q >= 0) {
        for (uint32_t spin = 0;; ++spin) {
          sk[j] = lb_load(lb + 2 * size_t(q));
          sp[j] = lb_load(lb + 2 * size_t(q) + 1);
          if ((sk[j] >> 62) && (sk[j] >> 62) == (sp[j] >> 62)) break;
          if (spin == kLbSpinCap) {
            sk[j] = sp[j] = kLbInc;
            gave_up = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    // the nearest inclusive prefix: the first (lane, j) in window order
    uint32_t jstop = kLbPerLane;
#pragma unroll
    for (int j = int(kLbPerLane) - 1; j >= 0; --j)
      if (q0 - int64_t(kLbPerLane * lane + uint32_t(j)) >= 0 && (sk[j] >> 62) == 2) jstop = uint32_t(j);
    const uint64_t inc = __ballot(jstop < kLbPerLane);
    const uint32_t stop = inc ? uint32_t(__ffsll((unsigned long long)inc)) - 1 : uint32_t(kWave);
    uint64_t vk = 0, vp = 0;
#pragma unroll
    for (uint32_t j = 0; j < kLbPerLane; ++j) {
      const int64_t q = q0 - int64_t(kLbPerLane * lane + j);
      const bool take = q >= 0 && (lane < stop || (lane == stop && j <= jstop));
      vk += take ? (sk[j] & kLbVal) : 0ull;
      vp += take ? (sp[j] & kLbVal) : 0ull;
    }
    ek += wave_sum64(vk);
    ep += wave_sum64(vp);
    if (inc) break;
  }
  if (gave_up) atomicAdd(hdr + 1, 1u);
  if (lane == 0) {
    lb_store(lb + 2 * g, kLbInc | (ek + agg_k));
    lb_store(lb + 2 * g + 1, kLbInc | (ep + agg_p));
  }
  *xk = ek;
  *xp = ep;
}

__global__ __launch_bounds__(kBlock) void k_keyed_init(PrepArgs P) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t j = size_t(blockIdx.x) * blockDim.x + threadIdx.x; j < 2 * P.n_groups; j += stride) P.lb[j] = 0;
  for (size_t j = size_t(blockIdx.x) * blockDim.x + threadIdx.x; j < P.dd_slices; j += stride) P.dd_counts[j] = 0;
  if (blockIdx.x == 0 && threadIdx.x < 2) P.hdr[threadIdx.x] = 0;
}

template <uint32_t TPW>
__global__ __launch_bounds__(kOpBlock, 4) void k_keyed_onepass(KeyArgs A, PrepArgs P, ChromTable tab) {
  __shared__ uint64_t s_kimg[kOpWaves * kKeyWave / 8];
  __shared__ uint64_t s_pimg[kOpWaves * kPathWave / 8];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM], s_l8off[AVDB_MAX_CHROM];
  __shared__ uint32_t s_tk[kOpWaves], s_tp[kOpWaves], s_dd[kOpWaves], s_hk[kOpWaves], s_hc[kOpWaves],
      s_err[kOpWaves];
  __shared__ uint64_t s_base[2];
  __shared__ uint32_t s_ddat;
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave, tid = threadIdx.x;
  lds_u64* kimg = (lds_u64*)s_kimg + wv * (kKeyWave / 8);
  lds_u64* pimg = (lds_u64*)s_pimg + wv * (kPathWave / 8);
  for (uint32_t q = lane; q < kKeyWave / 8; q += kWave) kimg[q] = 0;
  for (uint32_t q = lane; q < kPathWave / 8; q += kWave) pimg[q] = 0;
  if (tid < AVDB_MAX_CHROM) {
    s_len[tid] = tab.len[tid];
    s_l8off[tid] = tab.l8_off[tid];
  }
  __syncthreads();
  // Group = workgroup index.  A group waits only on groups before it, and workgroups
  // are dispatched in index order (rocPRIM's look-back scans rely on the same), so
  // every group waited on has started; a ticket from one atomic counter instead
  // (the launch-order guarantee without that reliance) serialised 488 k workgroups
  // at ~88 claims per microsecond.  A poll that never sees its predecessor gives up
  // after kLbSpinCap tries and counts itself (avdb_keyed_prep_lookback_errors), so a
  // broken order cannot hang.
  const size_t g = blockIdx.x;
  const size_t w0 = g * (size_t(kOpGroup) * TPW) + size_t(wv) * (kWave * TPW);  // this wave's first record
  const Heap hp = make_heap(A.heap, A.heap_bytes);

  // ---- 1. the SoA once (all TPW tiles' loads in flight together); K2's record
  // arithmetic (variant_annotator.py:36-79, bin_index.py:59-75)
  KeyTileIn cur[TPW];
  uint64_t wr[TPW], wa[TPW];
#pragma unroll
  for (uint32_t k = 0; k < TPW; ++k) {
    const size_t i = w0 + k * kWave + lane;
    cur[k] = KeyTileIn{};
    cur[k].cd = AVDB_BIN_NONE;
    if (i < A.n) {
      cur[k].c = A.chrom[i];
      cur[k].p = A.pos[i];
      cur[k].r = A.rl[i];
      cur[k].a = A.al[i];
      cur[k].e = A.ext ? A.ext[i] : 0ull;
      cur[k].off = A.off[i];
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < TPW; ++k) {
    const bool live = w0 + k * kWave + lane < A.n, snv = cur[k].r == 1u && cur[k].a == 1u;
    wr[k] = live && !snv ? heap_u64(hp, cur[k].off) : 0ull;
    wa[k] = live && !snv ? heap_u64(hp, cur[k].off + cur[k].r) : 0ull;
  }
  uint32_t hk = 0xFFFFFFFFu, hc = 0, e1 = 0, e2 = 0, e3 = 0, K = 0, Pt = 0, dd = 0;
  uint64_t listed[TPW];
  uint64_t prev_sm = 0;  // the previous tile's "shares its predecessor's position" ballot
#pragma unroll
  for (uint32_t k = 0; k < TPW; ++k) {
    const size_t i = w0 + k * kWave + lane;
    const bool live = i < A.n;
    uint32_t st = 0, key8 = 0xFFFFFFFFu;
    if (live) {
      uint32_t lcp, cd;
      const uint32_t e = infer_end(hp, cur[k].off, cur[k].r, cur[k].a, cur[k].p, wr[k], wa[k], &lcp);
      st = classify(cur[k].c, cur[k].p, e, tab.n, s_len, &cd);
      cur[k].cd = cd;
      __builtin_nontemporal_store(e, P.end + i);
      __builtin_nontemporal_store(cd, P.code + i);
      if (P.status) P.status[i] = uint8_t(st);
      if (P.long_codes) P.long_codes[i] = uint8_t(long_code(cur[k].r, cur[k].a, P.max_seq_len));
      if (P.keep) P.keep[i] = 1;
      if (cd != AVDB_BIN_NONE) key8 = s_l8off[cur[k].c] + (cur[k].p - 1u) / kL8Width;
    }
    // K3's first phase (removeDuplicates.sql:2-24 keep-first): a record that shares
    // (chrom, pos) with its predecessor is listed for the resolve if it could repeat
    // a primary key before it — the predecessor's lengths and refSNP id, or third or
    // later at its position (the keyed K2's filter, avdb_bins.hip)
    listed[k] = 0;
    if (P.keep) {
      uint32_t pc = __shfl_up(cur[k].c, 1, kWave), pp = __shfl_up(cur[k].p, 1, kWave);
      uint32_t pr = __shfl_up(cur[k].r, 1, kWave), pa = __shfl_up(cur[k].a, 1, kWave);
      uint64_t pe = (uint64_t(uint32_t(__shfl_up(uint32_t(cur[k].e >> 32), 1, kWave))) << 32) |
                    uint32_t(__shfl_up(uint32_t(cur[k].e), 1, kWave));
      uint32_t p2 = 0;  // lane 0: record i-1 shares its predecessor's position
      if (k == 0) {
        if (lane == 0 && live && i > 0) {
          pc = A.chrom[i - 1];
          pp = A.pos[i - 1];
          pr = A.rl[i - 1];
          pa = A.al[i - 1];
          pe = A.ext ? A.ext[i - 1] : 0ull;
          p2 = uint32_t(i >= 2 && A.chrom[i - 2] == pc && A.pos[i - 2] == pp);
        }
      } else {  // the previous tile's last record (lane 63) is the predecessor
        const uint32_t qc = __builtin_amdgcn_readlane(cur[k - 1].c, kWave - 1);
        const uint32_t qp = __builtin_amdgcn_readlane(cur[k - 1].p, kWave - 1);
        const uint32_t qr = __builtin_amdgcn_readlane(cur[k - 1].r, kWave - 1);
        const uint32_t qa = __builtin_amdgcn_readlane(cur[k - 1].a, kWave - 1);
        const uint64_t qe = (uint64_t(__builtin_amdgcn_readlane(uint32_t(cur[k - 1].e >> 32), kWave - 1)) << 32) |
                            __builtin_amdgcn_readlane(uint32_t(cur[k - 1].e), kWave - 1);
        if (lane == 0) {
          pc = qc;
          pp = qp;
          pr = qr;
          pa = qa;
          pe = qe;
          p2 = uint32_t(prev_sm >> (kWave - 1));
        }
      }
      const bool same = live && i > 0 && cur[k].c == pc && cur[k].p == pp;
      const uint64_t sm = __ballot(same);
      const uint32_t psame = lane == 0 ? p2 : uint32_t((sm >> (lane - 1)) & 1ull);
      const bool cand = cur[k].r == pr && cur[k].a == pa && cur[k].e == pe;
      listed[k] = __ballot(same && (cand || psame));
      prev_sm = sm;
      dd += uint32_t(__popcll(listed[k]));
    }
    // the L8 histogram / status counters as this wave's partials (k_keyed_stats)
    if (P.grp_stat) {
      const uint64_t valid = __ballot(key8 != 0xFFFFFFFFu);
      if (valid) {
        const uint32_t k0 = __builtin_amdgcn_readlane(key8, uint32_t(__ffsll((unsigned long long)valid)) - 1);
        if (!__ballot(key8 != 0xFFFFFFFFu && key8 != k0)) {
          const uint32_t cnt = uint32_t(__popcll(valid));
          if (hc && k0 != hk) {  // (uniform) a second key in this wave's tiles: the first goes out now
            if (P.hist && lane == 0) atomicAdd(P.hist + hk, hc);
            hc = 0;
          }
          hk = k0;
          hc += cnt;
        } else if (P.hist) {
          wave_hist_add(key8, P.hist);  // a tile across an L8 boundary (sorted) or unsorted records
        }
      }
      e1 += uint32_t(__popcll(__ballot(st == 1u)));
      e2 += uint32_t(__popcll(__ballot(st == 2u)));
      e3 += uint32_t(__popcll(__ballot(st == 3u)));
    }
    // the tile's key / path bytes (key_tile renders exactly these: key_path_sizes)
    uint32_t ks = 0, ps = 0;
    if (live)
      key_path_sizes(cur[k].c, cur[k].p, cur[k].r, cur[k].a, cur[k].e, cur[k].cd, A.max_seq_len, uint32_t(A.n_chrom),
                     A.digest != nullptr || A.defer, A.code != nullptr, &ks, &ps);
    K += wave_sum32(ks);
    Pt += wave_sum32(ps);
  }
  if (lane == 0) {
    s_tk[wv] = K;
    s_tp[wv] = Pt;
    s_dd[wv] = dd;
    s_hk[wv] = hk;
    s_hc[wv] = hc;
    s_err[wv] = e1 | (e2 << 10) | (e3 << 20);
  }
  __syncthreads();

  // ---- 2. the group's offsets (wave 0), its K3 slice space and statistics
  if (wv == 0) {
    uint64_t ak = 0, ap = 0;
    uint32_t gdd = 0;
#pragma unroll
    for (uint32_t w = 0; w < kOpWaves; ++w) {
      ak += s_tk[w];
      ap += s_tp[w];
      gdd += s_dd[w];
    }
    uint32_t at = 0;
    if (lane == 0 && gdd) at = atomicAdd(P.dd_counts + (g % P.dd_slices), gdd);
    if (lane == 0 && P.grp_stat) {
      uint32_t k0 = 0xFFFFFFFFu, c0 = 0, k1 = 0xFFFFFFFFu, c1 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
      for (uint32_t w = 0; w < kOpWaves; ++w) {
        const uint32_t kk = s_hk[w], c = s_hc[w];
        r1 += s_err[w] & 0x3FFu;
        r2 += (s_err[w] >> 10) & 0x3FFu;
        r3 += s_err[w] >> 20;
        if (!c) continue;
        if (kk == k0 || !c0) {
          k0 = kk;
          c0 += c;
        } else if (kk == k1 || !c1) {
          k1 = kk;
          c1 += c;
        } else if (P.hist) {
          atomicAdd(P.hist + kk, c);
        }
      }
      P.grp_stat[2 * g] = make_uint4(k0, c0, k1, c1);
      P.grp_stat[2 * g + 1] = make_uint4(r1, r2, r3, 0);
    }
    uint64_t xk, xp;
    group_lookback(P.lb, P.hdr, g, ak, ap, &xk, &xp);
    if (lane == 0) {
      s_base[0] = xk;
      s_base[1] = xp;
      s_ddat = at;
    }
  }
  __syncthreads();

  // ---- 3. the K3 list entries and this wave's tiles of text
  if (dd) {
    uint32_t before = s_ddat;
    for (uint32_t w = 0; w < wv; ++w) before += s_dd[w];
    uint32_t* slot = P.dd_list + size_t(g % P.dd_slices) * P.dd_slice;
#pragma unroll
    for (uint32_t k = 0; k < TPW; ++k) {
      if ((listed[k] >> lane) & 1ull)
        slot[before + uint32_t(__popcll(listed[k] & ((1ull << lane) - 1)))] = uint32_t(w0 + k * kWave + lane);
      before += uint32_t(__popcll(listed[k]));
    }
  }
  uint64_t run_k = s_base[0], run_p = s_base[1];
  for (uint32_t w = 0; w < wv; ++w) {
    run_k += s_tk[w];
    run_p += s_tp[w];
  }
  wave_lds_sync();  // (this wave's images were zeroed above)
  // (written out: a loop over key_tile is too large for the unroller, and cur[] indexed
  // at run time would live in scratch)
  key_tile(A, cur[0], w0, run_k, run_p, kimg, pimg, hp, lane);
  if constexpr (TPW > 1) key_tile(A, cur[1 % TPW], w0 + kWave, run_k, run_p, kimg, pimg, hp, lane);
  if constexpr (TPW > 2) key_tile(A, cur[2 % TPW], w0 + 2 * kWave, run_k, run_p, kimg, pimg, hp, lane);
  if constexpr (TPW > 3) key_tile(A, cur[3 % TPW], w0 + 3 * kWave, run_k, run_p, kimg, pimg, hp, lane);
  static_assert(TPW >= 1 && TPW <= 4, "tiles per wave");
}

// the histogram and counters from the groups' partials: a thread per 8 groups,
// one atomic per run of one L8 key (a sorted batch: a few per wave)
constexpr uint32_t kStatGroups = 8;
__global__ __launch_bounds__(kBlock) void k_keyed_stats(const uint4* __restrict__ grp, size_t n_groups, size_t n,
                                                        uint32_t* __restrict__ hist,
                                                        unsigned long long* __restrict__ ctr) {
  __shared__ unsigned long long s_c[4];
  if (threadIdx.x < 4) s_c[threadIdx.x] = 0;
  __syncthreads();
  const size_t g0 = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) * kStatGroups;
  uint32_t rk = 0xFFFFFFFFu, rc = 0, e1 = 0, e2 = 0, e3 = 0;
  uint64_t recs = 0;
  uint4 v[kStatGroups], x[kStatGroups];
#pragma unroll
  for (uint32_t k = 0; k < kStatGroups; ++k) {
    v[k] = g0 + k < n_groups ? grp[2 * (g0 + k)] : make_uint4(0xFFFFFFFFu, 0, 0xFFFFFFFFu, 0);
    x[k] = g0 + k < n_groups ? grp[2 * (g0 + k) + 1] : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (uint32_t k = 0; k < kStatGroups; ++k) {
    if (g0 + k >= n_groups) break;
    const size_t r0 = (g0 + k) * kOpGroupRecs;
    recs += n - r0 < kOpGroupRecs ? n - r0 : kOpGroupRecs;
    e1 += x[k].x;
    e2 += x[k].y;
    e3 += x[k].z;
    const uint32_t kk[2] = {v[k].x, v[k].z}, cc[2] = {v[k].y, v[k].w};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (!cc[q]) continue;
      if (kk[q] != rk) {
        if (rc && hist) atomicAdd(hist + rk, rc);
        rk = kk[q];
        rc = 0;
      }
      rc += cc[q];
    }
  }
  if (rc && hist) atomicAdd(hist + rk, rc);
  if (ctr) {
    const uint64_t t_rec = wave_sum64(recs);
    const uint64_t t1 = wave_sum64(e1), t2 = wave_sum64(e2), t3 = wave_sum64(e3);
    if (__lane_id() == 0) {
      atomicAdd(&s_c[0], (unsigned long long)t_rec);
      atomicAdd(&s_c[1], (unsigned long long)t1);
      atomicAdd(&s_c[2], (unsigned long long)t2);
      atomicAdd(&s_c[3], (unsigned long long)t3);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long bad_all = s_c[1] + s_c[2] + s_c[3];
      if (s_c[0]) {
        atomicAdd(ctr + AVDB_CTR_RECORDS, s_c[0]);
        atomicAdd(ctr + AVDB_CTR_STATUS0, s_c[0] - bad_all);
      }
      for (int k = 1; k <= 3; ++k)
        if (s_c[k]) atomicAdd(ctr + AVDB_CTR_STATUS0 + k, s_c[k]);
    }
  }
}

}  // namespace avdb

using namespace avdb;

static size_t scan_bytes(size_t n) { return (scan::workspace_bytes(n, 2) + 255) & ~size_t(255); }

extern "C" int avdb_display_attributes(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                       const uint32_t* end, const uint64_t* allele_off,
                                       const uint32_t* ref_len, const uint32_t* alt_len,
                                       const uint8_t* heap, size_t heap_bytes, size_t n, void* workspace,
                                       size_t workspace_bytes, uint64_t* out_off, uint8_t* out,
                                       uint8_t* rec_state, void* stream) {
  if (!ctx || !out_off || !rec_state) {
    avdb_set_error("avdb_display_attributes: null argument");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* oo = reinterpret_cast<unsigned long long*>(out_off);
  if (!out) {  // size pass + scan
    AVDB_HIP_TRY(hipMemsetAsync(oo + n, 0, 8, s));
    if (n == 0) return AVDB_OK;
    if (!chrom || !pos || !end || !allele_off || !ref_len || !alt_len || !heap) {
      avdb_set_error("avdb_display_attributes: null array");
      return AVDB_EINVAL;
    }
    size_t need = 0;
    avdb_format_workspace_size(n, &need);
    if (!workspace || workspace_bytes < need) {
      avdb_set_error("avdb_display_attributes: workspace of %zu bytes required", need);
      return AVDB_ERANGE;
    }
    const unsigned grid = stream_grid(n, kBlock, 4096);
    hipLaunchKernelGGL(k_display<false>, dim3(grid), dim3(kBlock), 0, s, chrom, pos, end, allele_off,
                       ref_len, alt_len, heap, heap_bytes, n, out_off, nullptr, rec_state);
    AVDB_LAUNCH_CHECK("k_display<size>");
    size_t tb = scan_bytes(n + 1);
    if (int e = scan::exclusive_u64(oo, oo, n + 1, workspace, tb, s)) return e;
    return AVDB_OK;
  }
  if (n == 0) return AVDB_OK;
  if (reinterpret_cast<uintptr_t>(out) % 8) {
    avdb_set_error("avdb_display_attributes: output must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  const unsigned grid = stream_grid(n, kBlock, 4096);
  hipLaunchKernelGGL(k_display<true>, dim3(grid), dim3(kBlock), 0, s, chrom, pos, end, allele_off, ref_len,
                     alt_len, heap, heap_bytes, n, out_off, out, rec_state);
  AVDB_LAUNCH_CHECK("k_display<write>");
  return AVDB_OK;
}

// ---- K7 with group offsets --------------------------------------------------------
#ifndef AVDB_K7_SMALL_LOG2
#define AVDB_K7_SMALL_LOG2 0u  // group size below kSmallGroupN records (A/B knob: 64 << this)
#endif
static uint32_t key_group_log2(size_t n) { return n < kSmallGroupN ? uint32_t(AVDB_K7_SMALL_LOG2) : kGroupLog2; }
static size_t key_groups(size_t n) {
  const size_t g = size_t(kWave) << key_group_log2(n);
  return (n + g - 1) / g;
}
static size_t key_group_blocks(size_t n) { return (key_groups(n) + kGroupsPerBlock - 1) / kGroupsPerBlock; }

namespace avdb {
// the keyed K2 (avdb_record_prep_keyed) writes K7's group totals straight into the
// one-pass workspace, at the group size K7 uses for n records
uint32_t key_totals_group_log2(size_t n) { return key_group_log2(n); }
uint2* key_totals_of(void* workspace) { return reinterpret_cast<uint2*>(static_cast<char*>(workspace) + 256); }
}  // namespace avdb

extern "C" int avdb_primary_keys_onepass_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = 256 + 16 * ((key_groups(n) + 1) & ~size_t(1)) + 16 * key_group_blocks(n);
  return AVDB_OK;
}

namespace avdb {
// the two-call form (avdb_format_workspace_size): the size call's paired scan,
// and the write call's one-pass layout (group totals and their scans)
size_t key_size_workspace(size_t n) {
  size_t one = 0;
  avdb_primary_keys_onepass_workspace_size(n, &one);
  const size_t sc = scan_bytes(n + 1);
  return sc > one ? sc : one;
}
}  // namespace avdb

extern "C" int avdb_primary_keys_bound(size_t n, size_t heap_bytes, size_t* key_cap, size_t* path_cap) {
  if (!key_cap || !path_cap) return AVDB_EINVAL;
  // key: label (2) ':' pos (10) ':' ref ':' alt | digest (32), ':rs' + 19 digits
  *key_cap = 69 * n + heap_bytes + 8;
  // path: "chr" + label (2) + 13 levels of <= 7 bytes, B up to 3 digits at L1
  *path_cap = 98 * n + 8;
  return AVDB_OK;
}

static KeyArgs key_args(const avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                        const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                        const uint64_t* ext_id, const uint32_t* bin_code, const char* digest, size_t n,
                        uint32_t max_seq_len, uint64_t* key_off, uint64_t* path_off, uint8_t* key_out, size_t key_cap,
                        uint8_t* path_out, size_t path_cap, uint8_t* key_state) {
  KeyArgs A;
  memset(&A, 0, sizeof(A));
  A.chrom = chrom;
  A.pos = pos;
  A.off = allele_off;
  A.rl = ref_len;
  A.al = alt_len;
  A.heap = heap;
  A.ext = ext_id;
  A.code = bin_code;
  A.digest = digest;
  A.heap_bytes = heap_bytes;
  A.n = n;
  A.max_seq_len = max_seq_len;
  A.n_chrom = ctx->tab.n < 25 ? ctx->tab.n : 25;  // labelled contigs (chromosomes.py:9-38)
  A.key_off = key_off;
  A.path_off = path_off;
  A.key_cap = key_cap;
  A.path_cap = path_cap;
  A.key_out = key_out;
  A.path_out = path_out;
  A.state = key_state;
  return A;
}

extern "C" int avdb_primary_keys_onepass_ex(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                            const uint64_t* allele_off, const uint32_t* ref_len,
                                            const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                                            const uint64_t* ext_id, const uint32_t* bin_code, const char* digest,
                                            size_t n, uint32_t max_seq_len, void* workspace, size_t workspace_bytes,
                                            uint64_t* key_off, uint64_t* path_off, uint8_t* key_out, size_t key_cap,
                                            uint8_t* path_out, size_t path_cap, uint8_t* key_state, uint32_t flags,
                                            void* stream) {
  if (!ctx || !key_off || (bin_code && !path_off) || !key_state || !key_out || (bin_code && !path_out)) {
    avdb_set_error("avdb_primary_keys_onepass: null argument");
    return AVDB_EINVAL;
  }
  if (flags & ~(AVDB_KEYS_TOTALS_READY | AVDB_KEYS_DIGEST_DEFERRED | AVDB_KEYS_OFF32)) {
    avdb_set_error("avdb_primary_keys_onepass_ex: unknown flags 0x%x", flags);
    return AVDB_EINVAL;
  }
  if ((flags & AVDB_KEYS_DIGEST_DEFERRED) && digest) {
    avdb_set_error("avdb_primary_keys_onepass_ex: AVDB_KEYS_DIGEST_DEFERRED takes digest == NULL");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t ob = (flags & AVDB_KEYS_OFF32) ? off32_bytes(0) : 8;  // (n = 0: low word 0 and base 0)
  if (n == 0) {
    AVDB_HIP_TRY(hipMemsetAsync(key_off, 0, ob, s));
    if (bin_code) AVDB_HIP_TRY(hipMemsetAsync(path_off, 0, ob, s));
    return AVDB_OK;
  }
  if ((flags & AVDB_KEYS_OFF32) && (reinterpret_cast<uintptr_t>(key_off) % 8 || (bin_code && reinterpret_cast<uintptr_t>(path_off) % 8))) {
    avdb_set_error("avdb_primary_keys_onepass_ex: AVDB_KEYS_OFF32 offset buffers must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap) {
    avdb_set_error("avdb_primary_keys_onepass: null array");
    return AVDB_EINVAL;
  }
  if (n >= (size_t(1) << 32)) {
    avdb_set_error("avdb_primary_keys_onepass: n must be < 2^32");
    return AVDB_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(key_out) % 8 || (path_out && reinterpret_cast<uintptr_t>(path_out) % 8)) {
    avdb_set_error("avdb_primary_keys_onepass: outputs must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_primary_keys_onepass_workspace_size(n, &need);
  if (!workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(workspace) % 16) {
    avdb_set_error("avdb_primary_keys_onepass: 16-byte aligned workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  const size_t ng = key_groups(n), nb = key_group_blocks(n);
  char* ws = static_cast<char*>(workspace) + 256;
  auto* tot = reinterpret_cast<uint2*>(ws);
  auto* gpre = tot + ((ng + 1) & ~size_t(1));
  auto* bpre = reinterpret_cast<uint64_t*>(gpre + ((ng + 1) & ~size_t(1)));
  KeyArgs A = key_args(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id, bin_code, digest, n,
                       max_seq_len, key_off, path_off, key_out, key_cap, path_out, path_cap, key_state);
  A.defer = (flags & AVDB_KEYS_DIGEST_DEFERRED) ? 1u : 0u;
  A.off32 = (flags & AVDB_KEYS_OFF32) ? 1u : 0u;
  A.grp_pre = gpre;
  A.blk_pre = bpre;
  A.group_log2 = key_group_log2(n);
  // (avdb_ctx_set_option AVDB_OPT_K7_GRID caps the write pass's workgroups: fewer
  // leave registers to K4 running beside it, AVDB_KEYS_DIGEST_DEFERRED)
  // Below kSmallGroupN records a group is one tile: the default grid is then one
  // resident generation of waves (n_cu x 4 SIMDs x the launch bound), each taking
  // several groups grid-stride, so a wave's image clearing and launch are spread
  // over more tiles (C1, 17 K groups: 0.0898 -> 0.0880 ms per step against one
  // workgroup per group; half a generation 0.109 ms, profiles/c1_ab/r06_k7_grid_ab.txt)
  size_t wmax = ctx->k7_grid > 0 ? size_t(ctx->k7_grid) : size_t(AVDB_K7_GRID) * kWavesPerBlock / kV2Waves;
  if (ctx->k7_grid <= 0 && n < kSmallGroupN)
    wmax = size_t(ctx->n_cu) * 4 * AVDB_K7_V2_WAVES / kV2Waves;
  const size_t wneed = (ng + kV2Waves - 1) / kV2Waves;
  A.blk_raw = nb <= ctx->k7_raw_blocks ? 1u : 0u;
  // the keyed K2 wrote every group's totals but the last one's, which may hold the
  // < 4 records its vector form leaves to a scalar tail: the scan sums that one again
  const int ready = (flags & AVDB_KEYS_TOTALS_READY) ? 1 : 0;
  if (!ready) {
    hipLaunchKernelGGL(k_key_group_totals, dim3(stream_grid(ng * kWave, kBlock, 4096)), dim3(kBlock), 0, s, A, tot,
                       ng, size_t(0));
    AVDB_LAUNCH_CHECK("k_key_group_totals");
  }
  hipLaunchKernelGGL(k_key_group_scan, dim3(unsigned(nb)), dim3(kScanThreads), 0, s, tot, ng, gpre, bpre, A, ready);
  AVDB_LAUNCH_CHECK("k_key_group_scan");
  if (!A.blk_raw) {
    hipLaunchKernelGGL(k_key_block_scan, dim3(1), dim3(kScanThreads), 0, s, bpre, nb, key_off,
                       bin_code ? path_off : nullptr, n, A.off32);
    AVDB_LAUNCH_CHECK("k_key_block_scan");
  }
  // (one workgroup doing both scans for C1's 17 K groups measured 11.9 us against
  // 5.2 + 4.9 us for the two launches: not kept; up to k7_raw_blocks blocks the
  // write pass sums the block totals itself.  One resident generation, 5
  // workgroups per CU, ran 12.3 vs 10.2 ms on C4k, with or without XCD-aware
  // renumbering: the finer grid balances better.)
  const dim3 wgrid(unsigned(wneed < wmax ? wneed : wmax));
  if (A.off32) hipLaunchKernelGGL(k_record_keys_v2<true>, wgrid, dim3(kV2Block), 0, s, A);
  else hipLaunchKernelGGL(k_record_keys_v2<false>, wgrid, dim3(kV2Block), 0, s, A);
  AVDB_LAUNCH_CHECK("k_record_keys_v2");
  return AVDB_OK;
}

extern "C" int avdb_primary_keys_onepass(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                         const uint64_t* allele_off, const uint32_t* ref_len,
                                         const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                                         const uint64_t* ext_id, const uint32_t* bin_code, const char* digest,
                                         size_t n, uint32_t max_seq_len, void* workspace, size_t workspace_bytes,
                                         uint64_t* key_off, uint64_t* path_off, uint8_t* key_out, size_t key_cap,
                                         uint8_t* path_out, size_t path_cap, uint8_t* key_state, void* stream) {
  return avdb_primary_keys_onepass_ex(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id,
                                      bin_code, digest, n, max_seq_len, workspace, workspace_bytes, key_off, path_off,
                                      key_out, key_cap, path_out, path_cap, key_state, 0u, stream);
}

// The two-call form.  Size call (key_out == NULL): each record's sizes in place,
// then one paired exclusive scan into key_off / path_off.  Write call: the one
// write pass above, with its own group totals in `workspace` (the format
// workspace holds the one-pass layout); it writes the same offsets again.
extern "C" int avdb_primary_keys(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                 const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                                 const uint8_t* heap, size_t heap_bytes, const uint64_t* ext_id,
                                 const uint32_t* bin_code, const char* digest, size_t n, uint32_t max_seq_len,
                                 void* workspace, size_t workspace_bytes, uint64_t* key_off, uint64_t* path_off,
                                 uint8_t* key_out, size_t key_cap, uint8_t* path_out, size_t path_cap,
                                 uint8_t* key_state, void* stream) {
  if (!ctx || !key_off || (bin_code && !path_off)) {
    avdb_set_error("avdb_primary_keys: null argument");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  size_t need = 0;
  avdb_format_workspace_size(n, &need);
  if (!key_out) {  // size pass + scans
    auto* ko = reinterpret_cast<unsigned long long*>(key_off);
    auto* po = reinterpret_cast<unsigned long long*>(path_off);
    AVDB_HIP_TRY(hipMemsetAsync(ko + n, 0, 8, s));
    if (bin_code) AVDB_HIP_TRY(hipMemsetAsync(po + n, 0, 8, s));
    if (n == 0) return AVDB_OK;
    if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap) {
      avdb_set_error("avdb_primary_keys: null array");
      return AVDB_EINVAL;
    }
    if (!workspace || workspace_bytes < need) {
      avdb_set_error("avdb_primary_keys: workspace of %zu bytes required", need);
      return AVDB_ERANGE;
    }
    KeyArgs A = key_args(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id, bin_code, digest,
                         n, max_seq_len, key_off, path_off, nullptr, 0, nullptr, 0, nullptr);
    hipLaunchKernelGGL(k_key_sizes, dim3(stream_grid(n, kBlock, 4096)), dim3(kBlock), 0, s, A);
    AVDB_LAUNCH_CHECK("k_key_sizes");
    const size_t tb = scan_bytes(n + 1);
    if (bin_code) return scan::exclusive_u64_pair(ko, ko, po, po, n + 1, workspace, tb, s);
    return scan::exclusive_u64(ko, ko, n + 1, workspace, tb, s);
  }
  if (n == 0) return AVDB_OK;
  if (!key_state || (bin_code && !path_out)) {
    avdb_set_error("avdb_primary_keys: null output");
    return AVDB_EINVAL;
  }
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_primary_keys: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  return avdb_primary_keys_onepass_ex(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id,
                                      bin_code, digest, n, max_seq_len, workspace, workspace_bytes, key_off, path_off,
                                      key_out, key_cap, path_out, path_cap, key_state, 0u, stream);
}

extern "C" int avdb_primary_keys_fill_digests(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, size_t n,
                                              const char* digest, const uint64_t* key_off, uint8_t* key_out,
                                              uint8_t* key_state, void* stream) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !digest || !key_off || !key_out || !key_state) {
    avdb_set_error("avdb_primary_keys_fill_digests: null array");
    return AVDB_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(digest) % 16 || reinterpret_cast<uintptr_t>(key_state) % 16) {
    avdb_set_error("avdb_primary_keys_fill_digests: digest and key_state must be 16-byte aligned");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_fill_digests, dim3(stream_grid((n + 15) / 16, kBlock, 2048)), dim3(kBlock), 0, s, chrom, pos,
                     n, digest, key_off, key_out, key_state);
  AVDB_LAUNCH_CHECK("k_fill_digests");
  return AVDB_OK;
}

// ---- the keyed one-pass prep (K2 + K7 in one launch) ------------------------------
static size_t onepass_groups(size_t n) { return (n + kOpGroupRecs - 1) / kOpGroupRecs; }

namespace avdb {
// K3's list layout under avdb_keyed_prep: `grid` slices of `slice` entries (group g
// lists into slice g % grid; every slice holds at most ceil(groups / grid) groups)
void keyed_onepass_dd_layout(size_t n, unsigned* grid, size_t* slice) {
  const size_t ng = onepass_groups(n);
  const size_t sl = ng < kOpSlicesMax ? (ng ? ng : 1) : kOpSlicesMax;
  *grid = unsigned(sl);
  *slice = ((ng + sl - 1) / sl) * kOpGroupRecs;
}
}  // namespace avdb

extern "C" int avdb_keyed_prep_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  const size_t ng = onepass_groups(n);
  *bytes = 256 + 16 * ng + 32 * ng;  // header | look-back granules (2 x u64) | group statistics (2 x uint4)
  return AVDB_OK;
}

extern "C" int avdb_keyed_prep(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                               const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap,
                               size_t heap_bytes, const uint64_t* ext_id, size_t n, uint32_t max_seq_len,
                               uint32_t* end_out, uint32_t* bin_code, uint8_t* status, uint32_t* hist_l8,
                               uint64_t* counters, void* workspace, size_t workspace_bytes, void* digest_workspace,
                               size_t digest_workspace_bytes, void* dedup_workspace, size_t dedup_workspace_bytes,
                               uint8_t* keep, uint64_t* key_off, uint64_t* path_off, uint8_t* key_out,
                               size_t key_cap, uint8_t* path_out, size_t path_cap, uint8_t* key_state,
                               uint32_t flags, int* written, void* stream) {
  if (!ctx || !written || !end_out || !bin_code || !key_off || !key_out || !key_state || (path_out && !path_off)) {
    avdb_set_error("avdb_keyed_prep: null argument");
    return AVDB_EINVAL;
  }
  *written = 0;
  if (flags & ~uint32_t(AVDB_KEYS_DIGEST_DEFERRED)) {
    avdb_set_error("avdb_keyed_prep: unknown flags 0x%x", flags);
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n == 0) {
    AVDB_HIP_TRY(hipMemsetAsync(key_off, 0, 8, s));
    if (path_out) AVDB_HIP_TRY(hipMemsetAsync(path_off, 0, 8, s));
    return AVDB_OK;
  }
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap) {
    avdb_set_error("avdb_keyed_prep: null array");
    return AVDB_EINVAL;
  }
  if (n >= (size_t(1) << 32)) {
    avdb_set_error("avdb_keyed_prep: n must be < 2^32");
    return AVDB_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(key_out) % 8 || (path_out && reinterpret_cast<uintptr_t>(path_out) % 8)) {
    avdb_set_error("avdb_keyed_prep: text outputs must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_keyed_prep_workspace_size(n, &need);
  if (!workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(workspace) % 16) {
    avdb_set_error("avdb_keyed_prep: 16-byte aligned workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  const size_t ng = onepass_groups(n);
  char* w = static_cast<char*>(workspace);
  PrepArgs P;
  memset(&P, 0, sizeof(P));
  P.end = end_out;
  P.code = bin_code;
  P.status = status;
  P.hdr = reinterpret_cast<uint32_t*>(w);
  P.lb = reinterpret_cast<unsigned long long*>(w + 256);
  P.grp_stat = (hist_l8 || counters) ? reinterpret_cast<uint4*>(w + 256 + 16 * ng) : nullptr;
  P.hist = hist_l8;
  P.n_groups = ng;
  P.max_seq_len = max_seq_len;
  if (digest_workspace) {
    size_t dneed = 0;
    avdb_vrs_digest_workspace_size(n, &dneed);
    if (digest_workspace_bytes < dneed || reinterpret_cast<uintptr_t>(digest_workspace) % 16) {
      avdb_set_error("avdb_keyed_prep: 16-byte aligned K4 workspace of %zu bytes required", dneed);
      return AVDB_ERANGE;
    }
    P.long_codes = vrs_long_codes_of(digest_workspace, n);
  }
  unsigned slices = 0;
  size_t slice = 0;
  keyed_onepass_dd_layout(n, &slices, &slice);
  P.dd_slices = 1;
  P.dd_counts = P.hdr + 2;  // (no marks: a dummy counter nobody reads)
  if (dedup_workspace && keep) {
    if (dedup_workspace_bytes < kDedupListHead + 4 * size_t(slices) * slice ||
        reinterpret_cast<uintptr_t>(dedup_workspace) % 16) {
      avdb_set_error("avdb_keyed_prep: 16-byte aligned K3 list workspace of %zu bytes required",
                     kDedupListHead + 4 * size_t(slices) * slice);
      return AVDB_ERANGE;
    }
    P.keep = keep;
    P.dd_counts = static_cast<uint32_t*>(dedup_workspace);
    P.dd_list = reinterpret_cast<uint32_t*>(static_cast<char*>(dedup_workspace) + kDedupListHead);
    P.dd_slice = slice;
    P.dd_slices = slices;
  }
  KeyArgs A = key_args(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, ext_id,
                       path_out ? bin_code : nullptr, nullptr, n, max_seq_len, key_off, path_off, key_out, key_cap,
                       path_out, path_cap, key_state);
  A.defer = (flags & AVDB_KEYS_DIGEST_DEFERRED) ? 1u : 0u;
  hipLaunchKernelGGL(k_keyed_init, dim3(stream_grid(2 * ng, kBlock, 1024)), dim3(kBlock), 0, s, P);
  AVDB_LAUNCH_CHECK("k_keyed_init");
  if (ng > 0xFFFFFFFFull) {
    avdb_set_error("avdb_keyed_prep: too many groups");
    return AVDB_EINVAL;
  }
  hipLaunchKernelGGL(k_keyed_onepass<kOpTpw>, dim3(unsigned(ng)), dim3(kOpBlock), 0, s, A, P, ctx->tab);
  AVDB_LAUNCH_CHECK("k_keyed_onepass");
  if (P.grp_stat) {
    const size_t threads = (ng + kStatGroups - 1) / kStatGroups;
    hipLaunchKernelGGL(k_keyed_stats, dim3(unsigned((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       P.grp_stat, ng, n, hist_l8, reinterpret_cast<unsigned long long*>(counters));
    AVDB_LAUNCH_CHECK("k_keyed_stats");
  }
  *written = (P.long_codes ? AVDB_KEYED_LONG_CODES : 0) | (P.keep ? AVDB_KEYED_DEDUP_MARKS : 0);
  return AVDB_OK;
}

extern "C" int avdb_keyed_prep_lookback_errors(avdb_ctx* ctx, const void* workspace, uint32_t* out) {
  if (!ctx || !workspace || !out) return AVDB_EINVAL;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  AVDB_HIP_TRY(hipMemcpy(out, static_cast<const uint32_t*>(workspace) + 1, 4, hipMemcpyDeviceToHost));
  return AVDB_OK;
}

extern "C" int avdb_keys_off32_bytes(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = off32_bytes(n);
  return AVDB_OK;
}
