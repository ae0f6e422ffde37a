// Internal declarations shared by the libavdb_hip translation units.
// gfx950 (CDNA4) only: wave64, 160 KiB LDS per CU, 256 CUs in 8 XCDs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/avdb.h"

namespace avdb {

// Record arithmetic shared by the kernels and the library's per-call host path
// (avdb_small_prep_host): one definition, compiled for both sides.
#define AVDB_HD __host__ __device__ __forceinline__

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr int kBlock = 256;               // 4 waves per workgroup
constexpr uint32_t kLeafWidth = 15625;    // L13 bin width, generate_bin_index_references.py:93
constexpr uint32_t kL8Width = 500000;     // L8 bin width (histogram granularity)
constexpr int kMaxLdsHistBins = 16384;    // 64 KiB LDS histogram; larger tables go straight to HBM

// Chromosome table passed BY VALUE as a kernel argument (lands in SGPRs /
// the kernarg segment); each workgroup stages the part it indexes per lane
// into LDS.  This is all of BinIndexRef the closed form needs: per-contig
// length (generate_bin_index_references.py:17-25,62-65) plus the prefix sum
// of L8 bins used by the histogram.
struct ChromTable {
  uint32_t len[AVDB_MAX_CHROM];
  uint32_t l8_off[AVDB_MAX_CHROM];
  int32_t n;
  uint32_t n_l8;
};

// smallest enclosing bin of the closed interval [lo, hi], 1 <= lo <= hi.
// Level = largest l in 1..13 with (lo-1)/w_l == (hi-1)/w_l, w_l = 15625<<(13-l),
// else 0 (whole chromosome) — BinIndexRef's nested (lo,hi] rows.
AVDB_HD uint32_t bin_code_closed(uint32_t lo, uint32_t hi) {
  const uint32_t qs = (lo - 1u) / kLeafWidth;   // magic-multiply, no divide
  const uint32_t qe = (hi - 1u) / kLeafWidth;
  const uint32_t x = qs ^ qe;
  const int blen = x ? 32 - __builtin_clz(x) : 0;
  const int level = blen <= 12 ? 13 - blen : 0;
  const uint32_t idx = level ? (qs >> (13 - level)) : 0u;
  return (uint32_t(level) << 28) | idx;
}

// Full classification of one record against the staged length table.
// Returns the status; writes code (AVDB_BIN_NONE when unmappable).
AVDB_HD uint32_t classify(uint32_t c, uint32_t s, uint32_t e, int n_chrom,
                                             const uint32_t* __restrict__ s_len, uint32_t* code) {
  if (c >= uint32_t(n_chrom)) { *code = AVDB_BIN_NONE; return AVDB_STATUS_UNKNOWN_CHROM; }
  uint32_t st = AVDB_STATUS_OK;
  uint32_t lo = s, hi = e;
  if (e < s) { lo = e; hi = s; st = AVDB_STATUS_END_BEFORE_START; }
  const uint32_t L = s_len[c];
  if (lo < 1u || hi > L) { *code = AVDB_BIN_NONE; return AVDB_STATUS_OUT_OF_RANGE; }
  *code = bin_code_closed(lo, hi);
  return st;
}

// ---- allele heap access ----------------------------------------------------
// Allele bytes are read as naturally aligned 8-byte words (one global_load_dwordx2
// per 8 bytes instead of 8 byte loads) and funnel-shifted into place; words
// straddling either end of the heap allocation are assembled bytewise, so no
// access ever leaves [heap, heap + heap_bytes).
struct Heap {
  uintptr_t lo, hi;
};

AVDB_HD Heap make_heap(const uint8_t* p, size_t bytes) {
  return Heap{reinterpret_cast<uintptr_t>(p), reinterpret_cast<uintptr_t>(p) + bytes};
}

// A device load from an integer address goes through a global-address-space
// pointer: a generic pointer made from an integer is a FLAT access, which counts on
// both vmcnt and lgkmcnt and retires out of order, so every use of its result
// waits vmcnt(0) + lgkmcnt(0) — behind every older store and LDS operation.
#if defined(__HIP_DEVICE_COMPILE__)
#define AVDB_GLOBAL __attribute__((address_space(1)))
#else
#define AVDB_GLOBAL
#endif
template <class T>
AVDB_HD const AVDB_GLOBAL T* gptr(uintptr_t a) {
  return reinterpret_cast<const AVDB_GLOBAL T*>(a);
}

AVDB_HD uint64_t heap_word(uintptr_t a, const Heap& h) {  // a 8-aligned
  if (a >= h.lo && a + 8 <= h.hi) return *gptr<uint64_t>(a);
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) {
    const uintptr_t b = a + k;
    if (b >= h.lo && b < h.hi) v |= uint64_t(*gptr<uint8_t>(b)) << (8 * k);
  }
  return v;
}

// One unaligned 8-byte global load (global_load_dwordx2: gfx950 runs in
// unaligned-access mode, and the compiler emits it for a packed struct).
struct __attribute__((packed)) U64u {
  uint64_t v;
};
typedef const __attribute__((address_space(1))) U64u* g_u64u;
struct __attribute__((packed)) U32u {
  uint32_t v;
};
struct __attribute__((packed)) U16u {
  uint16_t v;
};

// little-endian 8 bytes starting at heap offset p (bytes past the heap read 0)
AVDB_HD uint64_t heap_u64(const Heap& h, uint64_t p) {
  const uintptr_t addr = h.lo + p;
#if defined(__HIP_DEVICE_COMPILE__)
  if (addr + 8 <= h.hi) return reinterpret_cast<g_u64u>(addr)->v;
#else
  if (addr + 8 <= h.hi) return reinterpret_cast<const U64u*>(addr)->v;
#endif
  // within 8 bytes of the heap end: aligned words, zero fill
  const uintptr_t a = addr & ~uintptr_t(7);
  const uint32_t sh = uint32_t(addr & 7) * 8;
  const uint64_t lo = heap_word(a, h);
  if (!sh) return lo;
  const uint64_t hi = heap_word(a + 8, h);
  return (lo >> sh) | (hi << (64 - sh));
}

AVDB_HD uint64_t low_bytes_mask(uint32_t k) {  // k in 0..8
  return k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1);
}

// byte-exact equality of L bytes at heap offsets p and q
AVDB_HD bool heap_equal(const Heap& h, uint64_t p, uint64_t q, uint32_t L) {
  if (p == q) return true;
  for (uint32_t k = 0; k < L; k += 8) {
    const uint64_t m = low_bytes_mask(L - k);
    if ((heap_u64(h, p + k) ^ heap_u64(h, q + k)) & m) return false;
  }
  return true;
}

// ---- K2 end inference (shared by K2 and the small-batch kernel K8) ---------
// variant_annotator.py:36-79 with lcp from __normalize_alleles (:82-121).
// Allele bytes are compared 8 at a time (first mismatch via count-trailing-zeros
// of the XOR); the inversion test reverses 8-byte chunks with a byte swap.
// wr / wa are the first 8 bytes of ref / alt, loaded by the caller ahead of
// time; alleles of up to 8 bytes (the bulk) need no further heap reads.
AVDB_HD uint32_t infer_end(const Heap& h, uint64_t off, uint32_t r, uint32_t a,
                                              uint32_t pos, uint64_t wr, uint64_t wa,
                                              uint32_t* lcp_out) {
  if (r == 1u && a == 1u) { *lcp_out = 0; return pos; }        // SNV (:54-55)
  const uint64_t alt = off + r;
  const uint32_t m = r < a ? r : a;
  uint32_t n;                                                  // lcp (:100-108)
  const uint64_t x0 = (wr ^ wa) & low_bytes_mask(m < 8u ? m : 8u);
  if (x0) {
    n = uint32_t(__builtin_ctzll(x0)) >> 3;
  } else if (m <= 8u) {
    n = m;
  } else {
    n = 8;
    while (n < m) {
      const uint64_t x = (heap_u64(h, off + n) ^ heap_u64(h, alt + n)) & low_bytes_mask(m - n);
      if (x) { n += uint32_t(__builtin_ctzll(x)) >> 3; break; }
      n += 8;
    }
    if (n > m) n = m;
  }
  *lcp_out = n;
  const uint32_t nr = r - n, na = a - n;
  if (r == a) {                                                // MNV (:57-65)
    bool inv = true;                                           // ref == alt[::-1]
    if (r <= 8u) {
      if (r) {
        const uint64_t mk = low_bytes_mask(r);
        inv = (wr & mk) == (__builtin_bswap64(wa & mk) >> (8 * (8 - r)));
      }
    } else {
      for (uint32_t i = 0; i < r && inv; i += 8) {
        const uint32_t c = r - i < 8 ? r - i : 8;
        const uint64_t mk = low_bytes_mask(c);
        const uint64_t fw = heap_u64(h, off + i) & mk;
        const uint64_t bw = __builtin_bswap64(heap_u64(h, alt + (r - i - c)) & mk) >> (8 * (8 - c));
        inv = fw == bw;
      }
    }
    return inv ? pos + r - 1u : pos + nr - 1u;
  }
  if (na >= 1u)                                                // insertion (:67-74)
    return nr >= 1u ? pos + nr : (r > 1u ? pos + r - 1u : pos + 1u);
  return nr == 0u ? pos + r - 1u : pos + nr;                   // deletion (:77-79)
}


// ---- status counters ------------------------------------------------------
// Only error statuses (1..3) are counted per lane, in 8-bit fields of one u32;
// the OK count is records - errors, so the common path costs nothing.
__device__ __forceinline__ void flush_errors(uint32_t& err, unsigned long long* s_ctr) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint32_t a = (err >> (8 * k)) & 0xFFu;
    if (a) atomicAdd(&s_ctr[AVDB_CTR_STATUS0 + 1 + k], (unsigned long long)a);
  }
  err = 0;
}

struct ErrCounters {
  uint32_t err = 0, nrec = 0;
  int since = 0;
  __device__ __forceinline__ void add(uint32_t status) {
    ++nrec;
    err += status ? (1u << (8 * (status - 1))) : 0u;
  }
  // call once per record-slot pass by every lane of the workgroup
  __device__ __forceinline__ void tick(unsigned long long* s_ctr) {
    if (++since == 255) { flush_errors(err, s_ctr); since = 0; }
  }
  // workgroup epilogue: records + derived OK count into s_ctr (before publish)
  __device__ __forceinline__ void finish(unsigned long long* s_ctr) {
    flush_errors(err, s_ctr);
    for (int d = 32; d > 0; d >>= 1) nrec += __shfl_down(nrec, d, 64);
    if (__lane_id() == 0 && nrec) atomicAdd(&s_ctr[AVDB_CTR_RECORDS], (unsigned long long)nrec);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long bad = s_ctr[AVDB_CTR_STATUS0 + 1] + s_ctr[AVDB_CTR_STATUS0 + 2] +
                                     s_ctr[AVDB_CTR_STATUS0 + 3];
      s_ctr[AVDB_CTR_STATUS0] = s_ctr[AVDB_CTR_RECORDS] - bad;
    }
  }
};

// ---- wave-aggregated histogram add --------------------------------------
// Adds 1 to hist[key] for every active lane with key != ~0u.  Position-sorted
// input gives runs of equal keys in consecutive lanes: only the head lane of
// each run issues the (LDS or HBM) atomic, with the run length.  The whole
// wave must call it (ballots).
__device__ __forceinline__ void wave_hist_add(uint32_t key, uint32_t* hist) {
  const int lane = __lane_id();
  const uint32_t prev = __shfl_up(key, 1, kWave);
  const bool valid = key != 0xFFFFFFFFu;
  const bool head = valid && (lane == 0 || prev != key);
  // a run ends at the next lane whose key differs (head or invalid)
  const uint64_t breaks = __ballot(!valid || lane == 0 || prev != key);
  if (head) {
    const uint64_t above = (lane == 63) ? 0ull : (breaks >> (lane + 1)) << (lane + 1);
    const int next = above ? __ffsll((unsigned long long)above) - 1 : kWave;
    atomicAdd(&hist[key], uint32_t(next - lane));
  }
}

// ---- K4's long-record bucket code (shared by K4 and the keyed K2) ----------
// 0: short (ref + alt <= max_len, keyed by its alleles); else 1 + the record's
// bucket = the SHA-512 block count of its VRS Allele message (68 bytes before
// the ALT, 54 after; avdb_digest.hip), the last bucket taking the rest
constexpr int kLongBuckets = 32;
constexpr uint32_t kVrsAlleleFixedBytes = 68 + 54;
__device__ __forceinline__ uint32_t long_bucket(uint32_t a) {
  const uint32_t nb = uint32_t((uint64_t(kVrsAlleleFixedBytes) + a + 17 + 127) / 128);
  return nb < uint32_t(kLongBuckets) ? nb : uint32_t(kLongBuckets) - 1;
}
__device__ __forceinline__ uint32_t long_code(uint32_t r, uint32_t a, uint32_t max_len) {
  return uint64_t(r) + a > max_len ? 1u + long_bucket(a) : 0u;
}

// inclusive wave64 prefix sum through DPP row shifts and row broadcasts: six
// VALU adds with no LDS round trip (__shfl_up lowers to ds_bpermute: six
// dependent LDS trips per value)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
  return x;
}

}  // namespace avdb

struct avdb_ctx {
  int device;
  int n_cu;            // compute units on the device (256 on MI355X)
  int k1_blocks_per_cu;  // K1 grid = n_cu * k1_blocks_per_cu workgroups (env AVDB_K1_BLOCKS_PER_CU)
  int k2_blocks_per_cu;  // K2 grid = n_cu * this (env AVDB_K2_BLOCKS_PER_CU)
  int k4_blocks_per_cu;  // K4 digest grid = n_cu * this (env AVDB_K4_BLOCKS_PER_CU; default: its occupancy, 3)
  int k4_grid;           // K4 digest grid in workgroups when > 0 (avdb_ctx_set_option AVDB_OPT_K4_GRID)
  int k7_grid;           // K7 write-pass workgroups when > 0 (avdb_ctx_set_option AVDB_OPT_K7_GRID)
  size_t k7_raw_blocks;  // K7 one-pass: write pass sums up to this many block totals itself (env AVDB_K7_RAW_BLOCKS)
  avdb::ChromTable tab;
  char* d_seq_digest;  // device copy of the refget digests (n * 32 chars), or null
  uint64_t* d_loc_tail;  // K4: block 1 of each contig's SequenceLocation message per digit count (avdb_digest.hip)
  bool has_digests;
};

void avdb_set_error(const char* fmt, ...);

#include <vector>
namespace avdb {
// workspace bytes K7's size pass needs for n records (u16 sizes + their scan)
size_t key_size_workspace(size_t n);
// K7 one-pass workspace: group totals the keyed K2 fills (avdb_keys.hip)
uint32_t key_totals_group_log2(size_t n);
uint2* key_totals_of(void* workspace);
// K3 list-form workspace: per-workgroup suspect counts, then the suspect list
constexpr size_t kDedupListHead = 16384;
constexpr unsigned kDedupMaxGroups = kDedupListHead / 4;
// the keyed K2's workgroups and the records each may list as suspects (one slice
// of the K3 list per workgroup; avdb_bins.hip), for K3's resolve over them
void keyed_prep_layout(const avdb_ctx* ctx, size_t n, unsigned* grid, size_t* slice);
// K3's list layout under the one-pass keyed prep (avdb_keyed_prep, avdb_keys.hip)
void keyed_onepass_dd_layout(size_t n, unsigned* grid, size_t* slice);
// K4 workspace: the per-record bucket codes the keyed K2 fills (avdb_digest.hip)
uint8_t* vrs_long_codes_of(void* workspace, size_t n);
// K4's per-(contig, digit count) SequenceLocation block-1 table (host)
void location_tail_table(const char* digests, int n_chrom, std::vector<uint64_t>& out);
}  // namespace avdb

#define AVDB_HIP_TRY(expr)                                                         \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      avdb_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                     __LINE__);                                                    \
      return AVDB_EHIP;                                                            \
    }                                                                              \
  } while (0)

#define AVDB_LAUNCH_CHECK(name)                                                    \
  do {                                                                             \
    hipError_t _e = hipGetLastError();                                             \
    if (_e != hipSuccess) {                                                        \
      avdb_set_error("launch of %s failed: %s", name, hipGetErrorString(_e));      \
      return AVDB_EHIP;                                                            \
    }                                                                              \
  } while (0)

// grid size for a streaming kernel: enough workgroups to fill 256 CUs at the
// occupancy the kernel reaches, capped so each workgroup owns a contiguous
// chunk (keeps a sorted batch's histogram keys local to one workgroup).
static inline unsigned stream_grid(size_t work_items, unsigned per_block, unsigned cap = 2048) {
  size_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return unsigned(g);
}
