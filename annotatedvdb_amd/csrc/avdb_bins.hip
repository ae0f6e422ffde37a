// K1 bin_assign and K2 record_prep — gfx950.
//
// K1 replaces BinIndex.find_bin_index (BinIndex/lib/python/bin_index.py:59-75)
// and the SQL find_bin_index it reaches through BIN_INDEX_SQL (:9-14): the
// deepest BinIndexRef row (generate_bin_index_references.py:46-83) whose
// (lo,hi] holds the closed interval [start,end].  The table is nested and
// aligned, so the search is closed-form integer arithmetic: two magic-multiply
// divisions by 15,625, an XOR and a count-leading-zeros.
//
// K2 fuses the per-alt end inference (variant_annotator.py:36-121) in front of
// the same bin computation (vcf_variant_loader.py:309-311).
//
// Both are HBM-streaming kernels (9-13 algorithmic bytes per record for K1):
// coalesced 16-B-per-lane loads/stores, a block-contiguous partition of the
// batch (so a position-sorted batch hits a narrow, LDS-resident slice of the
// histogram), per-contig lengths and L8 offsets staged in LDS, and
// wave-ballot run aggregation for the histogram atomics.
#include "avdb_fmt.hpp"  // K7 key / path sizes for the keyed K2

namespace avdb {

// stage the per-lane-indexed part of the chromosome table + zero LDS state
__device__ __forceinline__ void stage_table(const ChromTable& tab, uint32_t* s_len, uint32_t* s_l8off,
                                            unsigned long long* s_ctr, uint32_t* s_hist,
                                            bool lds_hist) {
  const int t = threadIdx.x;
  if (t < AVDB_MAX_CHROM) {
    s_len[t] = tab.len[t];
    s_l8off[t] = tab.l8_off[t];
  }
  if (t < AVDB_N_COUNTERS) s_ctr[t] = 0;
  if (lds_hist)
    for (uint32_t b = t; b < tab.n_l8; b += blockDim.x) s_hist[b] = 0;
  __syncthreads();
}

__device__ __forceinline__ void publish(const ChromTable& tab, const unsigned long long* s_ctr,
                                        const uint32_t* s_hist, bool lds_hist, bool hist,
                                        uint32_t* __restrict__ g_hist,
                                        unsigned long long* __restrict__ g_ctr) {
  __syncthreads();
  const int t = threadIdx.x;
  if (g_ctr && t < AVDB_N_COUNTERS && s_ctr[t]) atomicAdd(&g_ctr[t], s_ctr[t]);
  if (hist && lds_hist)
    for (uint32_t b = t; b < tab.n_l8; b += blockDim.x)
      if (s_hist[b]) atomicAdd(&g_hist[b], s_hist[b]);
}

__device__ __forceinline__ uint32_t l8_key(uint32_t c, uint32_t s, uint32_t code,
                                           const uint32_t* s_l8off) {
  return code == AVDB_BIN_NONE ? 0xFFFFFFFFu : s_l8off[c] + (s - 1u) / kL8Width;
}

// ---------------------------------------------------------------------------
// K1, vector form: 4 records per lane-group (u32 of chrom codes, uint4 of
// starts/ends/codes), UNROLL groups in flight per lane.
// ---------------------------------------------------------------------------
// FLAGS bit0: plain (not nontemporal) loads; bit1: plain stores
template <int FLAGS, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (FLAGS & 1) return *p;
  else return __builtin_nontemporal_load(p);
}
template <int FLAGS, typename T>
__device__ __forceinline__ void st_(T v, T* p) {
  if constexpr (FLAGS & 2) *p = v;
  else __builtin_nontemporal_store(v, p);
}

constexpr int kK1Block = 512;  // 8 waves: one LDS histogram per 8 waves
constexpr int kK2Unroll = 2;       // plain K2: groups of 4 records per lane per trip
constexpr int kK2KeyedUnroll = 1;  // the keyed K2 (144 VGPRs at 2)

// chrom codes of one lane-group: V u32 words (4 codes each)
template <int V> struct ChromVec;
template <> struct ChromVec<1> { typedef uint32_t T; };
template <> struct ChromVec<2> { typedef uint32_t T __attribute__((ext_vector_type(2))); };
template <> struct ChromVec<4> { typedef u32x4 T; };

template <int V>
__device__ __forceinline__ uint32_t vec_word(const typename ChromVec<V>::T& x, int v) {
  if constexpr (V == 1) return x;
  else return x[v];
}

// V: u32x4 start vectors per lane-group (4V records per lane per step)
template <bool HAS_END, bool HIST, int V, int UNROLL, int FLAGS>
__global__ __launch_bounds__(kK1Block) void k_bin_assign4(
    const typename ChromVec<V>::T* __restrict__ chromv, const u32x4* __restrict__ start4,
    const u32x4* __restrict__ end4, size_t ngroups, u32x4* __restrict__ code4,
    typename ChromVec<V>::T* __restrict__ statusv, ChromTable tab, uint32_t* __restrict__ g_hist,
    unsigned long long* __restrict__ g_ctr, int lds_hist,
    // scalar tail [tail_begin, n): block 0, wave 0
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ start,
    const uint32_t* __restrict__ end, size_t tail_begin, size_t n,
    uint32_t* __restrict__ code, uint8_t* __restrict__ status) {
  typedef typename ChromVec<V>::T CT;
  extern __shared__ uint32_t s_hist[];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM];
  __shared__ uint32_t s_l8off[AVDB_MAX_CHROM];
  __shared__ unsigned long long s_ctr[AVDB_N_COUNTERS];
  const bool use_lds = HIST && lds_hist;
  stage_table(tab, s_len, s_l8off, s_ctr, s_hist, use_lds);
  uint32_t* hist = use_lds ? s_hist : g_hist;
  const bool ctrs = g_ctr != nullptr;
  const int n_chrom = tab.n;
  const uint32_t bdim = blockDim.x;
  constexpr int R = 4 * V;  // records per lane-group

  // FLAGS bit2: grid-stride sweep; otherwise each workgroup owns one
  // contiguous chunk (a sorted batch then touches a narrow histogram slice)
  size_t g0, g1, step;
  if (FLAGS & 4) {
    g0 = size_t(blockIdx.x) * bdim * UNROLL;
    g1 = ngroups;
    step = size_t(gridDim.x) * bdim * UNROLL;
  } else {
    const size_t per = (ngroups + gridDim.x - 1) / gridDim.x;
    g0 = size_t(blockIdx.x) * per;
    g1 = g0 + per < ngroups ? g0 + per : ngroups;
    step = size_t(bdim) * UNROLL;
  }

  // error statuses only (OK = records - errors): 8-bit fields for status 1..3
  uint32_t err = 0;
  uint32_t nrec = 0;
  int since_flush = 0;
  // wave-uniform run of histogram keys (sorted batches): one LDS atomic per run
  uint32_t run_key = 0xFFFFFFFFu, run_cnt = 0;
  for (size_t base = g0; base < g1; base += step) {
    CT c4[UNROLL];
    u32x4 s4[UNROLL][V], e4[UNROLL][V];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = base + size_t(u) * bdim + threadIdx.x;
      if (j < g1) {
        c4[u] = ld<FLAGS>(&chromv[j]);
#pragma unroll
        for (int v = 0; v < V; ++v) {
          s4[u][v] = ld<FLAGS>(&start4[size_t(V) * j + v]);
          if (HAS_END) e4[u][v] = ld<FLAGS>(&end4[size_t(V) * j + v]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = base + size_t(u) * bdim + threadIdx.x;
      const bool live = j < g1;
      uint32_t cv[R], key[R], stw[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const uint32_t cw = vec_word<V>(c4[u], v);
        uint32_t st = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t c = (cw >> (8 * k)) & 0xFFu;
          const uint32_t sv = s4[u][v][k];
          const uint32_t ev = HAS_END ? e4[u][v][k] : sv;
          const uint32_t s_k = classify(c, sv, ev, n_chrom, s_len, &cv[4 * v + k]);
          st |= s_k << (8 * k);
          key[4 * v + k] = live ? l8_key(c, sv, cv[4 * v + k], s_l8off) : 0xFFFFFFFFu;
        }
        stw[v] = st;
      }
      if (ctrs && live) {
        nrec += R;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if (stw[v]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t s_k = (stw[v] >> (8 * k)) & 0xFFu;
              err += s_k ? (1u << (8 * (s_k - 1))) : 0u;
            }
          }
        }
      }
      if (HIST) {
        // lane key: the group's common key, or MIXED; dead lanes match anything
        bool same = true;
#pragma unroll
        for (int k = 1; k < R; ++k) same = same && key[k] == key[0];
        const uint32_t lk = same ? key[0] : 0xFFFFFFFEu;
        const uint32_t first = __builtin_amdgcn_readfirstlane(lk);
        const uint64_t ok = __ballot(!live || lk == first);
        if (ok == ~0ull && first < 0xFFFFFFFEu) {
          const uint32_t cnt = uint32_t(R) * uint32_t(__popcll(__ballot(live)));
          if (first == run_key) {
            run_cnt += cnt;
          } else {
            if (run_cnt && __lane_id() == 0) atomicAdd(&hist[run_key], run_cnt);
            run_key = first;
            run_cnt = cnt;
          }
        } else if (!(ok == ~0ull && first == 0xFFFFFFFFu)) {
#pragma unroll
          for (int k = 0; k < R; ++k) wave_hist_add(key[k], hist);
        }
      }
      if (live) {
#pragma unroll
        for (int v = 0; v < V; ++v)
          st_<FLAGS>(u32x4{cv[4 * v], cv[4 * v + 1], cv[4 * v + 2], cv[4 * v + 3]},
                     &code4[size_t(V) * j + v]);
        if (statusv) {
          CT sw;
          if constexpr (V == 1) sw = stw[0];
          else {
#pragma unroll
            for (int v = 0; v < V; ++v) sw[v] = stw[v];
          }
          st_<FLAGS>(sw, &statusv[j]);
        }
      }
    }
    if (ctrs && ++since_flush == 255 / (UNROLL * R)) {  // 8-bit error fields never wrap
      flush_errors(err, s_ctr);
      since_flush = 0;
    }
  }
  if (HIST && run_cnt && __lane_id() == 0) atomicAdd(&hist[run_key], run_cnt);
  // scalar tail (< 4V records)
  if (blockIdx.x == 0 && threadIdx.x < kWave) {
    const size_t i = tail_begin + threadIdx.x;
    uint32_t key = 0xFFFFFFFFu;
    if (i < n) {
      const uint32_t c = chrom[i], s = start[i], e = HAS_END ? end[i] : s;
      uint32_t cv;
      const uint32_t s_k = classify(c, s, e, n_chrom, s_len, &cv);
      code[i] = cv;
      if (status) status[i] = uint8_t(s_k);
      nrec += 1;
      err += s_k ? (1u << (8 * (s_k - 1))) : 0u;
      key = l8_key(c, s, cv, s_l8off);
    }
    if (HIST) wave_hist_add(key, hist);
  }
  if (ctrs) {
    flush_errors(err, s_ctr);
    // records per workgroup: wave reduce, one LDS atomic per wave
    for (int d = 32; d > 0; d >>= 1) nrec += __shfl_down(nrec, d, kWave);
    if (__lane_id() == 0 && nrec) atomicAdd(&s_ctr[AVDB_CTR_RECORDS], (unsigned long long)nrec);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long bad = s_ctr[AVDB_CTR_STATUS0 + 1] + s_ctr[AVDB_CTR_STATUS0 + 2] +
                                     s_ctr[AVDB_CTR_STATUS0 + 3];
      s_ctr[AVDB_CTR_STATUS0] = s_ctr[AVDB_CTR_RECORDS] - bad;
    }
  }
  publish(tab, s_ctr, s_hist, use_lds, HIST, g_hist, g_ctr);
}

// K1, scalar form: any alignment, one record per lane.
template <bool HAS_END, bool HIST>
__global__ __launch_bounds__(kBlock) void k_bin_assign1(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ start,
    const uint32_t* __restrict__ end, size_t n, uint32_t* __restrict__ code,
    uint8_t* __restrict__ status, ChromTable tab, uint32_t* __restrict__ g_hist,
    unsigned long long* __restrict__ g_ctr, int lds_hist) {
  extern __shared__ uint32_t s_hist[];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM];
  __shared__ uint32_t s_l8off[AVDB_MAX_CHROM];
  __shared__ unsigned long long s_ctr[AVDB_N_COUNTERS];
  const bool use_lds = HIST && lds_hist;
  stage_table(tab, s_len, s_l8off, s_ctr, s_hist, use_lds);
  uint32_t* hist = use_lds ? s_hist : g_hist;
  const bool ctrs = g_ctr != nullptr;
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  ErrCounters ec;
  for (size_t base = i0; base < i1; base += kBlock) {
    const size_t i = base + threadIdx.x;
    uint32_t key = 0xFFFFFFFFu;
    if (i < i1) {
      const uint32_t c = chrom[i], s = start[i], e = HAS_END ? end[i] : s;
      uint32_t cv;
      const uint32_t s_k = classify(c, s, e, tab.n, s_len, &cv);
      code[i] = cv;
      if (status) status[i] = uint8_t(s_k);
      if (ctrs) ec.add(s_k);
      key = l8_key(c, s, cv, s_l8off);
    }
    if (HIST) wave_hist_add(key, hist);
    if (ctrs) ec.tick(s_ctr);
  }
  if (ctrs) ec.finish(s_ctr);
  publish(tab, s_ctr, s_hist, use_lds, HIST, g_hist, g_ctr);
}

// ---------------------------------------------------------------------------
// K2: end inference (+ common-prefix length) fused with the bin computation.
// ---------------------------------------------------------------------------
// Records per lane per pass: all their SoA loads, then all their first heap
// words, are issued before any is consumed (the heap reads depend on
// allele_off, so one record per lane leaves K2 latency-bound).
constexpr int kPrepU = 4;

template <bool HIST>
__global__ __launch_bounds__(kBlock) void k_record_prep(
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos,
    const uint64_t* __restrict__ allele_off, const uint32_t* __restrict__ ref_len,
    const uint32_t* __restrict__ alt_len, const uint8_t* __restrict__ heap, size_t heap_bytes,
    size_t n, uint32_t* __restrict__ end_out, uint32_t* __restrict__ code,
    uint8_t* __restrict__ status, uint32_t* __restrict__ lcp, ChromTable tab,
    uint32_t* __restrict__ g_hist, unsigned long long* __restrict__ g_ctr, int lds_hist) {
  const Heap hp = make_heap(heap, heap_bytes);
  extern __shared__ uint32_t s_hist[];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM];
  __shared__ uint32_t s_l8off[AVDB_MAX_CHROM];
  __shared__ unsigned long long s_ctr[AVDB_N_COUNTERS];
  const bool use_lds = HIST && lds_hist;
  stage_table(tab, s_len, s_l8off, s_ctr, s_hist, use_lds);
  uint32_t* hist = use_lds ? s_hist : g_hist;
  const bool ctrs = g_ctr != nullptr;
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t i0 = size_t(blockIdx.x) * per;
  const size_t i1 = i0 + per < n ? i0 + per : n;
  ErrCounters ec;
  for (size_t base = i0; base < i1; base += size_t(kBlock) * kPrepU) {
    uint32_t c[kPrepU], p[kPrepU], r[kPrepU], a[kPrepU];
    uint64_t off[kPrepU], wr[kPrepU], wa[kPrepU];
#pragma unroll
    for (int k = 0; k < kPrepU; ++k) {
      const size_t i = base + size_t(k) * kBlock + threadIdx.x;
      const size_t j = i < i1 ? i : i0;  // clamped: every lane loads in bounds
      c[k] = chrom[j];
      p[k] = pos[j];
      off[k] = allele_off[j];
      r[k] = ref_len[j];
      a[k] = alt_len[j];
    }
#pragma unroll
    for (int k = 0; k < kPrepU; ++k) {
      const bool snv = r[k] == 1u && a[k] == 1u;
      wr[k] = snv ? 0 : heap_u64(hp, off[k]);
      wa[k] = snv ? 0 : heap_u64(hp, off[k] + r[k]);
    }
#pragma unroll
    for (int k = 0; k < kPrepU; ++k) {
      const size_t i = base + size_t(k) * kBlock + threadIdx.x;
      uint32_t key = 0xFFFFFFFFu;
      if (i < i1) {
        uint32_t l;
        const uint32_t e = infer_end(hp, off[k], r[k], a[k], p[k], wr[k], wa[k], &l);
        uint32_t cv;
        const uint32_t s_k = classify(c[k], p[k], e, tab.n, s_len, &cv);
        end_out[i] = e;
        code[i] = cv;
        if (status) status[i] = uint8_t(s_k);
        if (lcp) lcp[i] = l;
        if (ctrs) ec.add(s_k);
        key = l8_key(c[k], p[k], cv, s_l8off);
      }
      if (HIST) wave_hist_add(key, hist);
      if (ctrs) ec.tick(s_ctr);
    }
  }
  if (ctrs) ec.finish(s_ctr);
  publish(tab, s_ctr, s_hist, use_lds, HIST, g_hist, g_ctr);
}

// K2, vector form (K1's memory discipline): each lane takes 4 consecutive
// records per group through 16-byte loads (chrom as one u32 of 4 codes, pos /
// ref_len / alt_len as u32x4, allele_off as two u64x2), UNROLL groups in flight;
// then all heap peeks of its non-SNV records are issued before any is used;
// end / code leave as u32x4 stores, status as one u32.  Consecutive lanes hold
// consecutive records, so a wave's heap peeks fall in one contiguous stretch of
// the heap.  Grid-stride over a resident grid, as K1.

// The keyed form (KEYS, avdb_record_prep_keyed) also gives K7 its group totals:
// a wave's 64 lanes x 4 records per step are exactly one of K7's 256-record scan
// groups, so the key / path sizes of its records (the SoA is in registers; only
// the refSNP ids are read in addition) are summed over the wave and stored as
// that group's totals — K7's own totals pass re-read 25 B per record.
struct KeyTotals {
  const u64x2* ext2;    // refSNP keys, 2 per u64x2 (nullable: none)
  uint2* tot;           // K7 group totals (avdb::key_totals_of(workspace))
  uint32_t max_seq_len;
  uint32_t n_key_chrom; // labelled contigs
  uint32_t has_digest, with_paths;
  uint32_t group_log2;  // K7's groups: 64 << group_log2 records (0: 16 lanes' records, 2: the wave's)
  uint8_t* long_codes;  // nullable: K4's long_code per record (avdb::vrs_long_codes_of(digest workspace))
  // nullable: K3's first phase (k_dedup_mark4) — keep = 1 for every record and the
  // records sharing their predecessor's (chrom, pos), listed in this workgroup's
  // slice of dd_list (dd_slice entries), their count in dd_counts[workgroup]
  uint8_t* keep;
  uint32_t* dd_counts;
  uint32_t* dd_list;
  size_t dd_slice;
};

// KEYS: 0 plain; 1 keyed; 2 keyed with registers for 6 waves per SIMD — for
// batches whose K7 groups are 64 records (below 4 Mi records), where the launch is
// one generation of workgroups only if 3 fit per CU (C1: 0.110 -> 0.107 ms); at
// C4k's size the unconstrained form is faster (record prep 1.19 vs 1.25 ms)
// (the keyed form's occupancy pinned to 5 / 6 waves: 1.25 / 1.51 ms against 1.25;
// profiles/c4k_ab/r05_occupancy_ab.log)
template <bool HIST, int UNROLL, int KEYS = 0>
__global__ __launch_bounds__(kK1Block, KEYS == 2 ? 6 : 1) void k_record_prep4(
    const uint32_t* __restrict__ chromv, const u32x4* __restrict__ pos4, const u64x2* __restrict__ off2,
    const u32x4* __restrict__ rl4, const u32x4* __restrict__ al4, const uint8_t* __restrict__ heap,
    size_t heap_bytes, size_t ngroups, u32x4* __restrict__ end4, u32x4* __restrict__ code4,
    uint32_t* __restrict__ statusv, u32x4* __restrict__ lcp4, ChromTable tab, uint32_t* __restrict__ g_hist,
    unsigned long long* __restrict__ g_ctr, int lds_hist, KeyTotals kt,
    // scalar tail [tail_begin, n): block 0, wave 0
    const uint8_t* __restrict__ chrom, const uint32_t* __restrict__ pos, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ rl, const uint32_t* __restrict__ al, size_t tail_begin, size_t n,
    uint32_t* __restrict__ end_out, uint32_t* __restrict__ code, uint8_t* __restrict__ status,
    uint32_t* __restrict__ lcp) {
  const Heap hp = make_heap(heap, heap_bytes);
  extern __shared__ uint32_t s_hist[];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM];
  __shared__ uint32_t s_l8off[AVDB_MAX_CHROM];
  __shared__ unsigned long long s_ctr[AVDB_N_COUNTERS];
  __shared__ uint32_t s_dd;  // KEYS with dd_list: suspects this workgroup listed
  if (threadIdx.x == 0) s_dd = 0;
  const bool use_lds = HIST && lds_hist;
  stage_table(tab, s_len, s_l8off, s_ctr, s_hist, use_lds);
  uint32_t* hist = use_lds ? s_hist : g_hist;
  const bool ctrs = g_ctr != nullptr;
  const int n_chrom = tab.n;
  const size_t bdim = blockDim.x;
  uint32_t* dd_mine = (KEYS != 0 && kt.dd_list) ? kt.dd_list + size_t(blockIdx.x) * kt.dd_slice : nullptr;
  uint32_t err = 0, nrec = 0;
  int since_flush = 0;
  uint32_t run_key = 0xFFFFFFFFu, run_cnt = 0;
  for (size_t base = size_t(blockIdx.x) * bdim * UNROLL; base < ngroups; base += size_t(gridDim.x) * bdim * UNROLL) {
    uint32_t cw[UNROLL];
    u32x4 p4[UNROLL], r4[UNROLL], a4[UNROLL];
    u64x2 o01[UNROLL], o23[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = base + size_t(u) * bdim + threadIdx.x;
      const size_t jj = j < ngroups ? j : 0;  // clamped: every lane loads in bounds
      cw[u] = __builtin_nontemporal_load(&chromv[jj]);
      p4[u] = __builtin_nontemporal_load(&pos4[jj]);
      o01[u] = __builtin_nontemporal_load(&off2[2 * jj]);
      o23[u] = __builtin_nontemporal_load(&off2[2 * jj + 1]);
      r4[u] = __builtin_nontemporal_load(&rl4[jj]);
      a4[u] = __builtin_nontemporal_load(&al4[jj]);
    }
    u64x2 x01[UNROLL], x23[UNROLL];  // KEYS: refSNP keys
    if constexpr (KEYS != 0) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const size_t j = base + size_t(u) * bdim + threadIdx.x;
        const size_t jj = j < ngroups ? j : 0;
        x01[u] = kt.ext2 ? __builtin_nontemporal_load(&kt.ext2[2 * jj]) : u64x2{0, 0};
        x23[u] = kt.ext2 ? __builtin_nontemporal_load(&kt.ext2[2 * jj + 1]) : u64x2{0, 0};
      }
    }
    // first 8 bytes of ref and alt of every non-SNV record, all issued first
    uint64_t wr[UNROLL][4], wa[UNROLL][4];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = k < 2 ? o01[u][k] : o23[u][k - 2];
        const bool snv = r4[u][k] == 1u && a4[u][k] == 1u;
        wr[u][k] = snv ? 0 : heap_u64(hp, o);
        wa[u][k] = snv ? 0 : heap_u64(hp, o + r4[u][k]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = base + size_t(u) * bdim + threadIdx.x;
      const bool live = j < ngroups;
      u32x4 e, cv, l;
      uint32_t stw = 0, key[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t o = k < 2 ? o01[u][k] : o23[u][k - 2];
        const uint32_t c = (cw[u] >> (8 * k)) & 0xFFu, p = p4[u][k];
        uint32_t lk;
        const uint32_t ek = infer_end(hp, o, r4[u][k], a4[u][k], p, wr[u][k], wa[u][k], &lk);
        uint32_t ck;
        const uint32_t s_k = classify(c, p, ek, n_chrom, s_len, &ck);
        e[k] = ek;
        cv[k] = ck;
        l[k] = lk;
        stw |= s_k << (8 * k);
        key[k] = live ? l8_key(c, p, ck, s_l8off) : 0xFFFFFFFFu;
      }
      if (ctrs && live) {
        nrec += 4;
        if (stw) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t s_k = (stw >> (8 * k)) & 0xFFu;
            err += s_k ? (1u << (8 * (s_k - 1))) : 0u;
          }
        }
      }
      if (HIST) {  // as K1: wave-uniform runs of one key cost one LDS atomic per run
        const bool same = key[1] == key[0] && key[2] == key[0] && key[3] == key[0];
        const uint32_t lk = same ? key[0] : 0xFFFFFFFEu;
        const uint32_t first = __builtin_amdgcn_readfirstlane(lk);
        const uint64_t ok = __ballot(!live || lk == first);
        if (ok == ~0ull && first < 0xFFFFFFFEu) {
          const uint32_t cnt = 4u * uint32_t(__popcll(__ballot(live)));
          if (first == run_key) {
            run_cnt += cnt;
          } else {
            if (run_cnt && __lane_id() == 0) atomicAdd(&hist[run_key], run_cnt);
            run_key = first;
            run_cnt = cnt;
          }
        } else if (!(ok == ~0ull && first == 0xFFFFFFFFu)) {
#pragma unroll
          for (int k = 0; k < 4; ++k) wave_hist_add(key[k], hist);
        }
      }
      if (KEYS != 0 && kt.tot) {  // this wave's 256 records are one K7 group (none: no K7 follows)
        uint32_t K = 0, P = 0;
        if (live) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t c = (cw[u] >> (8 * k)) & 0xFFu;
            const uint64_t ev = k < 2 ? x01[u][k] : x23[u][k - 2];
            uint32_t ks, ps;
            key_path_sizes(c, p4[u][k], r4[u][k], a4[u][k], ev, cv[k], kt.max_seq_len, kt.n_key_chrom,
                           kt.has_digest != 0, kt.with_paths != 0, &ks, &ps);
            K += ks;
            P += ps;
          }
        }
#pragma unroll
        for (int d = 8; d > 0; d >>= 1) {  // over each 16 lanes: 64 records
          K += __shfl_xor(K, d, kWave);
          P += __shfl_xor(P, d, kWave);
        }
        // a K7 group is 64 << group_log2 records = the records of 16 << group_log2 lanes
        if (kt.group_log2 >= 1) {
          K += __shfl_xor(K, 16, kWave);
          P += __shfl_xor(P, 16, kWave);
        }
        if (kt.group_log2 >= 2) {
          K += __shfl_xor(K, 32, kWave);
          P += __shfl_xor(P, 32, kWave);
        }
        if ((__lane_id() & ((16u << kt.group_log2) - 1)) == 0 && j < ngroups)
          kt.tot[j >> (4 + kt.group_log2)] = make_uint2(K, P);
      }
      if constexpr (KEYS != 0) {
        if (dd_mine) {  // K3's mark phase on the (chrom, pos) already in registers
          // A record sharing (chrom, pos) with its predecessor is listed for K3's
          // resolve only if it could repeat a primary key before it: it has the
          // predecessor's lengths and refSNP id, or it is third or later in its run.
          // The rest of a two-record run keeps 1 here (K3's own first test,
          // avdb_dedup.hip k_dedup_resolve_list), so the list holds the
          // duplicates and the longer runs, not every shared position.
          const uint32_t c4 = cw[u];
          const u32x4 q4 = p4[u], rr = r4[u], aa = a4[u];
          const uint64_t* ext1 = reinterpret_cast<const uint64_t*>(kt.ext2);
          uint32_t pc = __shfl_up(c4 >> 24, 1, kWave), pp = __shfl_up(q4.w, 1, kWave);
          uint32_t pr = __shfl_up(rr.w, 1, kWave), pa = __shfl_up(aa.w, 1, kWave);
          const uint64_t e3 = x23[u][1];
          uint64_t pe = (uint64_t(uint32_t(__shfl_up(uint32_t(e3 >> 32), 1, kWave))) << 32) |
                        uint32_t(__shfl_up(uint32_t(e3), 1, kWave));
          uint32_t same = 0;
          if (live) {
            same |= uint32_t(((c4 >> 8) & 0xFFu) == (c4 & 0xFFu) && q4.y == q4.x) << 1;
            same |= uint32_t(((c4 >> 16) & 0xFFu) == ((c4 >> 8) & 0xFFu) && q4.z == q4.y) << 2;
            same |= uint32_t((c4 >> 24) == ((c4 >> 16) & 0xFFu) && q4.w == q4.z) << 3;
          }
          // bit 0 of the previous lane's run bits: its record 3 shares its predecessor's position
          uint32_t psame = (uint32_t(__shfl_up(same, 1, kWave)) >> 3) & 1u;
          if (__lane_id() == 0 && live && j > 0) {
            pc = chrom[4 * j - 1];
            pp = pos[4 * j - 1];
            pr = rl[4 * j - 1];
            pa = al[4 * j - 1];
            pe = ext1 ? ext1[4 * j - 1] : 0ull;
            psame = uint32_t(chrom[4 * j - 2] == pc && pos[4 * j - 2] == pp);
          }
          if (live) same |= uint32_t(j > 0 && (c4 & 0xFFu) == pc && q4.x == pp);
          const uint32_t prev_same = ((same << 1) & 0xEu) | psame;
          uint32_t cand = uint32_t(rr.x == pr && aa.x == pa && x01[u][0] == pe);
          cand |= uint32_t(rr.y == rr.x && aa.y == aa.x && x01[u][1] == x01[u][0]) << 1;
          cand |= uint32_t(rr.z == rr.y && aa.z == aa.y && x23[u][0] == x01[u][1]) << 2;
          cand |= uint32_t(rr.w == rr.z && aa.w == aa.z && x23[u][1] == x23[u][0]) << 3;
          same &= cand | prev_same;
          const uint32_t cnt = __popc(same);
          uint32_t incl = cnt;
#pragma unroll
          for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t up = __shfl_up(incl, d, kWave);
            if (__lane_id() >= uint32_t(d)) incl += up;
          }
          const uint32_t total = __shfl(incl, kWave - 1, kWave);
          if (total) {
            uint32_t at = 0;
            if (__lane_id() == kWave - 1) at = atomicAdd(&s_dd, total);
            at = __shfl(at, kWave - 1, kWave) + incl - cnt;
            for (uint32_t m = same; m; m &= m - 1) dd_mine[at++] = uint32_t(4 * j + __builtin_ctz(m));
          }
          if (live) reinterpret_cast<uint32_t*>(kt.keep)[j] = 0x01010101u;
        }
        if (kt.long_codes && live) {
          uint32_t lc = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) lc |= long_code(r4[u][k], a4[u][k], kt.max_seq_len) << (8 * k);
          __builtin_nontemporal_store(lc, reinterpret_cast<uint32_t*>(kt.long_codes) + j);
        }
      }
      if (live) {
        __builtin_nontemporal_store(e, &end4[j]);
        __builtin_nontemporal_store(cv, &code4[j]);
        if (statusv) __builtin_nontemporal_store(stw, &statusv[j]);
        if (lcp4) lcp4[j] = l;
      }
    }
    if (ctrs && ++since_flush == 255 / (UNROLL * 4)) {  // 8-bit error fields never wrap
      flush_errors(err, s_ctr);
      since_flush = 0;
    }
  }
  if (HIST && run_cnt && __lane_id() == 0) atomicAdd(&hist[run_key], run_cnt);
  // scalar tail (< 4 records)
  if (blockIdx.x == 0 && threadIdx.x < kWave) {
    const size_t i = tail_begin + threadIdx.x;
    uint32_t key = 0xFFFFFFFFu;
    if (i < n) {
      const uint32_t r = rl[i], a = al[i], p = pos[i], c = chrom[i];
      const uint64_t o = off[i];
      const bool snv = r == 1u && a == 1u;
      uint32_t l, cv;
      const uint32_t e = infer_end(hp, o, r, a, p, snv ? 0 : heap_u64(hp, o), snv ? 0 : heap_u64(hp, o + r), &l);
      const uint32_t s_k = classify(c, p, e, n_chrom, s_len, &cv);
      end_out[i] = e;
      code[i] = cv;
      if (status) status[i] = uint8_t(s_k);
      if (lcp) lcp[i] = l;
      if (KEYS != 0 && kt.long_codes) kt.long_codes[i] = uint8_t(long_code(r, a, kt.max_seq_len));
      if (KEYS != 0 && dd_mine) {
        if (i > 0 && chrom[i - 1] == c && pos[i - 1] == p) dd_mine[atomicAdd(&s_dd, 1u)] = uint32_t(i);
        kt.keep[i] = 1;
      }
      nrec += 1;
      err += s_k ? (1u << (8 * (s_k - 1))) : 0u;
      key = l8_key(c, p, cv, s_l8off);
    }
    if (HIST) wave_hist_add(key, hist);
  }
  if (ctrs) {
    flush_errors(err, s_ctr);
    for (int d = 32; d > 0; d >>= 1) nrec += __shfl_down(nrec, d, kWave);
    if (__lane_id() == 0 && nrec) atomicAdd(&s_ctr[AVDB_CTR_RECORDS], (unsigned long long)nrec);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long bad = s_ctr[AVDB_CTR_STATUS0 + 1] + s_ctr[AVDB_CTR_STATUS0 + 2] +
                                     s_ctr[AVDB_CTR_STATUS0 + 3];
      s_ctr[AVDB_CTR_STATUS0] = s_ctr[AVDB_CTR_RECORDS] - bad;
    }
  }
  publish(tab, s_ctr, s_hist, use_lds, HIST, g_hist, g_ctr);  // (begins with a barrier)
  if (KEYS != 0 && dd_mine && threadIdx.x == 0) kt.dd_counts[blockIdx.x] = s_dd;
}

}  // namespace avdb

using namespace avdb;

static inline bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

static int check_ctx(const avdb_ctx* ctx) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  return AVDB_OK;
}

extern "C" int avdb_bin_assign(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* start,
                               const uint32_t* end, size_t n, uint32_t* bin_code, uint8_t* status,
                               uint32_t* hist_l8, uint64_t* counters, void* stream) {
  if (int rc = check_ctx(ctx)) return rc;
  if (n == 0) return AVDB_OK;
  if (!chrom || !start || !bin_code) { avdb_set_error("avdb_bin_assign: null array"); return AVDB_EINVAL; }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool hist = hist_l8 != nullptr;
  const int lds_hist = hist && ctx->tab.n_l8 <= uint32_t(kMaxLdsHistBins);
  const size_t shm = lds_hist ? size_t(ctx->tab.n_l8) * 4 : 0;
  auto* ctr = reinterpret_cast<unsigned long long*>(counters);
  // K1's shape: 4 records per lane-group (chrom as one u32, start / end / code as
  // u32x4), 2 groups in flight, nontemporal loads and stores, grid-stride — chosen among
  // eleven shapes and memory policies by on-device A/B (tools/k1_geom.py,
  // profiles/r01_k1_*.log; the others were removed in round 5)
  constexpr int kV = 1, kU = 2, kF = 4, R = 4 * kV;
  const bool vec = aligned(chrom, size_t(R)) && aligned(start, 16) && (!end || aligned(end, 16)) &&
                   aligned(bin_code, 16) && (!status || aligned(status, size_t(R))) && n >= size_t(R);
  if (vec) {
    const size_t ngroups = n / R;
    // One resident wave of workgroups (n_cu x blocks_per_cu); each step of a
    // workgroup covers kK1Block*U*R consecutive records.
    const unsigned bdim = unsigned(kK1Block);
    const unsigned grid =
        stream_grid(ngroups, bdim * kU, unsigned(ctx->n_cu * ctx->k1_blocks_per_cu));
    const size_t tail = ngroups * R;
#define K1V(HE, HI)                                                                             \
  hipLaunchKernelGGL((k_bin_assign4<HE, HI, kV, kU, kF>), dim3(grid), dim3(bdim), shm, s,      \
                     reinterpret_cast<const typename ChromVec<kV>::T*>(chrom),                   \
                     reinterpret_cast<const u32x4*>(start), reinterpret_cast<const u32x4*>(end), \
                     ngroups, reinterpret_cast<u32x4*>(bin_code),                               \
                     reinterpret_cast<typename ChromVec<kV>::T*>(status), ctx->tab, hist_l8, ctr, \
                     lds_hist, chrom, start, end, tail, n, bin_code, status)
    if (end) { if (hist) K1V(true, true); else K1V(true, false); }
    else { if (hist) K1V(false, true); else K1V(false, false); }
#undef K1V
    AVDB_LAUNCH_CHECK("k_bin_assign4");
  } else {
    const unsigned grid = stream_grid(n, kBlock * 8, 2048);
#define K1S(HE, HI)                                                                  \
  hipLaunchKernelGGL((k_bin_assign1<HE, HI>), dim3(grid), dim3(kBlock), shm, s, chrom, \
                     start, end, n, bin_code, status, ctx->tab, hist_l8, ctr, lds_hist)
    if (end) { if (hist) K1S(true, true); else K1S(true, false); }
    else { if (hist) K1S(false, true); else K1S(false, false); }
#undef K1S
    AVDB_LAUNCH_CHECK("k_bin_assign1");
  }
  return AVDB_OK;
}

static int record_prep_impl(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                            const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap,
                            size_t heap_bytes, size_t n, uint32_t* end_out, uint32_t* bin_code, uint8_t* status,
                            uint32_t* lcp, uint32_t* hist_l8, uint64_t* counters, void* stream, const KeyTotals* keyed,
                            int* totals_written);

// the keyed K2's grid, and the most records one of its workgroups handles (its
// grid-stride trips of bdim * U groups of 4, plus the < 4 records of block 0's
// scalar tail): one K3 list slice each
static unsigned keyed_grid(const avdb_ctx* ctx, size_t n) {
  return stream_grid(n / 4, unsigned(kK1Block) * unsigned(kK2KeyedUnroll),
                     unsigned(ctx->n_cu * ctx->k2_blocks_per_cu));
}
namespace avdb {
void keyed_prep_layout(const avdb_ctx* ctx, size_t n, unsigned* grid, size_t* slice) {
  *grid = 0;
  *slice = 0;
  if (!ctx || n < 4) return;
  const unsigned g = keyed_grid(ctx, n);
  const size_t per_trip = size_t(kK1Block) * size_t(kK2KeyedUnroll) * g;  // groups of 4 per grid trip
  const size_t trips = (n / 4 + per_trip - 1) / per_trip;
  *grid = g;
  *slice = 4 * size_t(kK1Block) * size_t(kK2KeyedUnroll) * trips + 4;
}
}  // namespace avdb

extern "C" int avdb_record_prep(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                const uint64_t* allele_off, const uint32_t* ref_len,
                                const uint32_t* alt_len, const uint8_t* heap, size_t heap_bytes,
                                size_t n, uint32_t* end_out, uint32_t* bin_code, uint8_t* status,
                                uint32_t* lcp, uint32_t* hist_l8, uint64_t* counters,
                                void* stream) {
  return record_prep_impl(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, n, end_out, bin_code,
                          status, lcp, hist_l8, counters, stream, nullptr, nullptr);
}

extern "C" int avdb_record_prep_keyed(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos,
                                      const uint64_t* allele_off, const uint32_t* ref_len, const uint32_t* alt_len,
                                      const uint8_t* heap, size_t heap_bytes, size_t n, uint32_t* end_out,
                                      uint32_t* bin_code, uint8_t* status, uint32_t* lcp, uint32_t* hist_l8,
                                      uint64_t* counters, const uint64_t* ext_id, uint32_t max_seq_len,
                                      int has_digest, int with_paths, void* key_workspace,
                                      size_t key_workspace_bytes, void* digest_workspace,
                                      size_t digest_workspace_bytes, void* dedup_workspace,
                                      size_t dedup_workspace_bytes, uint8_t* keep, int* totals_written,
                                      void* stream) {
  if (!totals_written) {
    avdb_set_error("avdb_record_prep_keyed: null totals_written");
    return AVDB_EINVAL;
  }
  *totals_written = 0;
  size_t need = 0;
  avdb_primary_keys_onepass_workspace_size(n, &need);
  // (no K7 workspace: no group totals — K4's codes and K3's marks only, for a step
  // without key text, as C5's)
  if (key_workspace && (key_workspace_bytes < need || reinterpret_cast<uintptr_t>(key_workspace) % 16)) {
    avdb_set_error("avdb_record_prep_keyed: 16-byte aligned K7 one-pass workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  KeyTotals kt;
  kt.ext2 = reinterpret_cast<const u64x2*>(ext_id);
  kt.tot = key_workspace ? avdb::key_totals_of(key_workspace) : nullptr;
  kt.max_seq_len = max_seq_len;
  kt.n_key_chrom = uint32_t(ctx && ctx->tab.n < 25 ? ctx->tab.n : 25);
  kt.has_digest = has_digest ? 1u : 0u;
  kt.with_paths = with_paths ? 1u : 0u;
  kt.group_log2 = avdb::key_totals_group_log2(n);
  kt.long_codes = nullptr;
  if (digest_workspace) {
    size_t dneed = 0;
    avdb_vrs_digest_workspace_size(n, &dneed);
    if (digest_workspace_bytes < dneed || reinterpret_cast<uintptr_t>(digest_workspace) % 16) {
      avdb_set_error("avdb_record_prep_keyed: 16-byte aligned K4 workspace of %zu bytes required", dneed);
      return AVDB_ERANGE;
    }
    kt.long_codes = avdb::vrs_long_codes_of(digest_workspace, n);
  }
  kt.keep = nullptr;
  kt.dd_counts = kt.dd_list = nullptr;
  kt.dd_slice = 0;
  if (dedup_workspace && keep) {  // K3's mark phase too, when the layout fits
    unsigned grid = 0;
    size_t slice = 0;
    avdb::keyed_prep_layout(ctx, n, &grid, &slice);
    if (grid && grid <= avdb::kDedupMaxGroups && reinterpret_cast<uintptr_t>(dedup_workspace) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(keep) % 4 == 0 &&
        dedup_workspace_bytes >= avdb::kDedupListHead + 4 * size_t(grid) * slice) {
      kt.keep = keep;
      kt.dd_counts = static_cast<uint32_t*>(dedup_workspace);
      kt.dd_list = reinterpret_cast<uint32_t*>(static_cast<char*>(dedup_workspace) + avdb::kDedupListHead);
      kt.dd_slice = slice;
    }
  }
  return record_prep_impl(ctx, chrom, pos, allele_off, ref_len, alt_len, heap, heap_bytes, n, end_out, bin_code,
                          status, lcp, hist_l8, counters, stream, &kt, totals_written);
}

static int record_prep_impl(avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* pos, const uint64_t* allele_off,
                            const uint32_t* ref_len, const uint32_t* alt_len, const uint8_t* heap,
                            size_t heap_bytes, size_t n, uint32_t* end_out, uint32_t* bin_code, uint8_t* status,
                            uint32_t* lcp, uint32_t* hist_l8, uint64_t* counters, void* stream, const KeyTotals* keyed,
                            int* totals_written) {
  if (int rc = check_ctx(ctx)) return rc;
  if (n == 0) return AVDB_OK;
  if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap || !end_out || !bin_code) {
    avdb_set_error("avdb_record_prep: null array");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool hist = hist_l8 != nullptr;
  const int lds_hist = hist && ctx->tab.n_l8 <= uint32_t(kMaxLdsHistBins);
  const size_t shm = lds_hist ? size_t(ctx->tab.n_l8) * 4 : 0;
  auto* ctr = reinterpret_cast<unsigned long long*>(counters);
  const bool vec = n >= 4 && aligned(chrom, 4) && aligned(pos, 16) && aligned(allele_off, 16) &&
                   aligned(ref_len, 16) && aligned(alt_len, 16) && aligned(end_out, 16) && aligned(bin_code, 16) &&
                   (!status || aligned(status, 4)) && (!lcp || aligned(lcp, 16));
  // keyed: the vector form with 16-byte aligned refSNP keys
  const bool keys = keyed && vec && (!keyed->ext2 || aligned(keyed->ext2, 16));
  const KeyTotals kt = keys ? *keyed : KeyTotals{};
  if (vec) {
    const size_t ngroups = n / 4;
    const unsigned bdim = unsigned(kK1Block);
    // groups of 4 records per lane per trip: 2 for plain K2, 1 for the keyed form
    // (its registers: 144 VGPRs at 2); 1 / 2 / 4 measured on the box
    // (tools/k2_probe.py: U=2 0.234-0.247 ms, U=1 0.26-0.31, U=4 0.44-0.47 with spills)
    const unsigned grid = keys ? keyed_grid(ctx, n)
                               : stream_grid(ngroups, bdim * kK2Unroll, unsigned(ctx->n_cu * ctx->k2_blocks_per_cu));
#define K2V(HI)                                                                                           \
  if (keys && kt.group_log2 < 2) K2VK(HI, kK2KeyedUnroll, 2); else if (keys) K2VK(HI, kK2KeyedUnroll, 1); \
  else K2VK(HI, kK2Unroll, 0)
#define K2VK(HI, UU, KK)                                                                                  \
  hipLaunchKernelGGL((k_record_prep4<HI, UU, KK>), dim3(grid), dim3(bdim), shm, s,                       \
                     reinterpret_cast<const uint32_t*>(chrom), reinterpret_cast<const u32x4*>(pos),      \
                     reinterpret_cast<const u64x2*>(allele_off), reinterpret_cast<const u32x4*>(ref_len), \
                     reinterpret_cast<const u32x4*>(alt_len), heap, heap_bytes, ngroups,                  \
                     reinterpret_cast<u32x4*>(end_out), reinterpret_cast<u32x4*>(bin_code),              \
                     reinterpret_cast<uint32_t*>(status), reinterpret_cast<u32x4*>(lcp), ctx->tab, hist_l8, \
                     ctr, lds_hist, kt, chrom, pos, allele_off, ref_len, alt_len, ngroups * 4, n, end_out,  \
                     bin_code, status, lcp)
    if (hist) K2V(true);
    else K2V(false);
#undef K2V
#undef K2VK
    AVDB_LAUNCH_CHECK("k_record_prep4");
    if (keys && totals_written)
      *totals_written = (kt.tot ? AVDB_KEYED_TOTALS : 0) | (kt.long_codes ? AVDB_KEYED_LONG_CODES : 0) |
                        (kt.dd_list ? AVDB_KEYED_DEDUP_MARKS : 0);
    return AVDB_OK;
  }
  const unsigned grid = stream_grid(n, kBlock * 8, 2048);
  if (hist)
    hipLaunchKernelGGL((k_record_prep<true>), dim3(grid), dim3(kBlock), shm, s, chrom, pos,
                       allele_off, ref_len, alt_len, heap, heap_bytes, n, end_out, bin_code, status, lcp,
                       ctx->tab, hist_l8, ctr, lds_hist);
  else
    hipLaunchKernelGGL((k_record_prep<false>), dim3(grid), dim3(kBlock), shm, s, chrom, pos,
                       allele_off, ref_len, alt_len, heap, heap_bytes, n, end_out, bin_code, status, lcp,
                       ctx->tab, hist_l8, ctr, lds_hist);
  AVDB_LAUNCH_CHECK("k_record_prep");
  return AVDB_OK;
}
