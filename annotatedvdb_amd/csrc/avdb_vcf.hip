// K0 — VCF text -> per-alt record SoA on the GPU (gfx950).
//
// Text half of VcfEntryParser (Util/lib/python/parsers/vcf_parser.py:76-169) and the
// per-alt loop head of VCFVariantLoader.__parse_alt_alleles
// (vcf_variant_loader.py:273-280), for a batch of lines resident in HBM:
//   k_vcf_count    per-workgroup count of '\n' bytes (8 bytes per lane-step, SWAR
//                  zero-byte detection), block-contiguous chunks, coalesced
//   k_vcf_starts   ordered line starts: each wave walks a contiguous sub-chunk 512 B
//                  at a time; a lane's newline count is ranked inside the wave with
//                  4 ballots + mbcnt (no LDS), so every start is written in order
//   k_vcf_parse    256 consecutive lines per workgroup: their text span is staged in
//                  LDS with 16-byte coalesced loads, then one lane per line parses from
//                  LDS: rstrip, tab fields, CHROM -> contig code, POS, ID / INFO RS ->
//                  refSNP key, ALT count, heap bytes (spans over kStage bytes parse
//                  straight from global memory)
//   (hipCUB exclusive scans: record and heap offsets per line)
//   k_vcf_emit     same staging; one lane per line: one record per ALT != '.',
//                  REF+ALT copied to the allele heap
// Only canonical text is resolved here; the rest is flagged (AVDB_VCF_*_HOST) for
// the host to resolve with Python's own coercion rules.
#include "avdb_fmt.hpp"
#include "avdb_vcfline.hpp"

#include <hipcub/hipcub.hpp>

namespace avdb {

constexpr int kVcfGrid = 1024;

__device__ __forceinline__ uint32_t count_byte(uint64_t x, uint64_t pattern) {
  return uint32_t(__popcll(zero_bytes_mask(x ^ pattern)));
}

constexpr uint64_t kNL = 0x0A0A0A0A0A0A0A0Aull;

// The text is cut into kVcfGrid * kVcfWaves contiguous, 64-byte-aligned wave
// sub-chunks; k_vcf_count and k_vcf_starts use the same cut, so the starts pass
// reads every wave's newline offset instead of recounting.
constexpr int kVcfWaves = kBlock / kWave;
constexpr size_t kCountWsBlkOff = 0;                              // u64[kVcfGrid] exclusive
constexpr size_t kCountWsTotal = 8 * kVcfGrid;                    // u64 total (+pad)
constexpr size_t kCountWsWave = kCountWsTotal + 256;              // u32[kVcfGrid * kVcfWaves]
constexpr size_t kCountWsBytes = kCountWsWave + 4 * kVcfGrid * kVcfWaves;
static_assert(kCountWsBytes <= AVDB_VCF_COUNT_WORKSPACE_BYTES, "count workspace");

__device__ __forceinline__ void wave_range(size_t text_bytes, size_t gw, size_t* t0, size_t* t1) {
  const size_t nw = size_t(kVcfGrid) * kVcfWaves;
  size_t per = (text_bytes + nw - 1) / nw;
  per = (per + 63) & ~size_t(63);
  *t0 = gw * per < text_bytes ? gw * per : text_bytes;
  *t1 = *t0 + per < text_bytes ? *t0 + per : text_bytes;
}

// newline masks (bit 7 of each '\n' byte) of the 16 bytes at 16-aligned address a,
// restricted to [lo, end)
struct Mask16 {
  uint64_t m0, m1;
  uint32_t commas;  // ',' bytes in the same range (k_vcf_count; dead code elsewhere)
};

__device__ __forceinline__ Mask16 nl_mask16(uintptr_t a, const Heap& h, uintptr_t lo, uintptr_t end) {
  uint64_t m0 = 0, m1 = 0;
  if (a >= end) return Mask16{0, 0, 0};
  uint64_t x, y;
  if (a >= h.lo && a + 16 <= h.hi) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a));
    x = uint64_t(v[0]) | uint64_t(v[1]) << 32;
    y = uint64_t(v[2]) | uint64_t(v[3]) << 32;
  } else {
    x = text_word(a, h);
    y = text_word(a + 8, h);
  }
  m0 = zero_bytes_mask(x ^ kNL) & 0x8080808080808080ull;
  m1 = zero_bytes_mask(y ^ kNL) & 0x8080808080808080ull;
  uint64_t k0 = bytes_eq_mask(x, ','), k1 = bytes_eq_mask(y, ',');
  if (a < lo) {
    const uint32_t sh = uint32_t(lo - a);  // 1..15 bytes before the range
    if (sh >= 8) { m0 = 0; m1 &= ~low_bytes_mask(sh - 8); k0 = 0; k1 &= ~low_bytes_mask(sh - 8); }
    else { m0 &= ~low_bytes_mask(sh); k0 &= ~low_bytes_mask(sh); }
  }
  if (a + 16 > end) {
    const uint32_t keep = uint32_t(end - a);  // 1..15 bytes inside the range
    if (keep <= 8) { m1 = 0; m0 &= low_bytes_mask(keep); k1 = 0; k0 &= low_bytes_mask(keep); }
    else { m1 &= low_bytes_mask(keep - 8); k1 &= low_bytes_mask(keep - 8); }
  }
  return Mask16{m0, m1, uint32_t(__popcll(k0) + __popcll(k1))};
}

constexpr int kNlUnroll = 4;                           // 16-byte lane loads in flight
constexpr uintptr_t kNlStep = 16 * kWave;              // bytes per wave load

__global__ __launch_bounds__(kBlock) void k_vcf_count(const uint8_t* __restrict__ text,
                                                      size_t text_bytes,
                                                      uint32_t* __restrict__ wave_cnt,
                                                      unsigned long long* __restrict__ commas) {
  const Heap h = make_heap(text, text_bytes);
  const size_t gw = size_t(blockIdx.x) * kVcfWaves + threadIdx.x / kWave;
  size_t t0, t1;
  wave_range(text_bytes, gw, &t0, &t1);
  const uintptr_t lo = h.lo + t0, end = h.lo + t1;
  uint32_t c = 0, k = 0;
  for (uintptr_t a = (lo & ~uintptr_t(15)) + 16 * __lane_id(); a < end; a += kNlUnroll * kNlStep) {
    Mask16 m[kNlUnroll];
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) m[u] = nl_mask16(a + u * kNlStep, h, lo, end);
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) {
      c += uint32_t(__popcll(m[u].m0) + __popcll(m[u].m1));
      k += m[u].commas;
    }
  }
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
  if (__lane_id() == 0) wave_cnt[gw] = c;
  if (commas) {  // (a bound on the records: every record is a line or follows a comma)
    for (int d = 32; d > 0; d >>= 1) k += __shfl_xor(k, d, kWave);
    if (__lane_id() == 0 && k) atomicAdd(commas, (unsigned long long)k);
  }
}

// per-workgroup newline totals -> exclusive offsets (one workgroup of kVcfGrid threads)
__global__ __launch_bounds__(kVcfGrid) void k_vcf_scan_blocks(const uint32_t* __restrict__ wave_cnt,
                                                              unsigned long long* __restrict__ blk_off,
                                                              unsigned long long* __restrict__ total) {
  __shared__ unsigned long long s[kVcfGrid];
  const int t = threadIdx.x;
  unsigned long long v = 0;
#pragma unroll
  for (int w = 0; w < kVcfWaves; ++w) v += wave_cnt[t * kVcfWaves + w];
  s[t] = v;
  __syncthreads();
  for (int d = 1; d < kVcfGrid; d <<= 1) {
    const unsigned long long x = t >= d ? s[t - d] : 0ull;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  blk_off[t] = s[t] - v;
  if (t == kVcfGrid - 1 && total) *total = s[t];
}

// popcount of `m` over the lanes below this one
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

// line starts in order: line 0 starts at 0, line k+1 after the k-th newline.  Each
// wave walks its sub-chunk once; a lane's newline count (0..16) is ranked inside the
// wave with 5 ballots.
__global__ __launch_bounds__(kBlock) void k_vcf_starts(const uint8_t* __restrict__ text,
                                                       size_t text_bytes,
                                                       const unsigned long long* __restrict__ blk_off,
                                                       const uint32_t* __restrict__ wave_cnt,
                                                       size_t n_lines,
                                                       uint64_t* __restrict__ starts) {
  const Heap h = make_heap(text, text_bytes);
  const int wave = threadIdx.x / kWave, lane = __lane_id();
  const size_t gw = size_t(blockIdx.x) * kVcfWaves + wave;
  size_t t0, t1;
  wave_range(text_bytes, gw, &t0, &t1);
  unsigned long long k = blk_off[blockIdx.x];  // newlines before t0
  for (int w = 0; w < wave; ++w) k += wave_cnt[size_t(blockIdx.x) * kVcfWaves + w];
  if (gw == 0 && lane == 0 && n_lines) starts[0] = 0;
  const uintptr_t lo = h.lo + t0, end = h.lo + t1;
  for (uintptr_t a0 = lo & ~uintptr_t(15); a0 < end; a0 += kNlUnroll * kNlStep) {
    Mask16 m[kNlUnroll];
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) m[u] = nl_mask16(a0 + u * kNlStep + 16 * lane, h, lo, end);
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) {
      const uint32_t cnt = uint32_t(__popcll(m[u].m0) + __popcll(m[u].m1));
      uint32_t below = 0, total = 0;
#pragma unroll
      for (int bit = 0; bit < 5; ++bit) {
        const uint64_t b = __ballot((cnt >> bit) & 1u);
        below += lanes_below(b) << bit;
        total += uint32_t(__popcll(b)) << bit;
      }
      if (cnt) {
        unsigned long long kk = k + below;
        const size_t wbase = size_t(a0 + u * kNlStep + 16 * lane - h.lo);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          uint64_t mm = half ? m[u].m1 : m[u].m0;
          while (mm) {
            const int bitpos = __builtin_ctzll(mm);
            mm &= mm - 1;
            if (kk + 1 < n_lines) starts[kk + 1] = wbase + 8 * half + size_t(bitpos >> 3) + 1;
            ++kk;
          }
        }
      }
      k += total;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_vcf_parse(const uint8_t* __restrict__ text,
                                                      size_t text_bytes, size_t n_lines,
                                                      const uint64_t* __restrict__ starts,
                                                      avdb_vcf_line* __restrict__ lines,
                                                      unsigned long long* __restrict__ rec_cnt,
                                                      unsigned long long* __restrict__ heap_cnt,
                                                      ChromMapView cm, uint32_t min_fields) {
  __shared__ u32x4 s_text[kStage / 16];
  const Heap h = make_heap(text, text_bytes);
  for (size_t base = size_t(blockIdx.x) * kBlock; base < n_lines; base += size_t(gridDim.x) * kBlock) {
    const size_t last = base + kBlock < n_lines ? base + kBlock : n_lines;
    const size_t s0 = starts[base];
    const size_t s1 = last < n_lines ? starts[last] : text_bytes;
    const Window w = stage_window(h, s0, s1, s_text);
    const size_t li = base + threadIdx.x;
    if (li < n_lines) {
      avdb_vcf_line L;
      L.start = starts[li];
      const size_t next = li + 1 < n_lines ? starts[li + 1] - 1 : text_bytes;  // newline or end
      const uint32_t raw = uint32_t(next - L.start);
      uint64_t recs, hbytes;
      const uint32_t mis = uint32_t((h.lo + L.start) & 7);
      if (w.staged) {
        const uint8_t* ls = reinterpret_cast<const uint8_t*>(s_text) + (h.lo + L.start - w.a0);
        const lds_cp64 lw = (lds_cp64)(reinterpret_cast<const uint64_t*>(ls - mis));
        parse_line((lds_cp)ls, [lw](uint32_t k) { return lw[k]; }, mis, raw, L, recs, hbytes, cm, min_fields);
      } else {
        const uintptr_t la = h.lo + L.start - mis;
        parse_line((glb_cp)(text + L.start), [la, h](uint32_t k) { return heap_word(la + 8 * size_t(k), h); },
                   mis, raw, L, recs, hbytes, cm, min_fields);
      }
      lines[li] = L;
      rec_cnt[li] = recs;
      heap_cnt[li] = hbytes;
    }
    __syncthreads();  // the window is reused by the next trip
  }
}

// (Rendering the allele heap through an LDS image of the tile's heap span with a
// coalesced flush, as K7 does for its text, measured slower: 0.66 vs 0.60 ms for
// 8.4 M lines — the pass is bound by re-staging the text, not by these stores.)
template <class CP>
__device__ __forceinline__ void emit_line(CP s, const avdb_vcf_line& L, size_t li,
                                          uint64_t r, uint64_t h, uint8_t* __restrict__ chrom,
                                          uint32_t* __restrict__ pos, uint64_t* __restrict__ allele_off,
                                          uint32_t* __restrict__ ref_len, uint32_t* __restrict__ alt_len,
                                          uint64_t* __restrict__ ext_id, uint8_t* __restrict__ heap,
                                          uint32_t* __restrict__ rec_line, uint32_t* __restrict__ rec_alt) {
    const uint32_t nfields = L.n_fields < 8 ? L.n_fields : 8;
    const uint32_t rend = L.field[4] - 1;
    const uint32_t aend = 5 < nfields ? L.field[5] - 1 : L.len;
    const CP ref = s + L.field[3];
    const uint32_t rlen = rend - L.field[3];
    const CP alt = s + L.field[4];
    const uint32_t an = aend - L.field[4];
    // ALTs found with SWAR comma scans; the heap bytes leave through the 8-byte
    // register sink (this lane's records are contiguous in the heap)
    Out<true> hs(heap, h);
    uint32_t ai = 0;
    for (uint32_t a0 = 0; a0 <= an; ++ai) {
      const uint32_t a1 = a0 + swar_find(alt + a0, an - a0, [](uint64_t x) { return bytes_eq_mask(x, ','); });
      const uint32_t al = a1 - a0;
      if (!(al == 1 && alt[a0] == '.')) {
        chrom[r] = L.chrom;
        pos[r] = L.pos;
        allele_off[r] = h;
        ref_len[r] = rlen;
        alt_len[r] = al;
        ext_id[r] = L.ext_id;
        rec_line[r] = uint32_t(li);
        rec_alt[r] = ai;
        hs.bytes(ref, rlen);
        hs.bytes(alt + a0, al);
        h += rlen + al;
        ++r;
      }
      a0 = a1 + 1;
    }
    hs.finish();
}

// ---------------------------------------------------------------------------
// K0 in one text pass (avdb_vcf_tokenize).  The text is cut into kTokChunk-byte
// chunks taken in order (ticket counter); a chunk owns the lines that START in
// it.  Its workgroup stages the chunk plus an overhang in LDS, finds its line
// starts from newline bitmaps (one 64-byte block per lane, block scan), parses
// each line (parse_line, as k_vcf_parse), and publishes its totals (lines,
// records, heap bytes).  A decoupled look-back over the chunks before it gives
// its line / record / heap offsets, and the same workgroup then writes the line
// table, the offsets, the record SoA and the allele heap from the staged text.
// The text is read once (the four-kernel path reads it four times and round-
// trips a line-start array and the 80-byte line table).
// ---------------------------------------------------------------------------
#ifndef AVDB_TOK_CHUNK
#define AVDB_TOK_CHUNK 16384
#endif
constexpr uint32_t kTokChunk = AVDB_TOK_CHUNK;        // owned bytes per chunk
constexpr uint32_t kTokOver = 4096;                   // staged past the chunk (lines crossing its end)
constexpr uint32_t kTokStage16 = (kTokChunk + kTokOver) / 16 + 2;
constexpr uint32_t kTokBlocks = kTokChunk / 64 + 1;   // 64-byte bitmap blocks of a chunk (+ the head byte)
static_assert(kTokChunk % 64 == 0 && kTokBlocks <= 2 * kBlock, "chunk / lane blocks");

struct TokArgs {
  const uint8_t* text;
  size_t text_bytes, n_chunks;
  size_t lines_cap, rec_cap, heap_cap;
  avdb_vcf_line* lines;
  uint64_t* rec_off;
  uint64_t* heap_off;
  uint8_t* chrom;
  uint32_t* pos;
  uint64_t* allele_off;
  uint32_t* ref_len;
  uint32_t* alt_len;
  uint64_t* ext_id;
  uint8_t* heap;
  uint32_t* rec_line;
  uint32_t* rec_alt;
  unsigned long long* totals;  // [0] lines [1] records [2] heap bytes [3] look-back waits given up (a bug signal)
  unsigned int* ticket;
  uint64_t* status;  // per chunk: flag (bits 63:62) | packed aggregate
  uint64_t* agg;     // per chunk 3 values (flag 3: an aggregate too wide to pack)
  uint64_t* pre;     // per chunk 3 inclusive prefixes (flag 2)
  uint32_t* trace;   // per chunk: the last phase its workgroup reached (diagnostics, plain stores)
  uint64_t* clock;   // per chunk: s_memrealtime when it published its aggregate / inclusive prefix
  uint64_t* stuck;   // the first look-back wait given up: (chunk, waited-on chunk, status seen, phase)
  ChromMapView cm;
  uint32_t min_fields;
};

constexpr uint64_t kTokAgg = 1ull << 62, kTokInc = 2ull << 62, kTokAggWide = 3ull << 62;
constexpr uint32_t kTokSpinLimit = 1u << 18;  // polls (each >= ~2 us): a wait this long is a bug

// '\n' bytes of an 8-byte word as 8 bits (bit k = byte k)
__device__ __forceinline__ uint32_t nl_bits8(uint64_t w) {
  const uint64_t m = zero_bytes_mask(w ^ kNL) & kHiBits;
  return uint32_t(((m >> 7) * 0x0102040810204080ull) >> 56);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int d) {
  return (uint64_t(uint32_t(__shfl_xor(uint32_t(v >> 32), d, kWave))) << 32) | uint32_t(__shfl_xor(uint32_t(v), d, kWave));
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
  return (uint64_t(uint32_t(__shfl_up(uint32_t(v >> 32), d, kWave))) << 32) | uint32_t(__shfl_up(uint32_t(v), d, kWave));
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += shfl_xor64(v, d);
  return v;
}

// exclusive block scan of two u64 values per thread (kBlock threads); *tot = sums
__device__ __forceinline__ void block_scan2(uint64_t a, uint64_t b, uint64_t* ea, uint64_t* eb, uint64_t* ta,
                                            uint64_t* tb, uint64_t* s_scr /* 2 * kVcfWaves */) {
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  uint64_t xa = a, xb = b;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t ua = shfl_up64(xa, d), ub = shfl_up64(xb, d);
    if (lane >= uint32_t(d)) {
      xa += ua;
      xb += ub;
    }
  }
  if (lane == kWave - 1) {
    s_scr[wv] = xa;
    s_scr[kVcfWaves + wv] = xb;
  }
  __syncthreads();
  uint64_t ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
  for (int w = 0; w < kVcfWaves; ++w) {
    const uint64_t va = s_scr[w], vb = s_scr[kVcfWaves + w];
    if (w < int(wv)) {
      ba += va;
      bb += vb;
    }
    sa += va;
    sb += vb;
  }
  *ea = ba + xa - a;
  *eb = bb + xb - b;
  *ta = sa;
  *tb = sb;
  __syncthreads();  // s_scr is reused by the next call
}

// The look-back's cross-workgroup words: relaxed agent-scope loads and stores
// (global_load/store sc1, as rocPRIM's look-back scan), the status word stored
// after an explicit s_waitcnt for the payload stores before it
// (MI355X_MICROARCH.md, compiler hazard).  tools/handoff_probe.hip measured this
// form and 8-byte agent atomics on both sides equally (no lost or stale hand-off).
__device__ __forceinline__ uint64_t tok_read(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tok_write(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tok_publish(uint64_t* st, uint64_t v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tok_write(st, v);
}

// aggregate (lines, records, heap) of a status word with flag 1 or 3
__device__ __forceinline__ void tok_agg(const TokArgs& A, uint64_t v, int64_t j, uint64_t& a0, uint64_t& a1,
                                        uint64_t& a2) {
  if ((v >> 62) == 1) {
    a0 += (v >> 42) & 0xFFFFFull;
    a1 += (v >> 22) & 0xFFFFFull;
    a2 += v & 0x3FFFFFull;
  } else {
    a0 += tok_read(A.agg + 3 * j);
    a1 += tok_read(A.agg + 3 * j + 1);
    a2 += tok_read(A.agg + 3 * j + 2);
  }
}

// the chunk's exclusive (lines, records, heap) prefix; wave 0 calls it.  Each
// poll step reads kLbPer status words per lane (512 chunks per round trip): all
// workgroups finish their parse at about the same time, so a chunk far from the
// last published prefix would otherwise walk back one 64-chunk window per round
// trip (tools/handoff_probe.hip: ~90 ns per chunk that way).
#ifndef AVDB_TOK_LBPER
#define AVDB_TOK_LBPER 1  // status words per lane per poll (A/B at 2 waves/SIMD: 8 4.13 ms, 1 3.84)
#endif
constexpr int kLbPer = AVDB_TOK_LBPER;
__device__ __forceinline__ void tok_lookback(const TokArgs& A, size_t c, uint64_t T, uint64_t R, uint64_t H,
                                             uint64_t* ex) {
  const uint32_t lane = __lane_id();
  uint64_t s0 = 0, s1 = 0, s2 = 0;
  if (c > 0) {
    if (lane == 0) {
      A.clock[2 * c] = __builtin_amdgcn_s_memrealtime();
      if (T < (1u << 20) && R < (1u << 20) && H < (1u << 22)) {
        tok_publish(A.status + c, kTokAgg | (T << 42) | (R << 22) | H);
      } else {
        tok_write(A.agg + 3 * c, T);
        tok_write(A.agg + 3 * c + 1, R);
        tok_write(A.agg + 3 * c + 2, H);
        tok_publish(A.status + c, kTokAggWide);
      }
    }
    int64_t base = int64_t(c) - 1;
    uint32_t spins = 0;
    while (true) {
      uint64_t v[kLbPer];
      uint32_t nr = 0;  // bit k: status k not published yet
#pragma unroll
      for (int k = 0; k < kLbPer; ++k) {
        const int64_t j = base - kLbPer * int64_t(lane) - k;
        v[k] = j >= 0 ? tok_read(A.status + j) : kTokInc;  // before chunk 0: a zero prefix
      }
#pragma unroll
      for (int k = 0; k < kLbPer; ++k) nr |= ((v[k] >> 62) == 0 ? 1u : 0u) << k;
      while (!__all(nr == 0)) {
        __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (int k = 0; k < kLbPer; ++k) {
          if (nr >> k & 1u) {
            v[k] = tok_read(A.status + (base - kLbPer * int64_t(lane) - k));
            if (v[k] >> 62) nr &= ~(1u << k);
          }
        }
        if (++spins > kTokSpinLimit) {  // never expected: count it, never hang
          const uint64_t nrb = __ballot(nr != 0);
          const uint32_t l0 = nrb ? uint32_t(__ffsll((unsigned long long)nrb)) - 1 : 0u;
          const uint32_t nr0 = __shfl(nr, l0, kWave);
          if (lane == 0 && atomicAdd(A.totals + 3, 1ull) == 0) {
            const int64_t jj = base - kLbPer * int64_t(l0) - (nr0 ? __builtin_ctz(nr0) : 0);
            A.stuck[0] = c;
            A.stuck[1] = uint64_t(jj);
            A.stuck[2] = jj >= 0 ? tok_read(A.status + jj) : ~0ull;
            A.stuck[3] = jj >= 0 ? A.trace[jj] : ~0u;
            A.stuck[4] = 0;
            A.stuck[5] = 0;
            A.stuck[6] = nrb;
            A.stuck[7] = __builtin_amdgcn_s_memrealtime();
          }
#pragma unroll
          for (int k = 0; k < kLbPer; ++k)
            if (nr >> k & 1u) v[k] = kTokInc;
          nr = 0;
        }
      }
      // the nearest published prefix: lane l, its status kf
      uint32_t kf = kLbPer;
#pragma unroll
      for (int k = kLbPer - 1; k >= 0; --k)
        if ((v[k] >> 62) == 2) kf = k;
      const uint64_t pm = __ballot(kf < uint32_t(kLbPer));
      const uint32_t l = pm ? uint32_t(__ffsll((unsigned long long)pm)) - 1 : kWave;
      uint64_t a0 = 0, a1 = 0, a2 = 0;
      if (lane <= l) {
        const uint32_t kn = lane < l ? uint32_t(kLbPer) : kf;  // aggregates before the prefix
#pragma unroll
        for (int k = 0; k < kLbPer; ++k) {
          const int64_t j = base - kLbPer * int64_t(lane) - k;
          if (uint32_t(k) < kn && j >= 0) tok_agg(A, v[k], j, a0, a1, a2);
        }
        if (lane == l && kf < uint32_t(kLbPer)) {
          const int64_t j = base - kLbPer * int64_t(lane) - kf;
          if (j >= 0) {
            a0 += tok_read(A.pre + 3 * j);
            a1 += tok_read(A.pre + 3 * j + 1);
            a2 += tok_read(A.pre + 3 * j + 2);
          }
        }
      }
      s0 += wave_sum64(a0);
      s1 += wave_sum64(a1);
      s2 += wave_sum64(a2);
      if (pm) break;
      base -= kLbPer * kWave;
    }
  }
  if (lane == 0) {
    tok_write(A.pre + 3 * c, s0 + T);
    tok_write(A.pre + 3 * c + 1, s1 + R);
    tok_write(A.pre + 3 * c + 2, s2 + H);
    tok_publish(A.status + c, kTokInc);
    A.clock[2 * c + 1] = __builtin_amdgcn_s_memrealtime();
  }
  ex[0] = s0;
  ex[1] = s1;
  ex[2] = s2;
}

#ifndef AVDB_TOK_WAVES
#define AVDB_TOK_WAVES 4  // min waves per SIMD the register allocation must allow (A/B: 2 4.13 ms, 3 3.34, 4 3.15)
#endif
__global__ __launch_bounds__(kBlock, AVDB_TOK_WAVES) void k_vcf_tokenize(TokArgs A) {
  __shared__ u32x4 s_text[kTokStage16];
  __shared__ uint32_t s_start[kBlock + 1];  // line starts of the round, relative to c0
  __shared__ uint64_t s_scr[2 * kVcfWaves];
  __shared__ uint64_t s_base[4];            // ticket; exclusive lines / records / heap
  __shared__ uint32_t s_tail;               // (first '\n' at or after c1 - 1) + 1 - c0
  const Heap h = make_heap(A.text, A.text_bytes);
  const size_t nb = A.text_bytes;
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid / kWave;
  for (;;) {
    if (tid == 0) s_base[0] = atomicAdd(A.ticket, 1u);
    __syncthreads();
    const size_t c = s_base[0];
    if (c >= A.n_chunks) return;  // (uniform: every thread read the same ticket)
    if (tid == 0) A.trace[c] = 1;  // ticket taken
    const size_t c0 = c * kTokChunk;
    const size_t c1 = c0 + kTokChunk < nb ? c0 + kTokChunk : nb;
    const size_t q0 = c0 ? c0 - 1 : 0;  // newline positions [q0, c1 - 1) start this chunk's lines
    // ---- stage [q0, c1 + kTokOver) ----
    const uintptr_t a0 = (h.lo + q0) & ~uintptr_t(15);
    const uintptr_t wend = h.lo + (c1 + kTokOver < nb ? c1 + kTokOver : nb);
    const uint32_t n16 = uint32_t((wend - a0 + 15) / 16);
    for (uint32_t i = tid; i < n16; i += kBlock) {
      const uintptr_t a = a0 + 16 * size_t(i);
      u32x4 v;
      if (a >= h.lo && a + 16 <= h.hi) {
        v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a));
      } else {
        const uint64_t x = text_word(a, h), y = text_word(a + 8, h);
        v = u32x4{uint32_t(x), uint32_t(x >> 32), uint32_t(y), uint32_t(y >> 32)};
      }
      s_text[i] = v;
    }
    __syncthreads();
    const lds_cp64 lw = (lds_cp64)(reinterpret_cast<const uint64_t*>(s_text));
    // ---- newline bitmaps of [q0, c1 - 1): 64 LDS bytes per block, blocks 2t and 2t + 1 for
    // thread t (adjacent, so the block scan numbers the lines in text order) ----
    const uint32_t o_lo = uint32_t(h.lo + q0 - a0), o_hi = uint32_t(h.lo + c1 - 1 - a0);
    const uint32_t nblk = c1 - 1 > q0 ? (o_hi + 63) / 64 : 0u;
    uint64_t bm[2] = {0, 0};
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t b = 2 * tid + k;
      if (b < nblk) {
        uint64_t m = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) m |= uint64_t(nl_bits8(lw[8 * b + q])) << (8 * q);
        const uint32_t blo = 64 * b;
        if (o_lo > blo) m &= o_lo - blo >= 64 ? 0ull : ~0ull << (o_lo - blo);
        if (o_hi < blo + 64) m &= o_hi <= blo ? 0ull : ~0ull >> (64 - (o_hi - blo));
        bm[k] = m;
        cnt += uint32_t(__popcll(m));
      }
    }
    uint64_t pref, unused, T, unused2;
    block_scan2(cnt, 0, &pref, &unused, &T, &unused2, s_scr);
    const uint32_t first = c0 == 0 && nb ? 1u : 0u;  // line 0 starts at byte 0
    T += first;
    // ---- the end of the chunk's last line: first '\n' at or after c1 - 1 ----
    if (T && wv == 0) {
      size_t q = c1 - 1;
      uint32_t found = 0;
      // in the staged overhang, 64 lanes x 8 bytes per step
      const uint32_t ob = uint32_t(h.lo + q - a0), oe = uint32_t(wend - a0);
      for (uint32_t o = ob & ~7u; o < oe && !found; o += 8 * kWave) {
        const uint32_t wo = o + 8 * lane;
        uint32_t m = wo < oe ? nl_bits8(lw[wo / 8]) : 0u;
        if (wo < ob) m &= ob - wo >= 8 ? 0u : ~0u << (ob - wo);
        if (wo + 8 > oe) m &= oe <= wo ? 0u : 0xFFu >> (8 - (oe - wo));
        const uint64_t bal = __ballot(m != 0);
        if (bal) {
          const uint32_t l = uint32_t(__ffsll((unsigned long long)bal)) - 1;
          const uint32_t ml = __shfl(m, l, kWave);
          q = (a0 - h.lo) + o + 8 * l + uint32_t(__builtin_ctz(ml));
          found = 1;
        }
      }
      // past the overhang (a line longer than it): global memory, 64 x 8 bytes per step
      for (uintptr_t ga = wend & ~uintptr_t(7); !found && ga < h.hi; ga += 8 * kWave) {
        const uintptr_t wa = ga + 8 * lane;
        uint32_t m = wa < h.hi ? nl_bits8(text_word(wa, h)) : 0u;
        if (wa < wend) m &= wend - wa >= 8 ? 0u : ~0u << (wend - wa);
        const uint64_t bal = __ballot(m != 0);
        if (bal) {
          const uint32_t l = uint32_t(__ffsll((unsigned long long)bal)) - 1;
          const uint32_t ml = __shfl(m, l, kWave);
          q = (ga - h.lo) + 8 * l + uint32_t(__builtin_ctz(ml));
          found = 1;
        }
      }
      if (lane == 0) s_tail = uint32_t((found ? q + 1 : nb + 1) - c0);
    }
    // ---- parse: rounds of kBlock lines ----
    const uint32_t rounds = uint32_t((T + kBlock - 1) / kBlock);
    avdb_vcf_line L0{};
    uint64_t rec0 = 0, hb0 = 0, Rt = 0, Ht = 0;
    // line starts [256 r, 256 r + 256] of the chunk into s_start (relative to c0)
    auto fill_starts = [&](uint32_t r) {
      const uint32_t lo = kBlock * r, hi = lo + kBlock;
      if (r == 0 && first && tid == 0) s_start[0] = 0;
      uint32_t idx = first + uint32_t(pref);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        uint64_t m = bm[k];
        while (m && idx <= hi) {
          const uint32_t bit = uint32_t(__builtin_ctzll(m));
          m &= m - 1;
          if (idx >= lo) s_start[idx - lo] = uint32_t(a0 - h.lo - c0) + 64 * (2 * tid + k) + bit + 1;
          ++idx;
        }
      }
      if (tid == 0 && T <= hi) s_start[T - lo] = s_tail;
      __syncthreads();
    };
    auto parse_at = [&](uint32_t t, avdb_vcf_line& L, uint64_t& recs, uint64_t& hbytes) {
      const size_t st = c0 + s_start[t];
      size_t nl = c0 + s_start[t + 1] - 1;  // its newline, or the text end
      if (nl < st || nl > nb) {  // never expected (line starts are increasing): bound the parse, flag it
        atomicAdd(A.totals + 3, 1ull);
        nl = st;
      }
      L.start = st;
      const uint32_t raw = uint32_t(nl - st);
      const uint32_t mis = uint32_t((h.lo + st) & 7);
      if (h.lo + nl <= wend) {
        const uint8_t* ls = reinterpret_cast<const uint8_t*>(s_text) + (h.lo + st - a0);
        const lds_cp64 lw2 = (lds_cp64)(reinterpret_cast<const uint64_t*>(ls - mis));
        parse_line((lds_cp)ls, [lw2](uint32_t k) { return lw2[k]; }, mis, raw, L, recs, hbytes, A.cm,
                   A.min_fields);
      } else {
        const uintptr_t la = h.lo + st - mis;
        parse_line((glb_cp)(A.text + st), [la, h](uint32_t k) { return heap_word(la + 8 * size_t(k), h); }, mis,
                   raw, L, recs, hbytes, A.cm, A.min_fields);
      }
    };
    for (uint32_t r = 0; r < rounds; ++r) {
      fill_starts(r);
      if (kBlock * r + tid < T) {
        avdb_vcf_line L;
        uint64_t recs, hbytes;
        parse_at(tid, L, recs, hbytes);
        Rt += recs;
        Ht += hbytes;
        if (r == 0) {
          L0 = L;
          rec0 = recs;
          hb0 = hbytes;
        }
      }
      __syncthreads();  // s_start is refilled by the next round
    }
    uint64_t e0, e1, R, H;
    block_scan2(Rt, Ht, &e0, &e1, &R, &H, s_scr);
    if (tid == 0) A.trace[c] = 2;  // parsed
    // ---- offsets: decoupled look-back over the chunks before this one ----
    if (wv == 0) {
      uint64_t ex[3];
      tok_lookback(A, c, T, R, H, ex);
      if (lane == 0) {
        s_base[1] = ex[0];
        s_base[2] = ex[1];
        s_base[3] = ex[2];
        if (c + 1 == A.n_chunks) {  // the grand totals
          const uint64_t nl = ex[0] + T, nr = ex[1] + R, nh = ex[2] + H;
          A.totals[0] = nl;
          A.totals[1] = nr;
          A.totals[2] = nh;
          if (nl <= A.lines_cap) {
            A.rec_off[nl] = nr;
            A.heap_off[nl] = nh;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) A.trace[c] = 3;  // offsets known
    uint64_t lb = s_base[1], rb = s_base[2], hb = s_base[3];
    // ---- emit: line table, offsets, record SoA, allele heap ----
    for (uint32_t r = 0; r < rounds; ++r) {
      avdb_vcf_line L = L0;
      uint64_t recs = rec0, hbytes = hb0;
      const bool live = kBlock * r + tid < T;
      if (r > 0) {  // (a chunk of more than kBlock lines parses its later rounds again)
        fill_starts(r);
        recs = hbytes = 0;
        if (live) parse_at(tid, L, recs, hbytes);
      }
      uint64_t er, eh, tr, th;
      block_scan2(live ? recs : 0, live ? hbytes : 0, &er, &eh, &tr, &th, s_scr);
      if (live) {
        const size_t li = lb + kBlock * r + tid;
        const uint64_t ro = rb + er, ho = hb + eh;
        if (li < A.lines_cap) {
          A.lines[li] = L;
          A.rec_off[li] = ro;
          A.heap_off[li] = ho;
        }
        if (L.n_rec && ro + L.n_rec <= A.rec_cap && ho + hbytes <= A.heap_cap) {
          const size_t st = L.start;
          if (h.lo + st + L.len <= wend)
            emit_line((lds_cp)(reinterpret_cast<const uint8_t*>(s_text) + (h.lo + st - a0)), L, li, ro, ho,
                      A.chrom, A.pos, A.allele_off, A.ref_len, A.alt_len, A.ext_id, A.heap, A.rec_line,
                      A.rec_alt);
          else
            emit_line((glb_cp)(A.text + st), L, li, ro, ho, A.chrom, A.pos, A.allele_off, A.ref_len, A.alt_len,
                      A.ext_id, A.heap, A.rec_line, A.rec_alt);
        }
      }
      rb += tr;
      hb += th;
      if (r + 1 < rounds) __syncthreads();
    }
    if (tid == 0) A.trace[c] = 4;  // emitted
    __syncthreads();  // the window, s_start and s_base are reused by the next chunk
  }
}

__global__ __launch_bounds__(kBlock) void k_vcf_emit(
    const uint8_t* __restrict__ text, size_t text_bytes, size_t n_lines,
    const avdb_vcf_line* __restrict__ lines, const uint64_t* __restrict__ rec_off,
    const uint64_t* __restrict__ heap_off, uint8_t* __restrict__ chrom, uint32_t* __restrict__ pos,
    uint64_t* __restrict__ allele_off, uint32_t* __restrict__ ref_len, uint32_t* __restrict__ alt_len,
    uint64_t* __restrict__ ext_id, uint8_t* __restrict__ heap, uint32_t* __restrict__ rec_line,
    uint32_t* __restrict__ rec_alt) {
  __shared__ u32x4 s_text[kStage / 16];
  const Heap h = make_heap(text, text_bytes);
  for (size_t base = size_t(blockIdx.x) * kBlock; base < n_lines; base += size_t(gridDim.x) * kBlock) {
    const size_t last = base + kBlock < n_lines ? base + kBlock : n_lines;
    // the window only has to reach the end of the last line's ALT field
    const size_t s0 = lines[base].start;
    const avdb_vcf_line& Z = lines[last - 1];
    const size_t s1 = Z.start + Z.len;
    const Window w = stage_window(h, s0, s1, s_text);
    const size_t li = base + threadIdx.x;
    if (li < n_lines) {
      const avdb_vcf_line L = lines[li];
      if (L.n_rec) {
        if (w.staged)
          emit_line((lds_cp)(reinterpret_cast<const uint8_t*>(s_text) + (h.lo + L.start - w.a0)), L, li,
                    rec_off[li], heap_off[li], chrom, pos, allele_off, ref_len, alt_len, ext_id, heap,
                    rec_line, rec_alt);
        else
          emit_line((glb_cp)(text + L.start), L, li, rec_off[li], heap_off[li], chrom, pos, allele_off, ref_len,
                    alt_len, ext_id, heap, rec_line, rec_alt);
      }
    }
    __syncthreads();
  }
}

}  // namespace avdb

using namespace avdb;

// k_vcf_count + k_vcf_scan_blocks into a count workspace (layout: kCountWs*)
static int count_pass(const uint8_t* text, size_t text_bytes, void* ws, unsigned long long* total,
                      hipStream_t s, unsigned long long* commas = nullptr) {
  char* w = static_cast<char*>(ws);
  auto* wave = reinterpret_cast<uint32_t*>(w + kCountWsWave);
  auto* blk = reinterpret_cast<unsigned long long*>(w + kCountWsBlkOff);
  if (commas) AVDB_HIP_TRY(hipMemsetAsync(commas, 0, 8, s));
  hipLaunchKernelGGL(k_vcf_count, dim3(kVcfGrid), dim3(kBlock), 0, s, text, text_bytes, wave, commas);
  AVDB_LAUNCH_CHECK("k_vcf_count");
  hipLaunchKernelGGL(k_vcf_scan_blocks, dim3(1), dim3(kVcfGrid), 0, s, wave, blk, total);
  AVDB_LAUNCH_CHECK("k_vcf_scan_blocks");
  return AVDB_OK;
}

static size_t scan_temp_bytes(size_t n) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, static_cast<const unsigned long long*>(nullptr),
                                         static_cast<unsigned long long*>(nullptr), n);
  return (t + 255) & ~size_t(255);
}

extern "C" int avdb_vcf_workspace_size(size_t text_bytes, size_t n_lines, size_t* bytes) {
  (void)text_bytes;
  if (!bytes) return AVDB_EINVAL;
  // count workspace | line starts | scan temp
  *bytes = AVDB_VCF_COUNT_WORKSPACE_BYTES + ((8 * n_lines + 255) & ~size_t(255)) +
           scan_temp_bytes(n_lines + 1) + 256;
  return AVDB_OK;
}

extern "C" int avdb_vcf_count_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes,
                                    void* workspace, size_t workspace_bytes, uint64_t* n_newlines,
                                    void* stream) {
  if (!ctx || !n_newlines) { avdb_set_error("avdb_vcf_count_lines: null argument"); return AVDB_EINVAL; }
  if (!workspace || workspace_bytes < AVDB_VCF_COUNT_WORKSPACE_BYTES) {
    avdb_set_error("avdb_vcf_count_lines: workspace too small");
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (text_bytes == 0) return hipMemsetAsync(n_newlines, 0, 8, s) == hipSuccess ? AVDB_OK : AVDB_EHIP;
  return count_pass(text, text_bytes, workspace, reinterpret_cast<unsigned long long*>(n_newlines), s);
}

extern "C" int avdb_vcf_parse_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes,
                                    size_t n_lines, const void* line_counts, void* workspace,
                                    size_t workspace_bytes,
                                    avdb_vcf_line* lines, uint64_t* rec_off, uint64_t* heap_off,
                                    const avdb_vcf_opts* opts, void* stream) {
  if (!ctx || !lines || !rec_off || !heap_off) {
    avdb_set_error("avdb_vcf_parse_lines: null argument");
    return AVDB_EINVAL;
  }
  if (opts && opts->struct_size != sizeof(avdb_vcf_opts)) {
    avdb_set_error("avdb_vcf_parse_lines: avdb_vcf_opts.struct_size %u, this library expects %zu",
                   opts->struct_size, sizeof(avdb_vcf_opts));
    return AVDB_EINVAL;
  }
  if (opts && opts->chrom_map && opts->chrom_map->device != ctx->device) {
    avdb_set_error("avdb_vcf_parse_lines: chromosome map made for device %d", opts->chrom_map->device);
    return AVDB_EINVAL;
  }
  const ChromMapView cm = opts && opts->chrom_map ? opts->chrom_map->dev : ChromMapView{};
  const uint32_t min_fields = opts ? opts->min_fields : 0u;
  size_t need = 0;
  avdb_vcf_workspace_size(text_bytes, n_lines, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_vcf_parse_lines: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n_lines == 0) {  // rec_off[0] = heap_off[0] = 0 (the totals of no lines)
    AVDB_HIP_TRY(hipMemsetAsync(rec_off, 0, 8, s));
    AVDB_HIP_TRY(hipMemsetAsync(heap_off, 0, 8, s));
    return AVDB_OK;
  }
  auto* starts = reinterpret_cast<uint64_t*>(static_cast<char*>(workspace) + AVDB_VCF_COUNT_WORKSPACE_BYTES);
  void* tmp = reinterpret_cast<char*>(starts) + ((8 * n_lines + 255) & ~size_t(255));
  size_t tmp_bytes = scan_temp_bytes(n_lines + 1);
  const char* cw = static_cast<const char*>(line_counts);
  if (!cw) {  // recount into the front of this workspace (same cut as k_vcf_starts)
    const int rc = count_pass(text, text_bytes, workspace, nullptr, s);
    if (rc != AVDB_OK) return rc;
    cw = static_cast<const char*>(workspace);
  }
  hipLaunchKernelGGL(k_vcf_starts, dim3(kVcfGrid), dim3(kBlock), 0, s, text, text_bytes,
                     reinterpret_cast<const unsigned long long*>(cw + kCountWsBlkOff),
                     reinterpret_cast<const uint32_t*>(cw + kCountWsWave), n_lines, starts);
  AVDB_LAUNCH_CHECK("k_vcf_starts");
  auto* rc = reinterpret_cast<unsigned long long*>(rec_off);
  auto* hc = reinterpret_cast<unsigned long long*>(heap_off);
  AVDB_HIP_TRY(hipMemsetAsync(rc + n_lines, 0, 8, s));
  AVDB_HIP_TRY(hipMemsetAsync(hc + n_lines, 0, 8, s));
  const unsigned grid = stream_grid(n_lines, kBlock, 4096);
  hipLaunchKernelGGL(k_vcf_parse, dim3(grid), dim3(kBlock), 0, s, text, text_bytes, n_lines, starts,
                     lines, rc, hc, cm, min_fields);
  AVDB_LAUNCH_CHECK("k_vcf_parse");
  AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, rc, rc, n_lines + 1, s));
  AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, hc, hc, n_lines + 1, s));
  return AVDB_OK;
}

extern "C" int avdb_vcf_emit(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                             const avdb_vcf_line* lines, const uint64_t* rec_off,
                             const uint64_t* heap_off, uint8_t* chrom, uint32_t* pos,
                             uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len,
                             uint64_t* ext_id, uint8_t* heap, uint32_t* rec_line, uint32_t* rec_alt,
                             void* stream) {
  if (!ctx || !lines || !rec_off || !heap_off || !chrom || !pos || !allele_off || !ref_len ||
      !alt_len || !ext_id || !heap || !rec_line || !rec_alt) {
    avdb_set_error("avdb_vcf_emit: null argument");
    return AVDB_EINVAL;
  }
  if (n_lines == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const unsigned grid = stream_grid(n_lines, kBlock, 4096);
  hipLaunchKernelGGL(k_vcf_emit, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     text, text_bytes, n_lines, lines, rec_off, heap_off, chrom, pos, allele_off, ref_len,
                     alt_len, ext_id, heap, rec_line, rec_alt);
  AVDB_LAUNCH_CHECK("k_vcf_emit");
  return AVDB_OK;
}

extern "C" int avdb_vcf_count_text(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, void* workspace,
                                   size_t workspace_bytes, uint64_t* counts, void* stream) {
  if (!ctx || !counts) { avdb_set_error("avdb_vcf_count_text: null argument"); return AVDB_EINVAL; }
  if (!workspace || workspace_bytes < AVDB_VCF_COUNT_WORKSPACE_BYTES) {
    avdb_set_error("avdb_vcf_count_text: workspace too small");
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (text_bytes == 0) return hipMemsetAsync(counts, 0, 16, s) == hipSuccess ? AVDB_OK : AVDB_EHIP;
  auto* c = reinterpret_cast<unsigned long long*>(counts);
  return count_pass(text, text_bytes, workspace, c, s, c + 1);
}

static size_t tok_chunks(size_t text_bytes) { return (text_bytes + kTokChunk - 1) / kTokChunk; }

extern "C" int avdb_vcf_tokenize_workspace_size(size_t text_bytes, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  const size_t nc = tok_chunks(text_bytes);
  *bytes = 256 + 8 * nc + 2 * 24 * nc + 4 * nc + 16 * nc + 64;  // ticket | status | aggregates | prefixes | trace | clock
  return AVDB_OK;
}

extern "C" int avdb_vcf_tokenize(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, void* workspace,
                                 size_t workspace_bytes, size_t lines_cap, avdb_vcf_line* lines, uint64_t* rec_off,
                                 uint64_t* heap_off, size_t rec_cap, uint8_t* chrom, uint32_t* pos,
                                 uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len, uint64_t* ext_id,
                                 uint32_t* rec_line, uint32_t* rec_alt, size_t heap_cap, uint8_t* heap,
                                 uint64_t* totals, const avdb_vcf_opts* opts, void* stream) {
  if (!ctx || !totals || !rec_off || !heap_off || (lines_cap && !lines) ||
      (rec_cap && (!chrom || !pos || !allele_off || !ref_len || !alt_len || !ext_id || !rec_line || !rec_alt)) ||
      (heap_cap && !heap)) {
    avdb_set_error("avdb_vcf_tokenize: null argument");
    return AVDB_EINVAL;
  }
  if (opts && opts->struct_size != sizeof(avdb_vcf_opts)) {
    avdb_set_error("avdb_vcf_tokenize: avdb_vcf_opts.struct_size %u, this library expects %zu", opts->struct_size,
                   sizeof(avdb_vcf_opts));
    return AVDB_EINVAL;
  }
  if (opts && opts->chrom_map && opts->chrom_map->device != ctx->device) {
    avdb_set_error("avdb_vcf_tokenize: chromosome map made for device %d", opts->chrom_map->device);
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_vcf_tokenize_workspace_size(text_bytes, &need);
  if (!workspace || workspace_bytes < need || reinterpret_cast<uintptr_t>(workspace) % 8) {
    avdb_set_error("avdb_vcf_tokenize: 8-byte aligned workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  AVDB_HIP_TRY(hipMemsetAsync(totals, 0, 32, s));
  if (text_bytes == 0) {
    AVDB_HIP_TRY(hipMemsetAsync(rec_off, 0, 8, s));
    AVDB_HIP_TRY(hipMemsetAsync(heap_off, 0, 8, s));
    return AVDB_OK;
  }
  const size_t nc = tok_chunks(text_bytes);
  char* ws = static_cast<char*>(workspace);
  AVDB_HIP_TRY(hipMemsetAsync(ws, 0, 256 + 8 * nc, s));  // ticket + chunk status words
  TokArgs A;
  A.text = text;
  A.text_bytes = text_bytes;
  A.n_chunks = nc;
  A.lines_cap = lines_cap;
  A.rec_cap = rec_cap;
  A.heap_cap = heap_cap;
  A.lines = lines;
  A.rec_off = rec_off;
  A.heap_off = heap_off;
  A.chrom = chrom;
  A.pos = pos;
  A.allele_off = allele_off;
  A.ref_len = ref_len;
  A.alt_len = alt_len;
  A.ext_id = ext_id;
  A.heap = heap;
  A.rec_line = rec_line;
  A.rec_alt = rec_alt;
  A.totals = reinterpret_cast<unsigned long long*>(totals);
  A.ticket = reinterpret_cast<unsigned int*>(ws);
  A.status = reinterpret_cast<uint64_t*>(ws + 256);
  A.agg = A.status + nc;
  A.pre = A.agg + 3 * nc;
  A.trace = reinterpret_cast<uint32_t*>(A.pre + 3 * nc);
  A.clock = reinterpret_cast<uint64_t*>(A.trace + ((nc + 1) & ~size_t(1)));
  A.stuck = reinterpret_cast<uint64_t*>(ws + 64);  // 8 words in the 256-byte head, zeroed with the ticket
  AVDB_HIP_TRY(hipMemsetAsync(A.trace, 0, 4 * nc, s));
  A.cm = opts && opts->chrom_map ? opts->chrom_map->dev : ChromMapView{};
  A.min_fields = opts ? opts->min_fields : 0u;
  const size_t g = size_t(ctx->n_cu) * ctx->k0_blocks_per_cu;
  hipLaunchKernelGGL(k_vcf_tokenize, dim3(unsigned(g < nc ? g : nc)), dim3(kBlock), 0, s, A);
  AVDB_LAUNCH_CHECK("k_vcf_tokenize");
  return AVDB_OK;
}

// ---- chromosome map (ChromosomeMap.get, chromosome_map_parser.py:84-91) ----------
extern "C" int avdb_chrom_map_create(avdb_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, size_t n_keys,
                                     const uint8_t* codes, avdb_chrom_map** out) {
  if (!ctx || !out || (n_keys && (!keys || !key_off || !codes)) || n_keys >= (1u << 24)) {
    avdb_set_error("avdb_chrom_map_create: null argument or more than 2^24-1 keys");
    return AVDB_EINVAL;
  }
  *out = nullptr;
  avdb_chrom_map* m = new (std::nothrow) avdb_chrom_map();
  if (!m) return AVDB_ENOMEM;
  m->device = ctx->device;
  m->d_mem = nullptr;
  size_t slots = 16;
  while (slots < 2 * n_keys + 2) slots <<= 1;
  m->slot.assign(slots, 0);
  m->key_off.resize(n_keys + 1);
  m->code.assign(codes, codes + n_keys);
  const size_t total = n_keys ? key_off[n_keys] : 0;
  if (total >= (1ull << 32)) {
    delete m;
    avdb_set_error("avdb_chrom_map_create: keys too long");
    return AVDB_EINVAL;
  }
  m->keys.assign(keys, keys + total);
  m->keys.push_back(0);
  for (size_t k = 0; k <= n_keys; ++k) m->key_off[k] = uint32_t(key_off[k]);
  for (size_t k = 0; k < n_keys; ++k) {
    if (key_off[k + 1] < key_off[k] || key_off[k + 1] > total) {
      delete m;
      avdb_set_error("avdb_chrom_map_create: key_off not ascending");
      return AVDB_EINVAL;
    }
    const uint64_t h = fnv1a(m->keys.data() + key_off[k], uint32_t(key_off[k + 1] - key_off[k]));
    uint32_t q = uint32_t(h) & uint32_t(slots - 1);
    while (m->slot[q]) q = (q + 1) & uint32_t(slots - 1);  // duplicate keys: the first stays found first
    m->slot[q] = ((h >> 24) << 24) | uint64_t(k + 1);
  }
  if (ctx->device >= 0) {
    const size_t b_slot = 8 * slots, b_off = 4 * (n_keys + 1), b_code = n_keys + 8, b_keys = m->keys.size();
    const size_t o_off = b_slot, o_code = o_off + ((b_off + 7) & ~size_t(7)), o_keys = o_code + ((b_code + 7) & ~size_t(7));
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&m->d_mem, o_keys + b_keys);
    char* d = static_cast<char*>(m->d_mem);
    if (e == hipSuccess) e = hipMemcpy(d, m->slot.data(), b_slot, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + o_off, m->key_off.data(), b_off, hipMemcpyHostToDevice);
    if (e == hipSuccess && n_keys) e = hipMemcpy(d + o_code, m->code.data(), n_keys, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + o_keys, m->keys.data(), b_keys, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (m->d_mem) (void)hipFree(m->d_mem);
      delete m;
      avdb_set_error("avdb_chrom_map_create: %s", hipGetErrorString(e));
      return AVDB_EHIP;
    }
    m->dev = ChromMapView{reinterpret_cast<const uint64_t*>(d), reinterpret_cast<const uint8_t*>(d + o_keys),
                          reinterpret_cast<const uint32_t*>(d + o_off), reinterpret_cast<const uint8_t*>(d + o_code),
                          uint32_t(slots - 1)};
  } else {
    m->dev = ChromMapView{};
  }
  *out = m;
  return AVDB_OK;
}

extern "C" int avdb_chrom_map_destroy(avdb_chrom_map* m) {
  if (!m) return AVDB_OK;
  if (m->d_mem) {
    (void)hipSetDevice(m->device);
    (void)hipFree(m->d_mem);
  }
  delete m;
  return AVDB_OK;
}
