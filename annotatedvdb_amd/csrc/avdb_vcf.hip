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
//   (exclusive scans, avdb_scan.hpp: record and heap offsets per line)
//   k_vcf_emit     same staging; one lane per line: one record per ALT != '.',
//                  REF+ALT copied to the allele heap
// The records-only path without the count pass (avdb_vcf_parse_local /
// avdb_vcf_emit_local): k_vcf_parse_windows<true> writes each window's lines,
// records and allele bytes to slots of its own, two small scans give the windows'
// bases, and k_vcf_emit_local moves the slots to their places (no second read of
// the text).
// Only canonical text is resolved here; the rest is flagged (AVDB_VCF_*_HOST) for
// the host to resolve with Python's own coercion rules.
#include "avdb_fmt.hpp"
#include "avdb_vcfline.hpp"

#include "avdb_scan.hpp"

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
};

__device__ __forceinline__ Mask16 nl_mask16(uintptr_t a, const Heap& h, uintptr_t lo, uintptr_t end) {
  uint64_t m0 = 0, m1 = 0;
  if (a >= end) return Mask16{0, 0};
  uint64_t x, y;
  if (a >= h.lo && a + 16 <= h.hi) {
    const u32x4 v = __builtin_nontemporal_load(gptr<u32x4>(a));
    x = uint64_t(v[0]) | uint64_t(v[1]) << 32;
    y = uint64_t(v[2]) | uint64_t(v[3]) << 32;
  } else {
    x = text_word(a, h);
    y = text_word(a + 8, h);
  }
  m0 = zero_bytes_mask(x ^ kNL) & 0x8080808080808080ull;
  m1 = zero_bytes_mask(y ^ kNL) & 0x8080808080808080ull;
  if (a < lo) {
    const uint32_t sh = uint32_t(lo - a);  // 1..15 bytes before the range
    if (sh >= 8) { m0 = 0; m1 &= ~low_bytes_mask(sh - 8); }
    else m0 &= ~low_bytes_mask(sh);
  }
  if (a + 16 > end) {
    const uint32_t keep = uint32_t(end - a);  // 1..15 bytes inside the range
    if (keep <= 8) { m1 = 0; m0 &= low_bytes_mask(keep); }
    else m1 &= low_bytes_mask(keep - 8);
  }
  return Mask16{m0, m1};
}

constexpr int kNlUnroll = 4;                           // 16-byte lane loads in flight
constexpr uintptr_t kNlStep = 16 * kWave;              // bytes per wave load

// The parse pass's windows: each wave sub-chunk [t0, t1) is cut into windows of
// kParseWin bytes from t0; with a count workspace of avdb_vcf_count_workspace_size
// bytes the count pass also writes every window's newline count, and the parse
// pass then takes one workgroup per window and finds its line starts itself.
#ifndef AVDB_VCF_PARSE_WIN_KB
#define AVDB_VCF_PARSE_WIN_KB 24  // window size (A/B knob; a multiple of 4)
#endif
#ifndef AVDB_VCF_PARSE_OVER
#define AVDB_VCF_PARSE_OVER 1024  // bytes staged past a window (A/B knob; a multiple of 64)
#endif
#ifndef AVDB_VCF_PARSE_WAVES
#define AVDB_VCF_PARSE_WAVES 5    // launch-bounds minimum waves per SIMD of the window parse (A/B knob; 6 is
                                  // missed at 95 VGPRs and ran the same, profiles/k0_ab/r05_parse_waves_ab.log)
#endif
// (8.4 M dbSNP lines, the stage sized to the window: 20 / 24 / 28 KB windows with
// 4 KB of overhang 1.86 / 1.78 / 1.89 ms per tokenize — 24 KB is the largest that
// leaves five workgroups' LDS on a CU, against four at 28 KB; then a 1 KB overhang
// (26.7 KB of LDS) and 80 VGPRs (6 waves per SIMD, 20 B of spills) put six on a
// CU: 1.71 ms.  A line that runs more than 1 KB past its window parses from
// global memory.)
constexpr uint32_t kParseWin = AVDB_VCF_PARSE_WIN_KB * 1024;   // (a multiple of kNlUnroll * kNlStep)
constexpr uint32_t kParseOver = AVDB_VCF_PARSE_OVER;           // staged past a window (its last line)
static_assert(kParseWin % (kNlUnroll * kNlStep) == 0, "window / count step");

// What k_vcf_emit needs of a line, when no caller asked for the public 80-byte
// avdb_vcf_line table (avdb_vcf_parse_lines2 with lines == NULL): 32 bytes in the
// parse workspace instead of 80 written and read back (the tokenize-only path;
// the load path keeps the public table, which K5 reads).
struct VcfEmitRec {
  uint64_t start_chrom;  // line start | contig code << 56
  uint64_t ext_id;
  uint32_t pos, ref0, alt0, aend;  // REF field [ref0, alt0 - 1), ALT field [alt0, aend), relative to start
};
static_assert(sizeof(VcfEmitRec) == 32, "emit record");

__device__ __forceinline__ VcfEmitRec emit_rec(const avdb_vcf_line& L) {
  const uint32_t nfields = L.n_fields < 8 ? L.n_fields : 8;
  return VcfEmitRec{L.start | (uint64_t(L.chrom) << 56), L.ext_id, L.pos, L.field[3], L.field[4],
                    5 < nfields ? L.field[5] - 1 : L.len};
}

// ---- the count-free records path (avdb_vcf_parse_local / avdb_vcf_emit_local) ----
#ifndef AVDB_VCF_LOCAL_CAP
#define AVDB_VCF_LOCAL_CAP 1024  // line slots per parse window (lines >= 24 B on average; more: counted path)
#endif
constexpr uint32_t kLocalCap = AVDB_VCF_LOCAL_CAP;
static_assert(kLocalCap % kBlock == 0, "whole rounds of slots");
// The parse writes each window's records and allele bytes itself, from the text it
// has staged, to slots of the window's own (records at window * kLocalCap + the
// record's offset in the window, REF+ALT bytes at window * kLocalHeap + the heap
// offset in the window); the emit then only moves them to their final places
// (coalesced copies, no second read of the text).  A window with more records or
// heap bytes than its slots hold flags the overflow word (the counted path).
#ifndef AVDB_VCF_LOCAL_HEAP_KB
#define AVDB_VCF_LOCAL_HEAP_KB AVDB_VCF_PARSE_WIN_KB  // single-ALT lines never hold more allele bytes than text
#endif
constexpr uint32_t kLocalHeap = AVDB_VCF_LOCAL_HEAP_KB * 1024;
static_assert(kLocalHeap % 16 == 0, "heap slots keep 16-byte alignment");
struct LocalWin {  // one parse window's lines, records and heap bytes
  uint32_t lines, recs;
  uint64_t heap;
};
struct LocalRec {  // one record in its window's slots
  uint64_t ext_id;
  uint32_t pos, ref_len, alt_len, hoff;  // hoff: REF's offset in the window's heap slots
  uint32_t alt;                          // ALT index in the line (rec_alt)
  uint16_t line;                         // line index in the window (< kLocalCap)
  uint8_t chrom, pad;
};
static_assert(sizeof(LocalRec) == 32, "record slot");
struct LocalOut {
  LocalWin* win;               // [windows]
  LocalRec* rec;               // [windows * kLocalCap]
  uint8_t* heap;               // [windows * kLocalHeap]
  uint2* cnt;                  // [windows * kLocalCap] (records, heap bytes) per line
  unsigned long long* overflow;  // windows with more lines, records or heap bytes than their slots
};

// the line's public record or its emit record, one of them (the other NULL)
__device__ __forceinline__ void put_line(avdb_vcf_line* lines, VcfEmitRec* erec, size_t li, const avdb_vcf_line& L) {
  if (lines) lines[li] = L;
  else erec[li] = emit_rec(L);
}

__global__ __launch_bounds__(kBlock) void k_vcf_count(const uint8_t* __restrict__ text,
                                                      size_t text_bytes,
                                                      uint32_t* __restrict__ wave_cnt,
                                                      uint32_t* __restrict__ win_cnt, uint32_t wps) {
  const Heap h = make_heap(text, text_bytes);
  const size_t gw = size_t(blockIdx.x) * kVcfWaves + threadIdx.x / kWave;
  size_t t0, t1;
  wave_range(text_bytes, gw, &t0, &t1);
  uint32_t c = 0;
  uint32_t wk = 0;
  for (size_t w0 = t0; w0 < t1; w0 += kParseWin, ++wk) {  // (one trip without windows: kParseWin is
    const size_t w1 = win_cnt && w0 + kParseWin < t1 ? w0 + kParseWin : t1;  //  then the whole sub-chunk)
    const uintptr_t lo = h.lo + w0, end = h.lo + w1;
    uint32_t cw = 0;
    for (uintptr_t a = (lo & ~uintptr_t(15)) + 16 * __lane_id(); a < end; a += kNlUnroll * kNlStep) {
      Mask16 m[kNlUnroll];
#pragma unroll
      for (int u = 0; u < kNlUnroll; ++u) m[u] = nl_mask16(a + u * kNlStep, h, lo, end);
#pragma unroll
      for (int u = 0; u < kNlUnroll; ++u) cw += uint32_t(__popcll(m[u].m0) + __popcll(m[u].m1));
    }
    if (win_cnt) {
      uint32_t x = cw;
      for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, kWave);
      if (__lane_id() == 0 && wk < wps) win_cnt[gw * wps + wk] = x;
    }
    c += cw;
    if (!win_cnt) break;
  }
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
  if (__lane_id() == 0) wave_cnt[gw] = c;
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
                                                      VcfEmitRec* __restrict__ erec,
                                                      unsigned long long* __restrict__ rec_cnt,
                                                      unsigned long long* __restrict__ heap_cnt,
                                                      ChromMapView cm, uint32_t min_fields) {
  __shared__ u32x4 s_text[kStage / 16];
  const Heap h = make_heap(text, text_bytes);
  for (size_t base = size_t(blockIdx.x) * kBlock; base < n_lines; base += size_t(gridDim.x) * kBlock) {
    const size_t last = base + kBlock < n_lines ? base + kBlock : n_lines;
    const size_t s0 = starts[base];
    const size_t s1 = last < n_lines ? starts[last] : text_bytes;
    const Window w = stage_window<kBlock>(h, s0, s1, s_text);
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
      put_line(lines, erec, li, L);
      rec_cnt[li] = recs;
      heap_cnt[li] = hbytes;
    }
    __syncthreads();  // the window is reused by the next trip
  }
}

// ---- k_vcf_parse_windows: the parse pass without the line-starts pass ---------
// One workgroup per window (kParseWin bytes of a count-pass sub-chunk, whose
// newline count the count pass wrote).  The window is staged in LDS with the byte
// before it and kParseOver bytes after it; newline bitmaps (64 bytes per bitmap
// word, two adjacent words per thread, so the block scan numbers lines in text
// order) give the starts of the lines that begin in it; the end of its last line is
// the first '\n' at or after its last byte; then one lane per line parses it
// (parse_line, as k_vcf_parse), 256 lines a round.  Lines start at byte 0 and
// after every '\n' except a final one.
static_assert(kParseWin % 64 == 0 && kParseWin / 64 + 2 <= 2 * kBlock, "window bitmap words");
// the window kernel's own stage: the window, its overhang and the 16-byte
// alignment slack on both sides (LDS per workgroup decides how many fit a CU)
constexpr uint32_t kParseStage = kParseWin + kParseOver + 48;
static_assert(kParseStage <= kStage, "window stage");
constexpr uint32_t kParseStage64 = (kParseStage + 63) & ~63u;  // whole 64-byte bitmap blocks
static_assert(kParseStage64 / 64 <= 2 * kBlock, "two bitmap blocks per thread");

__device__ __forceinline__ uint32_t byte_bits8(uint64_t w, uint64_t pat) {  // bit k: byte k of w is pat's byte
  const uint64_t m = zero_bytes_mask(w ^ pat) & kHiBits;
  return uint32_t(((m >> 7) * 0x0102040810204080ull) >> 56);
}
__device__ __forceinline__ uint32_t nl_bits8(uint64_t w) { return byte_bits8(w, kNL); }

// fields_swar from the window's tab bitmap (bit t of tab[t / 64]: stage byte t is
// a tab): the line is stage bytes [sp, sp + len).  Each field start is a ctz on a
// register word; a line of ~100 bytes spans two or three bitmap words, where the
// SWAR scan reads and tests every 8-byte word of the line.
__device__ __forceinline__ uint32_t fields_bits(lds_cp64 tab, uint32_t sp, uint32_t len, avdb_vcf_line& L) {
  const uint32_t e = sp + len;
  const uint32_t we = (e + 63) >> 6;  // words [sp / 64, we) hold the line
  uint32_t wi = sp >> 6;
  auto clip = [e](uint32_t w, uint64_t x) {  // bits of word w at stage bytes < e
    const uint32_t hi = e - 64 * w;
    return hi >= 64 ? x : x & ((uint64_t(1) << hi) - 1);
  };
  uint64_t m = wi < we ? clip(wi, tab[wi] & (~uint64_t(0) << (sp & 63))) : 0ull;
  uint32_t nf = 1;
#pragma unroll
  for (int f = 1; f <= 8; ++f) {
    while (!m && wi + 1 < we) {
      ++wi;
      m = clip(wi, tab[wi]);
    }
    if (m) {
      const uint32_t t = 64 * wi + uint32_t(__builtin_ctzll(m)) - sp;
      if (f < 8) L.field[f] = t + 1;
      else L.field_end8 = t;
      m &= m - 1;
      ++nf;
    }
  }
  if (nf > 8) {  // past INFO: only the count matters
    nf += uint32_t(__popcll(m));
    while (wi + 1 < we) {
      ++wi;
      nf += uint32_t(__popcll(clip(wi, tab[wi])));
    }
  }
  return nf;
}

// bytes [p, p + 16) of the stage as two registers (bytes at and past `end` read
// as 0; words past the stage read as 0: LDS reads outside the allocation return 0)
__device__ __forceinline__ void stage16(lds_cp64 lw, uint32_t p, uint32_t end, uint64_t* y0, uint64_t* y1) {
  const uint32_t k = p >> 3, sh = 8 * (p & 7);
  const uint64_t w0 = lw[k], w1 = lw[k + 1], w2 = lw[k + 2];
  uint64_t a = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  uint64_t b = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  const uint32_t n = end > p ? end - p : 0u;
  if (n < 16) {
    b &= n > 8 ? low_bytes_mask(n - 8) : 0ull;
    a &= low_bytes_mask(n < 8 ? n : 8);
  }
  *y0 = a;
  *y1 = b;
}

// The INFO refSNP of a staged line, INFO = stage bytes [A, B): the last entry whose
// key is exactly "RS" (dict(...) keeps the last; vcf_parser.py:155-169), as the
// SWAR scan of parse_line_with decides it.  Entries after a ';' are 4-byte
// windows ";RS=" / ";RS;" at every byte of the INFO words, with the bytes outside
// [A, B) zeroed (so no window reaches past INFO): one v_alignbyte and two compares
// per byte instead of five byte-equality masks per word.  The entry at the INFO
// start and a bare ";RS" ending INFO are checked once.  Returns 0 (no "RS"
// entry), kRsFound | the number, or kRsFound | kRsHost (a value the reference
// coerces to something other than rs<int>).
constexpr uint64_t kRsFound = uint64_t(1) << 62, kRsHost = uint64_t(1) << 63;
// an "RS=" entry's value, stage bytes [vs, next ';' or B): all digits, 1..18 of
// them, gives kRsFound | the number; anything else kRsFound | kRsHost
__device__ __forceinline__ uint64_t info_rs_value(lds_cp64 lw, lds_cp stage, uint32_t vs, uint32_t B) {
  const uint32_t vmax = B - vs;
  uint64_t y0, y1, v = 0;
  bool ok = false;
  stage16(lw, vs, B, &y0, &y1);
  const uint64_t nd0 = nondigit_mask(y0), nd1 = nondigit_mask(y1);
  const uint32_t nd = nd0 ? uint32_t(__builtin_ctzll(nd0)) >> 3 : (nd1 ? 8u + (uint32_t(__builtin_ctzll(nd1)) >> 3) : 16u);
  if (nd < 16 || vmax <= 16) {
    const uint32_t n = nd < vmax ? nd : vmax;
    const bool term = n == vmax || (n < 16 && (((n < 8 ? y0 >> (8 * n) : y1 >> (8 * (n - 8))) & 0xFF) == ';'));
    if (term && n >= 1) v = decimal16(y0, y1, n, &ok);
  } else {  // 16 digits and more: the byte loop (<= 18 digits)
    uint32_t n = 0;
    while (n < vmax && stage[vs + n] != ';') ++n;
    ok = n <= 18;
    for (uint32_t q = 0; ok && q < n; ++q) {
      ok = is_digit(stage[vs + q]);
      v = v * 10 + (stage[vs + q] - '0');
    }
  }
  return ok && v >= 1 ? (kRsFound | v) : (kRsFound | kRsHost);
}

__device__ __noinline__ uint64_t info_rs_staged(lds_cp64 lw, lds_cp stage, uint32_t A, uint32_t B) {
  int32_t at = -1;  // stage offset of the last entry's 'R'
  bool val = false;
  if (B >= A + 4) {
    auto masked = [A, B](uint32_t k, uint64_t w) {
      const int32_t lo = int32_t(A) - int32_t(8 * k), hi = int32_t(B) - int32_t(8 * k);
      if (lo > 0) w &= lo >= 8 ? 0ull : ~low_bytes_mask(uint32_t(lo));
      if (hi < 8) w &= hi > 0 ? low_bytes_mask(uint32_t(hi)) : 0ull;
      return w;
    };
    const uint32_t k0 = A >> 3, k1 = (B - 4) >> 3;  // words holding the ';' of a window [p, p + 4), p + 4 <= B
    uint64_t x = masked(k0, lw[k0]);
    for (uint32_t k = k0; k <= k1; ++k) {
      const uint64_t nx = masked(k + 1, lw[k + 1]);
      const uint32_t x0 = uint32_t(x), x1 = uint32_t(x >> 32), n0 = uint32_t(nx);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = j < 4 ? __builtin_amdgcn_alignbyte(x1, x0, j) : __builtin_amdgcn_alignbyte(n0, x1, j - 4);
        const bool eq = w == 0x3D53523Bu;  // ";RS="
        if (eq || w == 0x3B53523Bu) {      // ";RS;"
          at = int32_t(8 * k) + j + 1;
          val = eq;
        }
      }
      x = nx;
    }
  }
  uint64_t y0, y1;
  if (B >= A + 3) {  // a bare "RS" ending INFO is its last entry
    stage16(lw, B - 3, B, &y0, &y1);
    if ((y0 & 0xFFFFFFull) == 0x53523Bull) {
      at = int32_t(B) - 2;
      val = false;
    }
  }
  if (at < 0 && B >= A + 2) {  // the first entry: "RS=", "RS;" or all of INFO "RS"
    stage16(lw, A, B, &y0, &y1);
    const uint64_t t = y0 & 0xFFFFFFull;
    if (t == 0x3D5352ull || t == 0x3B5352ull || (B == A + 2 && t == 0x5352ull)) {
      at = int32_t(A);
      val = t == 0x3D5352ull;
    }
  }
  if (at < 0) return 0;
  return val ? info_rs_value(lw, stage, uint32_t(at) + 3, B) : (kRsFound | kRsHost);
}

// "RS" entry candidates of the stage, found by the whole workgroup in the bitmap
// pass: bit j set when word x (nx the next word) holds [';' or tab] 'R' 'S' at
// bytes j .. j + 2 — a possible "RS" / "RS=..." INFO entry starting at byte j + 1;
// the byte after it decides the kind when the candidate is placed in its line
__device__ __forceinline__ uint32_t rs_cand_bits8(uint64_t x, uint64_t nx) {
  const uint64_t v1 = (x >> 8) | (nx << 56), v2 = (x >> 16) | (nx << 48);
  const uint64_t m = (bytes_eq_mask(x, ';') | bytes_eq_mask(x, '\t')) & bytes_eq_mask(v1, 'R') &
                     bytes_eq_mask(v2, 'S');
  return uint32_t((((m & kHiBits) >> 7) * 0x0102040810204080ull) >> 56);
}

// exclusive block scan of one u32 per thread (kBlock threads); *total = sum
__device__ __forceinline__ uint32_t block_excl32(uint32_t v, uint32_t* s_w, uint32_t* total) {
  const uint32_t lane = __lane_id(), wv = threadIdx.x / kWave;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t u = __shfl_up(x, d, kWave);
    if (lane >= uint32_t(d)) x += u;
  }
  if (lane == kWave - 1) s_w[wv] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kVcfWaves; ++w) {
    const uint32_t t = s_w[w];
    if (w < wv) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// (LOCAL) one line's records into its window's record slots and its REF+ALT bytes
// into the window's heap slots at window-local heap offset h (the rows emit_line
// writes, without their final offsets)
template <class CP>
__device__ __forceinline__ void slot_line(CP s, const VcfEmitRec& E, uint16_t line, LocalRec* __restrict__ rs,
                                          uint8_t* __restrict__ heap, uint32_t h) {
  const uint32_t rlen = E.alt0 - 1 - E.ref0;
  const CP ref = s + E.ref0;
  const CP alt = s + E.alt0;
  const uint32_t an = E.aend - E.alt0;
  const uint8_t cc = uint8_t(E.start_chrom >> 56);
  Out<true> hs(heap, h);
  uint32_t ai = 0;
  for (uint32_t a0 = 0; a0 <= an; ++ai) {
    const uint32_t a1 = a0 + swar_find(alt + a0, an - a0, [](uint64_t x) { return bytes_eq_mask(x, ','); });
    const uint32_t al = a1 - a0;
    if (!(al == 1 && alt[a0] == '.')) {
      LocalRec R;
      R.ext_id = E.ext_id;
      R.pos = E.pos;
      R.ref_len = rlen;
      R.alt_len = al;
      R.hoff = h;
      R.alt = ai;
      R.line = line;
      R.chrom = cc;
      R.pad = 0;
      *rs++ = R;
      hs.bytes(ref, rlen);
      hs.bytes(alt + a0, al);
      h += rlen + al;
    }
    a0 = a1 + 1;
  }
  hs.finish();
}

// LOCAL (the records-only path without the count pass, avdb_vcf_parse_local): no
// line numbers are known, so a window writes its lines' record / heap offsets in the
// window to its line slots (window * kLocalCap + its line), their records and allele
// bytes to its record and heap slots (slot_line), and its line / record / heap totals
// to LocalWin; a window with more lines, records or allele bytes than its slots
// flags the overflow word.
template <bool LOCAL>
__global__ __launch_bounds__(kBlock, AVDB_VCF_PARSE_WAVES) void k_vcf_parse_windows(const uint8_t* __restrict__ text, size_t text_bytes,
                                                              size_t n_lines,
                                                              const unsigned long long* __restrict__ blk_off,
                                                              const uint32_t* __restrict__ wave_cnt,
                                                              const uint32_t* __restrict__ win_cnt, uint32_t wps,
                                                              avdb_vcf_line* __restrict__ lines,
                                                              VcfEmitRec* __restrict__ erec,
                                                              unsigned long long* __restrict__ rec_cnt,
                                                              unsigned long long* __restrict__ heap_cnt,
                                                              ChromMapView cm, uint32_t min_fields, LocalOut lo_out) {
  __shared__ u32x4 s_text[kParseStage64 / 16];
  __shared__ uint64_t s_tab[kParseStage64 / 64];  // tab bitmap of the staged bytes
  __shared__ uint32_t s_start[kBlock + 1];  // line starts of the round, relative to the window start
  __shared__ uint64_t s_rs[kBlock];         // the round's INFO refSNP results (info_rs_staged)
  __shared__ uint32_t s_w[kVcfWaves];
  __shared__ uint32_t s_wp[kVcfWaves];      // the round's pending INFO scans per wave
  __shared__ uint32_t s_tail;               // (first '\n' at or after w1 - 1) + 1 - w0
  __shared__ uint32_t s_lr[LOCAL ? kVcfWaves : 1], s_lh[LOCAL ? kVcfWaves : 1];  // (LOCAL) the round's per-wave sums
  const Heap h = make_heap(text, text_bytes);
  const size_t nb = text_bytes;
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid / kWave;
  const size_t gw = blockIdx.x / wps;
  const uint32_t wk = blockIdx.x % wps;
  size_t t0, t1;
  wave_range(nb, gw, &t0, &t1);
  const size_t w0 = t0 + size_t(wk) * kParseWin;
  if (w0 >= t1) {  // (uniform)
    if (LOCAL && tid == 0) lo_out.win[blockIdx.x] = LocalWin{0, 0, 0};
    return;
  }
  const size_t w1 = w0 + kParseWin < t1 ? w0 + kParseWin : t1;
  // lines starting before w0: 1 + the newlines in [0, w0 - 1)
  size_t li0 = 0;
  if (!LOCAL && w0) {
    unsigned long long k = blk_off[gw / kVcfWaves];
    for (size_t w = (gw / kVcfWaves) * kVcfWaves; w < gw; ++w) k += wave_cnt[w];
    for (uint32_t j = 0; j < wk; ++j) k += win_cnt[gw * wps + j];
    li0 = 1 + k - (text[w0 - 1] == '\n' ? 1u : 0u);
  }
  const lds_cp64 lw = (lds_cp64)(reinterpret_cast<const uint64_t*>(s_text));
  const size_t q0 = w0 ? w0 - 1 : 0;  // newline positions [q0, w1 - 1) start this window's lines
  // ---- stage [q0, w1 + kParseOver) ----
  const uintptr_t a0 = (h.lo + q0) & ~uintptr_t(15);
  const uintptr_t wend = h.lo + (w1 + kParseOver < nb ? w1 + kParseOver : nb);
  const uint32_t n16 = uint32_t((wend - a0 + 15) / 16);
  stage_copy<(kParseStage64 / 16 + kBlock - 1) / kBlock, kBlock>(s_text, a0, n16, h);
  __syncthreads();
  // ---- newline bitmaps of [q0, w1 - 1); the tab bitmap of the whole stage ----
  const uint32_t o_lo = uint32_t(h.lo + q0 - a0), o_hi = uint32_t(h.lo + w1 - 1 - a0);
  const uint32_t nblk = w1 - 1 > q0 ? (o_hi + 63) / 64 : 0u;
  const uint32_t nstage = (16 * n16 + 63) / 64;
  uint64_t bm[2] = {0, 0}, rsc[2] = {0, 0};
  uint32_t cnt = 0;
  uint32_t* s_rsc = reinterpret_cast<uint32_t*>(s_rs);  // the window's "RS" candidate per line (one round)
  s_rsc[tid] = 0;  // (read after the block scans' barriers)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t b = 2 * tid + k;
    if (b < nstage) {
      uint64_t m = 0, t = 0, c = 0;
      uint64_t w = lw[8 * b];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t nw = lw[8 * b + q + 1];
        m |= uint64_t(nl_bits8(w)) << (8 * q);
        t |= uint64_t(byte_bits8(w, kTab)) << (8 * q);
        c |= uint64_t(rs_cand_bits8(w, nw)) << (8 * q);
        w = nw;
      }
      s_tab[b] = t;
      rsc[k] = c;
      if (b >= nblk) continue;
      const uint32_t blo = 64 * b;
      if (o_lo > blo) m &= o_lo - blo >= 64 ? 0ull : ~0ull << (o_lo - blo);
      if (o_hi < blo + 64) m &= o_hi <= blo ? 0ull : ~0ull >> (64 - (o_hi - blo));
      bm[k] = m;
      cnt += uint32_t(__popcll(m));
    }
  }
  uint32_t T;
  const uint32_t pref = block_excl32(cnt, s_w, &T);
  const uint32_t first = w0 == 0 ? 1u : 0u;  // line 0 starts at byte 0
  T += first;
  if (!T) {  // (uniform; no line starts here)
    if (LOCAL && tid == 0) lo_out.win[blockIdx.x] = LocalWin{0, 0, 0};
    return;
  }
  if (LOCAL && T > kLocalCap) {  // (uniform) the caller takes the counted path
    if (tid == 0) {
      lo_out.win[blockIdx.x] = LocalWin{0, 0, 0};
      atomicAdd(lo_out.overflow, 1ull);
    }
    return;
  }
  // ---- the end of the window's last line: first '\n' at or after w1 - 1 ----
  if (wv == 0) {
    size_t q = w1 - 1;
    uint32_t found = 0;
    const uint32_t ob = uint32_t(h.lo + q - a0), oe = uint32_t(wend - a0);
    for (uint32_t o = ob & ~7u; o < oe && !found; o += 8 * kWave) {  // in the staged overhang
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
    for (uintptr_t ga = wend & ~uintptr_t(7); !found && ga < h.hi; ga += 8 * kWave) {  // past it
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
    if (lane == 0) s_tail = uint32_t((found ? q + 1 : nb + 1) - w0);
  }
  // ---- parse: rounds of kBlock lines ----
  const uint32_t rounds = (T + kBlock - 1) / kBlock;
  // ---- a one-round window: each line's last "RS" entry candidate (stage offset of
  // its ';' / tab << 2 | kind: 1 "RS=", 2 bare, 3 resolve by scanning) ----
  if (rounds == 1) {
    __syncthreads();  // (s_tail)
    const uint32_t tail = uint32_t(w0 + s_tail - (a0 - h.lo));  // stage end of the window's last line
    const lds_cp stage = (lds_cp)(reinterpret_cast<const uint8_t*>(s_text));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint64_t m = rsc[k];
      while (m) {
        const uint32_t bit = uint32_t(__builtin_ctzll(m));
        m &= m - 1;
        const uint32_t p = 64 * (2 * tid + k) + bit;
        if (p >= tail) break;
        const uint64_t below = (uint64_t(1) << bit) - 1;
        const uint32_t nls = pref + (k ? uint32_t(__popcll(bm[0])) : 0u) + uint32_t(__popcll(bm[k] & below));
        const int32_t line = int32_t(first + nls) - 1;
        if (line < 0 || line >= int32_t(T)) continue;
        // the byte after "RS": '=' an entry with a value, ';' / tab / '\n' a bare one; a
        // byte below '!' (space, '\r', NUL ...: whitespace rstrip may remove) the line's
        // own scan decides; anything else ("RSPOS", ...) is no "RS" entry
        const uint8_t e = stage[p + 3];
        const uint32_t kind = e == '=' ? 1u : ((e == ';' || e == '\t' || e == '\n') ? 2u : (e < 0x21 ? 3u : 0u));
        if (kind) atomicMax(&s_rsc[line], (p << 2) | kind);
      }
    }
  }
  uint32_t run_r = 0;  // (LOCAL) records and heap bytes of the window's earlier rounds
  uint64_t run_h = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    const uint32_t lo = kBlock * r, hi = lo + kBlock;
    if (r == 0 && first && tid == 0) s_start[0] = 0;
    uint32_t idx = first + pref;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint64_t m = bm[k];
      while (m && idx <= hi) {
        const uint32_t bit = uint32_t(__builtin_ctzll(m));
        m &= m - 1;
        if (idx >= lo) s_start[idx - lo] = uint32_t(a0 - h.lo - w0) + 64 * (2 * tid + k) + bit + 1;
        ++idx;
      }
    }
    if (tid == 0 && T <= hi) s_start[T - lo] = s_tail;
    __syncthreads();
    const size_t li = LOCAL ? size_t(blockIdx.x) * kLocalCap + lo + tid : li0 + lo + tid;
    const bool live = lo + tid < T && (LOCAL || li < n_lines);
    avdb_vcf_line L;
    uint64_t recs = 0, hbytes = 0;
    uint32_t info_item = 0;  // a pending INFO: stage offset | length << 15
    if (live) {
      L.start = w0 + s_start[tid];
      size_t nl = w0 + s_start[tid + 1] - 1;  // its newline, or the text end
      if (nl < L.start || nl > nb) nl = L.start;  // (never expected: starts increase)
      const uint32_t raw = uint32_t(nl - L.start);
      const uint32_t mis = uint32_t((h.lo + L.start) & 7);
      if (h.lo + nl <= wend) {
        const uint8_t* ls = reinterpret_cast<const uint8_t*>(s_text) + (h.lo + L.start - a0);
        const lds_cp64 lw2 = (lds_cp64)(reinterpret_cast<const uint64_t*>(ls - mis));
        const uint32_t sp = uint32_t(h.lo + L.start - a0);
        const lds_cp64 tb = (lds_cp64)(reinterpret_cast<const uint64_t*>(s_tab));
        parse_line_with<true>([tb, sp](uint32_t n, avdb_vcf_line& l) { return fields_bits(tb, sp, n, l); },
                              (lds_cp)ls, [lw2](uint32_t k) { return lw2[k]; }, mis, raw, L, recs, hbytes, cm,
                              min_fields);
        if (L.pad[0] == kInfoPending) {  // INFO = stage bytes [A, B)
          const uint32_t A = sp + L.field[7], B = sp + L.field_end8;
          bool done = false;
          uint64_t rs = 0;
          if (rounds == 1) {  // the line's last candidate decides, when it lies in INFO
            const uint32_t c = s_rsc[tid], q = c >> 2, kind = c & 3u;
            if (c == 0 || q + 1 < A) {
              done = true;  // no "RS" entry in INFO
            } else if (kind != 3u && q + 3 <= B) {
              rs = kind == 1u ? info_rs_value(lw, (lds_cp)(reinterpret_cast<const uint8_t*>(s_text)), q + 4, B)
                              : (kRsFound | kRsHost);
              done = true;
            }
          }
          if (done) {
            L.pad[0] = 0;
            if (rs & kRsFound) {
              L.flags |= AVDB_VCF_INFO_RS;
              if (rs & kRsHost) L.flags |= AVDB_VCF_EXT_HOST;
              else L.ext_id = rs & (kRsFound - 1);
            }
          } else {  // a later round or a candidate past INFO: the gathered scan
            info_item = A | ((B - A) << 15);
          }
        }
      } else {
        const uintptr_t la = h.lo + L.start - mis;
        parse_line((glb_cp)(text + L.start), [la, h](uint32_t k) { return heap_word(la + 8 * size_t(k), h); }, mis,
                   raw, L, recs, hbytes, cm, min_fields);
      }
    }
    // (LOCAL) each line's records / heap bytes within the window: wave sums here,
    // the waves below it after the barrier that follows (no barrier of its own).
    // Lines up to 2^23 records / heap bytes and windows below 2^32 heap bytes, else
    // the counted path.
    uint32_t xr = 0, xh = 0;
    if constexpr (LOCAL) {
      if ((recs | hbytes) >> 23) atomicAdd(lo_out.overflow, 1ull);
      xr = wave_incl_sum(uint32_t(recs));
      xh = wave_incl_sum(uint32_t(hbytes));
      if (lane == kWave - 1) {
        s_lr[wv] = xr;
        s_lh[wv] = xh;
      }
    }
    // the round's pending INFO scans, gathered into the first lanes of the workgroup
    // (a wave scans INFO once for its lanes that need it, instead of every wave for
    // the ~40 % of its lines without an rs ID)
    const uint64_t pend = __ballot(info_item != 0);
    if (lane == 0) s_wp[wv] = uint32_t(__popcll(pend));
    __syncthreads();  // (after it s_start and s_rs are free: this round's starts and candidates are read)
    uint32_t pr = 0, ph = 0;  // (LOCAL) the line's record / heap offset within the window
    if constexpr (LOCAL) {
      uint32_t br = 0, bh = 0, tr = 0, th = 0;
#pragma unroll
      for (uint32_t w = 0; w < kVcfWaves; ++w) {
        const uint32_t c = s_lr[w], d = s_lh[w];
        if (w < wv) {
          br += c;
          bh += d;
        }
        tr += c;
        th += d;
      }
      pr = run_r + br + xr - uint32_t(recs);
      ph = uint32_t(run_h) + bh + xh - uint32_t(hbytes);
      run_r += tr;
      run_h += th;
    }
    uint32_t n_pend = 0, slot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kVcfWaves; ++w) {
      const uint32_t c = s_wp[w];
      if (w < wv) slot += c;
      n_pend += c;
    }
    slot += uint32_t(__popcll(pend & ((uint64_t(1) << lane) - 1)));
    if (n_pend) {  // (uniform)
      if (info_item) s_start[slot] = info_item;
      __syncthreads();
      if (tid < n_pend) {
        const uint32_t it = s_start[tid], A = it & 0x7FFFu;
        s_rs[tid] = info_rs_staged(lw, (lds_cp)(reinterpret_cast<const uint8_t*>(s_text)), A, A + (it >> 15));
      }
      __syncthreads();
    }
    if (live) {
      if (info_item) {
        const uint64_t rs = s_rs[slot];
        L.pad[0] = 0;
        if (rs & kRsFound) {
          L.flags |= AVDB_VCF_INFO_RS;
          if (rs & kRsHost) L.flags |= AVDB_VCF_EXT_HOST;
          else L.ext_id = rs & (kRsFound - 1);
        }
      }
      if constexpr (LOCAL) {
        lo_out.cnt[li] = make_uint2(pr, ph);
        if (recs) {
          if (pr + recs > kLocalCap || ph + hbytes > kLocalHeap) {
            atomicAdd(lo_out.overflow, 1ull);
          } else {
            const VcfEmitRec E = emit_rec(L);
            LocalRec* rs = lo_out.rec + size_t(blockIdx.x) * kLocalCap + pr;
            uint8_t* hs = lo_out.heap + size_t(blockIdx.x) * kLocalHeap;
            const uint16_t ln = uint16_t(lo + tid);
            if (h.lo + L.start + E.aend <= wend)
              slot_line((lds_cp)(reinterpret_cast<const uint8_t*>(s_text) + (h.lo + L.start - a0)), E, ln, rs, hs, ph);
            else
              slot_line((glb_cp)(text + L.start), E, ln, rs, hs, ph);
          }
        }
      } else {
        put_line(lines, erec, li, L);
        rec_cnt[li] = recs;
        heap_cnt[li] = hbytes;
      }
    }
    if (r + 1 < rounds) __syncthreads();  // s_start is refilled by the next round
  }
  if constexpr (LOCAL) {
    if (tid == 0) {
      if (run_h >> 32) atomicAdd(lo_out.overflow, 1ull);
      lo_out.win[blockIdx.x] = LocalWin{T, run_r, run_h};
    }
  }
}

// (Rendering the allele heap through an LDS image of the tile's heap span with a
// coalesced flush, as K7 does for its text, measured slower: 0.66 vs 0.60 ms for
// 8.4 M lines — the pass is bound by re-staging the text, not by these stores.)
template <class CP>
__device__ __forceinline__ void emit_line(CP s, const VcfEmitRec& E, size_t li,
                                          uint64_t r, uint64_t h, uint8_t* __restrict__ chrom,
                                          uint32_t* __restrict__ pos, uint64_t* __restrict__ allele_off,
                                          uint32_t* __restrict__ ref_len, uint32_t* __restrict__ alt_len,
                                          uint64_t* __restrict__ ext_id, uint8_t* __restrict__ heap,
                                          uint32_t* __restrict__ rec_line, uint32_t* __restrict__ rec_alt) {
    const uint32_t rend = E.alt0 - 1;
    const uint32_t aend = E.aend;
    const CP ref = s + E.ref0;
    const uint32_t rlen = rend - E.ref0;
    const CP alt = s + E.alt0;
    const uint32_t an = aend - E.alt0;
    const uint8_t cc = uint8_t(E.start_chrom >> 56);
    // ALTs found with SWAR comma scans; the heap bytes leave through the 8-byte
    // register sink (this lane's records are contiguous in the heap)
    Out<true> hs(heap, h);
    uint32_t ai = 0;
    for (uint32_t a0 = 0; a0 <= an; ++ai) {
      const uint32_t a1 = a0 + swar_find(alt + a0, an - a0, [](uint64_t x) { return bytes_eq_mask(x, ','); });
      const uint32_t al = a1 - a0;
      if (!(al == 1 && alt[a0] == '.')) {
        chrom[r] = cc;
        pos[r] = E.pos;
        allele_off[r] = h;
        ref_len[r] = rlen;
        alt_len[r] = al;
        ext_id[r] = E.ext_id;
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

// EMIT_LINES lines per workgroup (one thread each), their text staged in an LDS
// window of EMIT_STAGE bytes: smaller tiles with a right-sized stage put more
// workgroups on a CU (as the window parse)
#ifndef AVDB_VCF_EMIT_LINES
#define AVDB_VCF_EMIT_LINES 256
#endif
#ifndef AVDB_VCF_EMIT_STAGE_KB
#define AVDB_VCF_EMIT_STAGE_KB 36
#endif
#ifndef AVDB_VCF_EMIT_GRID
#define AVDB_VCF_EMIT_GRID (1u << 30)  // emit workgroups (one per tile; a cap grid-strides: 4096 was 0.5 % slower)
#endif
constexpr uint32_t kEmitLines = AVDB_VCF_EMIT_LINES;
constexpr uint32_t kEmitStage = AVDB_VCF_EMIT_STAGE_KB * 1024;
static_assert(kEmitStage <= kStage && kEmitLines <= 1024, "emit tile");

// COMPACT: the lines come as emit records (lines == NULL at parse), else as the
// public table
template <bool COMPACT>
__global__ __launch_bounds__(kEmitLines) void k_vcf_emit(
    const uint8_t* __restrict__ text, size_t text_bytes, size_t n_lines,
    const avdb_vcf_line* __restrict__ lines, const VcfEmitRec* __restrict__ erec, const uint64_t* __restrict__ rec_off,
    const uint64_t* __restrict__ heap_off, uint8_t* __restrict__ chrom, uint32_t* __restrict__ pos,
    uint64_t* __restrict__ allele_off, uint32_t* __restrict__ ref_len, uint32_t* __restrict__ alt_len,
    uint64_t* __restrict__ ext_id, uint8_t* __restrict__ heap, uint32_t* __restrict__ rec_line,
    uint32_t* __restrict__ rec_alt) {
  __shared__ u32x4 s_text[kEmitStage / 16];
  const Heap h = make_heap(text, text_bytes);
  constexpr uint64_t kStartMask = (uint64_t(1) << 56) - 1;
  for (size_t base = size_t(blockIdx.x) * kEmitLines; base < n_lines; base += size_t(gridDim.x) * kEmitLines) {
    const size_t last = base + kEmitLines < n_lines ? base + kEmitLines : n_lines;
    // the window only has to reach the end of the last line's ALT field
    size_t s0, s1;
    if constexpr (COMPACT) {
      s0 = erec[base].start_chrom & kStartMask;
      const VcfEmitRec& Z = erec[last - 1];
      s1 = (Z.start_chrom & kStartMask) + Z.aend;
    } else {
      s0 = lines[base].start;
      const avdb_vcf_line& Z = lines[last - 1];
      s1 = Z.start + Z.len;
    }
    // (reading each line's REF / ALT bytes from global memory instead of staging the
    // tile's text: 519 vs 349 us, profiles/k0_ab/r05_emit_direct_ab.log)
    const Window w = stage_window<kEmitLines, kEmitStage>(h, s0, s1, s_text);
    const size_t li = base + threadIdx.x;
    if (li < n_lines) {
      const uint64_t r0 = rec_off[li], r1 = rec_off[li + 1];
      if (r1 > r0) {
        const VcfEmitRec E = COMPACT ? erec[li] : emit_rec(lines[li]);
        const size_t st = E.start_chrom & kStartMask;
        if (w.staged)
          emit_line((lds_cp)(reinterpret_cast<const uint8_t*>(s_text) + (h.lo + st - w.a0)), E, li, r0,
                    heap_off[li], chrom, pos, allele_off, ref_len, alt_len, ext_id, heap, rec_line, rec_alt);
        else
          emit_line((glb_cp)(text + st), E, li, r0, heap_off[li], chrom, pos, allele_off, ref_len, alt_len, ext_id,
                    heap, rec_line, rec_alt);
      }
    }
    __syncthreads();
  }
}

// ---- the count-free records path: window totals -> bases, then emit per window ----
// Two levels, no one-workgroup pass over all windows (that ran 108 us for 41 k
// windows): k_vcf_local_tiles scans 256 windows per workgroup (bases within the
// tile) and writes each tile's totals; k_vcf_local_top scans the tile totals (one
// workgroup, NW / 256 of them) and writes the totals the host reads; the emit adds
// the two.  tot = {lines, records, heap bytes, overflow windows}.
struct LocalTot {
  unsigned long long lines, recs, heap;
};
constexpr uint32_t kTileWins = 256;

__device__ __forceinline__ unsigned long long wave_incl_sum64(unsigned long long x) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const unsigned long long u = scan::shfl_up64(x, d);
    if (__lane_id() >= uint32_t(d)) x += u;
  }
  return x;
}

__global__ __launch_bounds__(kTileWins) void k_vcf_local_tiles(const LocalWin* __restrict__ win, size_t nw,
                                                               ulonglong2* __restrict__ base_lr,
                                                               unsigned long long* __restrict__ base_h,
                                                               LocalTot* __restrict__ tile_tot) {
  __shared__ uint32_t s_a[kTileWins / kWave], s_b[kTileWins / kWave];
  __shared__ unsigned long long s_c[kTileWins / kWave];
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid / kWave;
  const size_t w = size_t(blockIdx.x) * kTileWins + tid;
  const LocalWin v = w < nw ? win[w] : LocalWin{0, 0, 0};
  const uint32_t xa = wave_incl_sum(v.lines), xb = wave_incl_sum(v.recs);
  const unsigned long long xc = wave_incl_sum64(v.heap);
  if (lane == kWave - 1) {
    s_a[wv] = xa;
    s_b[wv] = xb;
    s_c[wv] = xc;
  }
  __syncthreads();
  uint32_t pa = 0, pb = 0, ta = 0, tb = 0;
  unsigned long long pc = 0, tc = 0;
#pragma unroll
  for (uint32_t q = 0; q < kTileWins / kWave; ++q) {
    if (q < wv) {
      pa += s_a[q];
      pb += s_b[q];
      pc += s_c[q];
    }
    ta += s_a[q];
    tb += s_b[q];
    tc += s_c[q];
  }
  if (w < nw) {
    base_lr[w] = make_ulonglong2(pa + xa - v.lines, pb + xb - v.recs);
    base_h[w] = pc + xc - v.heap;
  }
  if (tid == 0) tile_tot[blockIdx.x] = LocalTot{ta, tb, tc};
}

// exclusive scan of the tile totals in place (one workgroup), the grand totals to
// tot (the workspace header) and out (the caller's)
__global__ __launch_bounds__(kTileWins) void k_vcf_local_top(LocalTot* __restrict__ tile, size_t nt,
                                                             unsigned long long* __restrict__ tot,
                                                             unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s_a[kTileWins / kWave], s_b[kTileWins / kWave], s_c[kTileWins / kWave];
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid / kWave;
  unsigned long long ra = 0, rb = 0, rc = 0;
  for (size_t c0 = 0; c0 < nt; c0 += kTileWins) {
    const size_t i = c0 + tid;
    const LocalTot v = i < nt ? tile[i] : LocalTot{0, 0, 0};
    const unsigned long long xa = wave_incl_sum64(v.lines), xb = wave_incl_sum64(v.recs),
                             xc = wave_incl_sum64(v.heap);
    if (lane == kWave - 1) {
      s_a[wv] = xa;
      s_b[wv] = xb;
      s_c[wv] = xc;
    }
    __syncthreads();
    unsigned long long pa = 0, pb = 0, pc = 0, ta = 0, tb = 0, tc = 0;
#pragma unroll
    for (uint32_t q = 0; q < kTileWins / kWave; ++q) {
      if (q < wv) {
        pa += s_a[q];
        pb += s_b[q];
        pc += s_c[q];
      }
      ta += s_a[q];
      tb += s_b[q];
      tc += s_c[q];
    }
    if (i < nt) tile[i] = LocalTot{ra + pa + xa - v.lines, rb + pb + xb - v.recs, rc + pc + xc - v.heap};
    ra += ta;
    rb += tb;
    rc += tc;
    __syncthreads();
  }
  if (tid == 0) {
    tot[0] = out[0] = ra;
    tot[1] = out[1] = rb;
    tot[2] = out[2] = rc;
    out[3] = tot[3];  // (the parse's overflow count, same stream)
  }
}

// One workgroup per parse window: its lines' record / heap offsets are the window's
// bases plus the in-window offsets the parse left in the slots; its records and
// allele bytes, which the parse wrote to the window's slots, are moved to their
// places (coalesced: slot k -> record base + k, the heap slots as one 8-byte-chunk
// copy); rec_off / heap_off per line (nullable).  The text is not read again.
__global__ __launch_bounds__(kEmitLines) void k_vcf_emit_local(
    const LocalWin* __restrict__ win, const ulonglong2* __restrict__ base_lr,
    const unsigned long long* __restrict__ base_h, const LocalTot* __restrict__ tile_pre,
    const LocalRec* __restrict__ rslot, const uint8_t* __restrict__ hslot, const uint2* __restrict__ cnt,
    const unsigned long long* __restrict__ tot,
    uint64_t* __restrict__ rec_off, uint64_t* __restrict__ heap_off, uint8_t* __restrict__ chrom,
    uint32_t* __restrict__ pos, uint64_t* __restrict__ allele_off, uint32_t* __restrict__ ref_len,
    uint32_t* __restrict__ alt_len, uint64_t* __restrict__ ext_id, uint8_t* __restrict__ heap,
    uint32_t* __restrict__ rec_line, uint32_t* __restrict__ rec_alt) {
  const size_t w = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  if (w == 0 && tid == 0) {  // the totals row of the per-line offsets
    if (rec_off) rec_off[tot[0]] = tot[1];
    if (heap_off) heap_off[tot[0]] = tot[2];
  }
  const LocalWin W = win[w];
  // (uniform; an overflowed window's slots are incomplete — the caller takes the
  // counted path — and are never read past their capacity)
  if (W.lines == 0 || W.lines > kLocalCap || W.recs > kLocalCap || W.heap > kLocalHeap) return;
  const size_t slot0 = w * kLocalCap;
  const LocalTot tp = tile_pre[w / kTileWins];
  ulonglong2 blr = base_lr[w];
  blr.x += tp.lines;
  blr.y += tp.recs;
  const uint64_t hb = base_h[w] + tp.heap;
  if (rec_off || heap_off) {
    for (uint32_t k = tid; k < W.lines; k += kEmitLines) {
      const uint2 c = cnt[slot0 + k];
      if (rec_off) rec_off[blr.x + k] = blr.y + c.x;
      if (heap_off) heap_off[blr.x + k] = hb + c.y;
    }
  }
  for (uint32_t k = tid; k < W.recs; k += kEmitLines) {
    const LocalRec R = rslot[slot0 + k];
    const size_t r = blr.y + k;
    chrom[r] = R.chrom;
    pos[r] = R.pos;
    allele_off[r] = hb + R.hoff;
    ref_len[r] = R.ref_len;
    alt_len[r] = R.alt_len;
    ext_id[r] = R.ext_id;
    rec_line[r] = uint32_t(blr.x + R.line);
    rec_alt[r] = R.alt;
  }
  // the window's allele bytes [0, W.heap): 8-byte chunks (aligned loads from the
  // slots, unaligned stores), the last < 8 bytes one at a time
  const uint64_t* src = reinterpret_cast<const uint64_t*>(hslot + w * kLocalHeap);
  const uint32_t nh = uint32_t(W.heap), n8 = nh / 8;
  for (uint32_t k = tid; k < n8; k += kEmitLines) reinterpret_cast<gw_u64u>((gbyte*)heap + hb + 8 * k)->v = src[k];
  if (tid < (nh & 7u)) heap[hb + 8 * n8 + tid] = hslot[w * kLocalHeap + 8 * n8 + tid];
}

}  // namespace avdb

using namespace avdb;

// k_vcf_count + k_vcf_scan_blocks into a count workspace (layout: kCountWs*)
// the count pass's cut (wave_range) and the parse windows inside it, host side
static size_t sub_chunk_bytes(size_t text_bytes) {
  const size_t nw = size_t(kVcfGrid) * kVcfWaves;
  const size_t per = (text_bytes + nw - 1) / nw;
  return (per + 63) & ~size_t(63);
}
static uint32_t windows_per_chunk(size_t text_bytes) {
  const size_t per = sub_chunk_bytes(text_bytes);
  return per ? uint32_t((per + kParseWin - 1) / kParseWin) : 1u;
}
static size_t count_ws_full(size_t text_bytes) {  // header part + one u32 per window
  return AVDB_VCF_COUNT_WORKSPACE_BYTES +
         ((4 * size_t(kVcfGrid) * kVcfWaves * windows_per_chunk(text_bytes) + 255) & ~size_t(255));
}

extern "C" int avdb_vcf_count_workspace_size(size_t text_bytes, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = count_ws_full(text_bytes);
  return AVDB_OK;
}

// k_vcf_count + k_vcf_scan_blocks into a count workspace (layout: kCountWs*, then
// the window counts when `windows`)
static int count_pass(const uint8_t* text, size_t text_bytes, void* ws, unsigned long long* total, hipStream_t s,
                      bool windows) {
  char* w = static_cast<char*>(ws);
  auto* wave = reinterpret_cast<uint32_t*>(w + kCountWsWave);
  auto* blk = reinterpret_cast<unsigned long long*>(w + kCountWsBlkOff);
  auto* win = windows ? reinterpret_cast<uint32_t*>(w + AVDB_VCF_COUNT_WORKSPACE_BYTES) : nullptr;
  hipLaunchKernelGGL(k_vcf_count, dim3(kVcfGrid), dim3(kBlock), 0, s, text, text_bytes, wave, win,
                     windows_per_chunk(text_bytes));
  AVDB_LAUNCH_CHECK("k_vcf_count");
  hipLaunchKernelGGL(k_vcf_scan_blocks, dim3(1), dim3(kVcfGrid), 0, s, wave, blk, total);
  AVDB_LAUNCH_CHECK("k_vcf_scan_blocks");
  return AVDB_OK;
}

static size_t scan_temp_bytes(size_t n) { return (scan::workspace_bytes(n, 2) + 255) & ~size_t(255); }

static VcfEmitRec* emit_recs_of(void* workspace, size_t text_bytes, size_t n_lines) {
  return reinterpret_cast<VcfEmitRec*>(static_cast<char*>(workspace) + count_ws_full(text_bytes) +
                                       ((8 * n_lines + 255) & ~size_t(255)) + scan_temp_bytes(n_lines + 1));
}

extern "C" int avdb_vcf_workspace_size(size_t text_bytes, size_t n_lines, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  // count workspace (for a recount) | line starts | scan temp | emit records
  *bytes = count_ws_full(text_bytes) + ((8 * n_lines + 255) & ~size_t(255)) + scan_temp_bytes(n_lines + 1) +
           sizeof(VcfEmitRec) * n_lines + 256;
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
  return count_pass(text, text_bytes, workspace, reinterpret_cast<unsigned long long*>(n_newlines), s,
                    workspace_bytes >= count_ws_full(text_bytes));
}

static int parse_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                       const void* line_counts, size_t line_counts_bytes, void* workspace, size_t workspace_bytes,
                       avdb_vcf_line* lines, uint64_t* rec_off, uint64_t* heap_off, const avdb_vcf_opts* opts,
                       void* stream) {
  if (!ctx || !rec_off || !heap_off) {
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
  const size_t cw_full = count_ws_full(text_bytes);
  auto* starts = reinterpret_cast<uint64_t*>(static_cast<char*>(workspace) + cw_full);
  void* tmp = reinterpret_cast<char*>(starts) + ((8 * n_lines + 255) & ~size_t(255));
  size_t tmp_bytes = scan_temp_bytes(n_lines + 1);
  // lines == NULL: no public table; the emit records go to the workspace instead
  VcfEmitRec* erec = lines ? nullptr : emit_recs_of(workspace, text_bytes, n_lines);
  const char* cw = static_cast<const char*>(line_counts);
  bool windows = cw && line_counts_bytes >= cw_full;
  if (!cw) {  // recount into the front of this workspace (same cut, window counts included)
    const int rc = count_pass(text, text_bytes, workspace, nullptr, s, true);
    if (rc != AVDB_OK) return rc;
    cw = static_cast<const char*>(workspace);
    windows = true;
  }
  auto* rc = reinterpret_cast<unsigned long long*>(rec_off);
  auto* hc = reinterpret_cast<unsigned long long*>(heap_off);
  AVDB_HIP_TRY(hipMemsetAsync(rc + n_lines, 0, 8, s));
  AVDB_HIP_TRY(hipMemsetAsync(hc + n_lines, 0, 8, s));
  const auto* blk = reinterpret_cast<const unsigned long long*>(cw + kCountWsBlkOff);
  const auto* wave = reinterpret_cast<const uint32_t*>(cw + kCountWsWave);
  if (windows) {  // one workgroup per parse window, line starts found in it
    const uint32_t wps = windows_per_chunk(text_bytes);
    hipLaunchKernelGGL(k_vcf_parse_windows<false>, dim3(unsigned(size_t(kVcfGrid) * kVcfWaves * wps)), dim3(kBlock), 0,
                       s, text, text_bytes, n_lines, blk, wave,
                       reinterpret_cast<const uint32_t*>(cw + AVDB_VCF_COUNT_WORKSPACE_BYTES), wps, lines, erec, rc,
                       hc, cm, min_fields, LocalOut{});
    AVDB_LAUNCH_CHECK("k_vcf_parse_windows");
  } else {  // the line-starts pass, then 256 lines per workgroup
    hipLaunchKernelGGL(k_vcf_starts, dim3(kVcfGrid), dim3(kBlock), 0, s, text, text_bytes, blk, wave, n_lines, starts);
    AVDB_LAUNCH_CHECK("k_vcf_starts");
    const unsigned grid = stream_grid(n_lines, kBlock, 4096);
    hipLaunchKernelGGL(k_vcf_parse, dim3(grid), dim3(kBlock), 0, s, text, text_bytes, n_lines, starts,
                       lines, erec, rc, hc, cm, min_fields);
    AVDB_LAUNCH_CHECK("k_vcf_parse");
  }
  if (int e = scan::exclusive_u64_pair(rec_off, rec_off, heap_off, heap_off, n_lines + 1, tmp, tmp_bytes, s)) return e;
  return AVDB_OK;
}

extern "C" int avdb_vcf_parse_lines(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes,
                                    size_t n_lines, const void* line_counts, void* workspace,
                                    size_t workspace_bytes,
                                    avdb_vcf_line* lines, uint64_t* rec_off, uint64_t* heap_off,
                                    const avdb_vcf_opts* opts, void* stream) {
  return parse_lines(ctx, text, text_bytes, n_lines, line_counts, AVDB_VCF_COUNT_WORKSPACE_BYTES, workspace,
                     workspace_bytes, lines, rec_off, heap_off, opts, stream);
}

extern "C" int avdb_vcf_parse_lines2(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                                     const void* line_counts, size_t line_counts_bytes, void* workspace,
                                     size_t workspace_bytes, avdb_vcf_line* lines, uint64_t* rec_off,
                                     uint64_t* heap_off, const avdb_vcf_opts* opts, void* stream) {
  return parse_lines(ctx, text, text_bytes, n_lines, line_counts, line_counts_bytes, workspace, workspace_bytes,
                     lines, rec_off, heap_off, opts, stream);
}

static int emit_impl(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines, const avdb_vcf_line* lines,
                     const VcfEmitRec* erec, const uint64_t* rec_off, const uint64_t* heap_off, uint8_t* chrom,
                     uint32_t* pos, uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len, uint64_t* ext_id,
                     uint8_t* heap, uint32_t* rec_line, uint32_t* rec_alt, void* stream) {
  if (!ctx || !(lines || erec) || !rec_off || !heap_off || !chrom || !pos || !allele_off || !ref_len ||
      !alt_len || !ext_id || !heap || !rec_line || !rec_alt) {
    avdb_set_error("avdb_vcf_emit: null argument");
    return AVDB_EINVAL;
  }
  if (n_lines == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const unsigned grid = stream_grid(n_lines, kEmitLines, AVDB_VCF_EMIT_GRID);
  if (lines)
    hipLaunchKernelGGL(k_vcf_emit<false>, dim3(grid), dim3(kEmitLines), 0, static_cast<hipStream_t>(stream), text,
                       text_bytes, n_lines, lines, nullptr, rec_off, heap_off, chrom, pos, allele_off, ref_len, alt_len,
                       ext_id, heap, rec_line, rec_alt);
  else
    hipLaunchKernelGGL(k_vcf_emit<true>, dim3(grid), dim3(kEmitLines), 0, static_cast<hipStream_t>(stream), text,
                       text_bytes, n_lines, nullptr, erec, rec_off, heap_off, chrom, pos, allele_off, ref_len, alt_len,
                       ext_id, heap, rec_line, rec_alt);
  AVDB_LAUNCH_CHECK("k_vcf_emit");
  return AVDB_OK;
}

extern "C" int avdb_vcf_emit(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                             const avdb_vcf_line* lines, const uint64_t* rec_off,
                             const uint64_t* heap_off, uint8_t* chrom, uint32_t* pos,
                             uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len,
                             uint64_t* ext_id, uint8_t* heap, uint32_t* rec_line, uint32_t* rec_alt,
                             void* stream) {
  if (!lines) {
    avdb_set_error("avdb_vcf_emit: null line table (use avdb_vcf_emit_ws after a parse without one)");
    return AVDB_EINVAL;
  }
  return emit_impl(ctx, text, text_bytes, n_lines, lines, nullptr, rec_off, heap_off, chrom, pos, allele_off,
                   ref_len, alt_len, ext_id, heap, rec_line, rec_alt, stream);
}

extern "C" int avdb_vcf_emit_ws(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                                const void* parse_workspace, size_t parse_workspace_bytes, const uint64_t* rec_off,
                                const uint64_t* heap_off, uint8_t* chrom, uint32_t* pos, uint64_t* allele_off,
                                uint32_t* ref_len, uint32_t* alt_len, uint64_t* ext_id, uint8_t* heap,
                                uint32_t* rec_line, uint32_t* rec_alt, void* stream) {
  size_t need = 0;
  avdb_vcf_workspace_size(text_bytes, n_lines, &need);
  if (!parse_workspace || parse_workspace_bytes < need) {
    avdb_set_error("avdb_vcf_emit_ws: the parse workspace (%zu bytes) required", need);
    return AVDB_ERANGE;
  }
  return emit_impl(ctx, text, text_bytes, n_lines, nullptr,
                   emit_recs_of(const_cast<void*>(parse_workspace), text_bytes, n_lines), rec_off, heap_off, chrom,
                   pos, allele_off, ref_len, alt_len, ext_id, heap, rec_line, rec_alt, stream);
}

// ---- chromosome map (ChromosomeMap.get, chromosome_map_parser.py:84-91) ----------
// ---- the count-free records path: host side ----
// workspace: header (totals: lines, records, heap bytes, overflow windows) | LocalWin
// per window | (line, record) bases per window | heap base per window | tile totals |
// record slots | heap slots | (records, heap bytes) per line slot
struct LocalLayout {
  size_t nw, nt, win, blr, bh, tile, rec, heap, cnt, bytes;
};
static LocalLayout local_layout(size_t text_bytes) {
  auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
  LocalLayout L;
  // only the windows of sub-chunks that hold text (the count pass's cut gives the
  // sub-chunks past ceil(text_bytes / sub_chunk_bytes) no bytes): a short text gets
  // a few windows' slots, not kVcfGrid * kVcfWaves of them (160 MiB)
  const size_t per = sub_chunk_bytes(text_bytes);
  const size_t live = per ? (text_bytes + per - 1) / per : 0;
  L.nw = live * windows_per_chunk(text_bytes);
  L.nt = (L.nw + kTileWins - 1) / kTileWins;
  L.win = 256;
  L.blr = L.win + up(sizeof(LocalWin) * L.nw);
  L.bh = L.blr + up(16 * L.nw);
  L.tile = L.bh + up(8 * L.nw);
  L.rec = L.tile + up(sizeof(LocalTot) * L.nt);
  L.heap = L.rec + up(sizeof(LocalRec) * L.nw * kLocalCap);
  L.cnt = L.heap + up(size_t(kLocalHeap) * L.nw);
  L.bytes = L.cnt + up(8 * L.nw * kLocalCap);
  return L;
}

extern "C" int avdb_vcf_local_workspace_size(size_t text_bytes, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = local_layout(text_bytes).bytes;
  return AVDB_OK;
}

static const char* local_ws_error(const void* ws, size_t ws_bytes, size_t text_bytes) {
  if (!ws || reinterpret_cast<uintptr_t>(ws) % 16 || ws_bytes < local_layout(text_bytes).bytes)
    return "16-byte aligned workspace of avdb_vcf_local_workspace_size(text_bytes) bytes required";
  return nullptr;
}

extern "C" int avdb_vcf_parse_local(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, void* workspace,
                                    size_t workspace_bytes, const avdb_vcf_opts* opts, uint64_t* totals,
                                    void* stream) {
  if (!ctx || !totals || (text_bytes && !text)) {
    avdb_set_error("avdb_vcf_parse_local: null argument");
    return AVDB_EINVAL;
  }
  if (opts && opts->struct_size != sizeof(avdb_vcf_opts)) {
    avdb_set_error("avdb_vcf_parse_local: avdb_vcf_opts.struct_size %u, this library expects %zu",
                   opts->struct_size, sizeof(avdb_vcf_opts));
    return AVDB_EINVAL;
  }
  if (opts && opts->chrom_map && opts->chrom_map->device != ctx->device) {
    avdb_set_error("avdb_vcf_parse_local: chromosome map made for device %d", opts->chrom_map->device);
    return AVDB_EINVAL;
  }
  if (const char* e = local_ws_error(workspace, workspace_bytes, text_bytes)) {
    avdb_set_error("avdb_vcf_parse_local: %s", e);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  auto* hdr = reinterpret_cast<unsigned long long*>(w);
  AVDB_HIP_TRY(hipMemsetAsync(hdr, 0, 32, s));
  if (text_bytes == 0) {
    AVDB_HIP_TRY(hipMemsetAsync(totals, 0, 32, s));
    return AVDB_OK;
  }
  const ChromMapView cm = opts && opts->chrom_map ? opts->chrom_map->dev : ChromMapView{};
  const uint32_t min_fields = opts ? opts->min_fields : 0u;
  const LocalLayout L = local_layout(text_bytes);
  LocalOut o{reinterpret_cast<LocalWin*>(w + L.win), reinterpret_cast<LocalRec*>(w + L.rec),
             reinterpret_cast<uint8_t*>(w + L.heap), reinterpret_cast<uint2*>(w + L.cnt), hdr + 3};
  hipLaunchKernelGGL(k_vcf_parse_windows<true>, dim3(unsigned(L.nw)), dim3(kBlock), 0, s, text, text_bytes, size_t(0),
                     nullptr, nullptr, nullptr, windows_per_chunk(text_bytes), nullptr, nullptr, nullptr, nullptr, cm,
                     min_fields, o);
  AVDB_LAUNCH_CHECK("k_vcf_parse_windows<local>");
  hipLaunchKernelGGL(k_vcf_local_tiles, dim3(unsigned(L.nt)), dim3(kTileWins), 0, s, o.win, L.nw,
                     reinterpret_cast<ulonglong2*>(w + L.blr), reinterpret_cast<unsigned long long*>(w + L.bh),
                     reinterpret_cast<LocalTot*>(w + L.tile));
  AVDB_LAUNCH_CHECK("k_vcf_local_tiles");
  hipLaunchKernelGGL(k_vcf_local_top, dim3(1), dim3(kTileWins), 0, s, reinterpret_cast<LocalTot*>(w + L.tile), L.nt,
                     hdr, reinterpret_cast<unsigned long long*>(totals));
  AVDB_LAUNCH_CHECK("k_vcf_local_top");
  return AVDB_OK;
}

extern "C" int avdb_vcf_emit_local(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, const void* workspace,
                                   size_t workspace_bytes, uint64_t* rec_off, uint64_t* heap_off, uint8_t* chrom,
                                   uint32_t* pos, uint64_t* allele_off, uint32_t* ref_len, uint32_t* alt_len,
                                   uint64_t* ext_id, uint8_t* heap, uint32_t* rec_line, uint32_t* rec_alt,
                                   void* stream) {
  if (!ctx || !chrom || !pos || !allele_off || !ref_len || !alt_len || !ext_id || !heap || !rec_line || !rec_alt) {
    avdb_set_error("avdb_vcf_emit_local: null argument");
    return AVDB_EINVAL;
  }
  if (const char* e = local_ws_error(workspace, workspace_bytes, text_bytes)) {
    avdb_set_error("avdb_vcf_emit_local: %s", e);
    return AVDB_ERANGE;
  }
  if (text_bytes == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  const char* w = static_cast<const char*>(workspace);
  const LocalLayout L = local_layout(text_bytes);
  hipLaunchKernelGGL(k_vcf_emit_local, dim3(unsigned(L.nw)), dim3(kEmitLines), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const LocalWin*>(w + L.win), reinterpret_cast<const ulonglong2*>(w + L.blr),
                     reinterpret_cast<const unsigned long long*>(w + L.bh), reinterpret_cast<const LocalTot*>(w + L.tile),
                     reinterpret_cast<const LocalRec*>(w + L.rec), reinterpret_cast<const uint8_t*>(w + L.heap),
                     reinterpret_cast<const uint2*>(w + L.cnt), reinterpret_cast<const unsigned long long*>(w),
                     rec_off, heap_off, chrom, pos, allele_off, ref_len, alt_len, ext_id, heap, rec_line, rec_alt);
  AVDB_LAUNCH_CHECK("k_vcf_emit_local");
  return AVDB_OK;
}

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
