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
};

__device__ __forceinline__ Mask16 nl_mask16(uintptr_t a, const Heap& h, uintptr_t lo, uintptr_t end) {
  uint64_t m0 = 0, m1 = 0;
  if (a >= end) return Mask16{0, 0};
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

__global__ __launch_bounds__(kBlock) void k_vcf_count(const uint8_t* __restrict__ text,
                                                      size_t text_bytes,
                                                      uint32_t* __restrict__ wave_cnt) {
  const Heap h = make_heap(text, text_bytes);
  const size_t gw = size_t(blockIdx.x) * kVcfWaves + threadIdx.x / kWave;
  size_t t0, t1;
  wave_range(text_bytes, gw, &t0, &t1);
  const uintptr_t lo = h.lo + t0, end = h.lo + t1;
  uint32_t c = 0;
  for (uintptr_t a = (lo & ~uintptr_t(15)) + 16 * __lane_id(); a < end; a += kNlUnroll * kNlStep) {
    Mask16 m[kNlUnroll];
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) m[u] = nl_mask16(a + u * kNlStep, h, lo, end);
#pragma unroll
    for (int u = 0; u < kNlUnroll; ++u) c += uint32_t(__popcll(m[u].m0) + __popcll(m[u].m1));
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

// contig code of a CHROM field (vcf_parser.py:133-150 + bin_index.py:64): plain
// digits go through int(); 'MT' -> 'M'; every 'chr' removed in one left-to-right
// pass (str.replace); then chr1..22, X, Y, M.  *host set for non-alphanumeric bytes.
template <class CP>
__device__ uint8_t chrom_code_of(CP p, uint32_t n, bool* host) {
  *host = false;
  if (n == 0) return 255;
  bool digits = true;
  for (uint32_t i = 0; i < n; ++i) {
    if (!is_alnum(p[i])) { *host = true; return 255; }
    digits = digits && is_digit(p[i]);
  }
  if (digits) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; ++i) {
      v = v * 10 + (p[i] - '0');
      if (v > 1000) return 255;
    }
    return (v >= 1 && v <= 22) ? uint8_t(v - 1) : 255;
  }
  if (n == 2 && p[0] == 'M' && p[1] == 'T') return 24;
  uint8_t lab[3];
  uint32_t m = 0;
  for (uint32_t i = 0; i < n;) {
    if (i + 3 <= n && p[i] == 'c' && p[i + 1] == 'h' && p[i + 2] == 'r') { i += 3; continue; }
    if (m == 3) return 255;
    lab[m++] = p[i++];
  }
  if (m == 1) {
    if (lab[0] >= '1' && lab[0] <= '9') return uint8_t(lab[0] - '1');
    if (lab[0] == 'X') return 22;
    if (lab[0] == 'Y') return 23;
    if (lab[0] == 'M') return 24;
    return 255;
  }
  if (m == 2 && is_digit(lab[0]) && is_digit(lab[1]) && lab[0] != '0') {
    const uint32_t v = (lab[0] - '0') * 10 + (lab[1] - '0');
    return (v >= 10 && v <= 22) ? uint8_t(v - 1) : 255;
  }
  return 255;
}

// canonical refSNP number of "rs<N>" bytes (N without leading zeros, < 10^18), else 0
template <class CP>
__device__ uint64_t rs_number(CP p, uint32_t n) {
  if (n < 3 || n > 20 || p[0] != 'r' || p[1] != 's' || p[2] == '0') return 0;
  uint64_t v = 0;
  for (uint32_t i = 2; i < n; ++i) {
    if (!is_digit(p[i])) return 0;
    v = v * 10 + (p[i] - '0');
  }
  return v;
}

// ---- SWAR field helpers: a field's bytes as two registers, read with
// independent aligned word loads (the byte loops these replace waited on one
// dependent LDS byte read per iteration) ----
// 16 bytes of the line from line offset f (bytes at and past `len` read as 0)
template <class WordAt>
__device__ __forceinline__ void line16(const WordAt& word_at, uint32_t mis, uint32_t len, uint32_t f,
                                       uint64_t* x0, uint64_t* x1) {
  const uint32_t a = f + mis, k = a >> 3, sh = 8 * (a & 7);
  const uint32_t kend = (len + mis + 7) >> 3;  // words holding line bytes
  const uint64_t w0 = k < kend ? word_at(k) : 0ull;
  const uint64_t w1 = k + 1 < kend ? word_at(k + 1) : 0ull;
  const uint64_t w2 = k + 2 < kend ? word_at(k + 2) : 0ull;
  uint64_t y0 = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  uint64_t y1 = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  // clip at the line end
  const uint32_t n = len > f ? len - f : 0u;
  if (n < 16) {
    y1 &= n > 8 ? low_bytes_mask(n - 8) : 0ull;
    y0 &= low_bytes_mask(n < 8 ? n : 8);
  }
  *x0 = y0;
  *x1 = y1;
}


// up to 8 ASCII digits (most significant in the lowest byte, n of them) -> value
__device__ __forceinline__ uint32_t digits8_value(uint64_t x, uint32_t n) {
  if (n == 0) return 0;
  uint64_t v = (x ^ 0x3030303030303030ull) << (8 * (8 - n));  // leading zero digits below
  v = (v * 10 + (v >> 8)) & 0x00FF00FF00FF00FFull;
  v = (v * 100 + (v >> 16)) & 0x0000FFFF0000FFFFull;
  v = (v * 10000 + (v >> 32)) & 0xFFFFFFFFull;
  return uint32_t(v);
}

// a decimal field of n <= 16 bytes in (x0, x1): *ok = all digits; value (64-bit)
__device__ __forceinline__ uint64_t decimal16(uint64_t x0, uint64_t x1, uint32_t n, bool* ok) {
  const uint64_t m0 = low_bytes_mask(n < 8 ? n : 8), m1 = n > 8 ? low_bytes_mask(n - 8) : 0ull;
  *ok = n > 0 && !((nondigit_mask(x0) & m0) | (nondigit_mask(x1) & m1));
  if (n <= 8) return digits8_value(x0 & m0, n);
  // the first n - 8 digits, then 8 more
  const uint32_t h = n - 8, sh = 8 * h;
  const uint64_t hi = x0 & low_bytes_mask(h);
  const uint64_t lo = sh < 64 ? (x0 >> sh) | (x1 << (64 - sh)) : x1;
  return uint64_t(digits8_value(hi, h)) * 100000000ull + digits8_value(lo, 8);
}

constexpr uint64_t kTab = 0x0909090909090909ull;
constexpr uint64_t kSemi = 0x3B3B3B3B3B3B3B3Bull;

// one line: s points at its first byte (LDS or global), len = bytes up to its
// newline; word_at/mis give the same bytes as aligned 8-byte words (SWAR scans)
template <class CP, class WordAt>
__device__ __forceinline__ void parse_line(CP s, const WordAt& word_at, uint32_t mis,
                                           uint32_t len, avdb_vcf_line& L, uint64_t& recs,
                                           uint64_t& hbytes) {
    while (len && is_ws(s[len - 1])) --len;  // str.rstrip()
    L.len = len;
    L.flags = 0;
    L.pos = 0;
    L.ext_id = 0;
    L.n_alt = 0;
    L.n_rec = 0;
    L.chrom = 255;
    L.pad[0] = L.pad[1] = L.pad[2] = 0;
    uint32_t nf = 1;
    L.field[0] = 0;
    for (int k = 1; k < 8; ++k) L.field[k] = len + 1;
    L.field_end8 = len;
    if (len && s[0] == '#') L.flags |= AVDB_VCF_COMMENT;
    if (!len) L.flags |= AVDB_VCF_EMPTY;
    // tab-separated fields (first 8 starts; INFO ends at the 8th tab or the end)
    {
      const uint32_t k1 = (len + mis + 7) >> 3;
      for (uint32_t k = 0; k < k1; ++k) {
        uint64_t m = zero_bytes_mask(word_at(k) ^ kTab) & kHiBits;
        if (k == 0) m &= ~low_bytes_mask(mis);
        const uint32_t hi = len + mis - 8 * k;
        if (hi < 8) m &= low_bytes_mask(hi);
        if (nf > 8) {  // past INFO: only the count matters
          nf += uint32_t(__popcll(m));
          continue;
        }
        while (m) {
          const uint32_t i = 8 * k + (uint32_t(__builtin_ctzll(m)) >> 3) - mis;
          m &= m - 1;
#pragma unroll
          for (int f = 1; f < 8; ++f)  // register-resident field table (no dynamic index)
            if (nf == uint32_t(f)) L.field[f] = i + 1;
          if (nf == 8) L.field_end8 = i;
          ++nf;
        }
      }
    }
    L.n_fields = nf;
    recs = 0;
    hbytes = 0;
    if (!(L.flags & (AVDB_VCF_COMMENT | AVDB_VCF_EMPTY))) {
      if (nf < 8) L.flags |= AVDB_VCF_FEW_FIELDS;
      const uint32_t nfields = nf < 8 ? nf : 8;
      auto fend = [&](int k) -> uint32_t {  // end of field k (exclusive)
        return (k + 1 < int(nfields)) ? L.field[k + 1] - 1 : (k == 7 ? L.field_end8 : len);
      };
      if (!(L.flags & AVDB_VCF_FEW_FIELDS)) {
        // CHROM
        bool host = false;
        L.chrom = chrom_code_of(s, fend(0), &host);
        if (host) L.flags |= AVDB_VCF_CHROM_HOST;
        // POS: plain decimal < 2^32
        {
          const uint32_t n = fend(1) - L.field[1];
          uint64_t x0, x1;
          line16(word_at, mis, len, L.field[1], &x0, &x1);
          bool ok = false;
          const uint64_t v = n <= 10 ? decimal16(x0, x1, n, &ok) : 0ull;
          if (ok && v <= 0xFFFFFFFFull) L.pos = uint32_t(v); else L.flags |= AVDB_VCF_BAD_POS;
        }
        // ID
        const CP id = s + L.field[2];
        const uint32_t idn = fend(2) - L.field[2];
        // ID, 16 bytes at a time: digits / number-like bytes / an "rs" pair
        bool has_rs = false;
        {
          bool numlike = idn > 0, has_digit = false;
          uint64_t carry_r = 0;  // bit 7: the byte before this block is 'r'
          for (uint32_t b = 0; b < idn; b += 16) {
            uint64_t y[2];
            line16(word_at, mis, len, L.field[2] + b, &y[0], &y[1]);
            const uint32_t nb = idn - b < 16u ? idn - b : 16u;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t nh = h ? (nb > 8 ? nb - 8 : 0u) : (nb < 8 ? nb : 8u);
              const uint64_t m = low_bytes_mask(nh) & kHiBits;
              const uint64_t x = y[h];
              const uint64_t dig = ~nondigit_mask(x) & m;
              has_digit = has_digit || dig;
              const uint64_t numb = dig | bytes_eq_mask(x, '+') | bytes_eq_mask(x, '-') | bytes_eq_mask(x, '.') |
                                    bytes_eq_mask(x, 'e') | bytes_eq_mask(x, 'E') | bytes_eq_mask(x, '_');
              numlike = numlike && !((~numb) & m);
              const uint64_t rm = bytes_eq_mask(x, 'r') & m, sm = bytes_eq_mask(x, 's') & m;
              has_rs = has_rs || (((rm << 8) | carry_r) & sm);
              carry_r = nh == 8 ? (rm >> 56) : 0ull;
            }
          }
          if (numlike && has_digit) L.flags |= AVDB_VCF_ID_HOST;  // Python coerces it to a number
        }
        if ((idn == 1 && id[0] == '.') || (idn >= 2 && id[0] == 'r' && id[1] == 's'))
          L.flags |= AVDB_VCF_ID_METASEQ;
        if (has_rs) {
          L.flags |= AVDB_VCF_ID_RS;
          if (idn >= 3 && idn <= 18 && id[0] == 'r' && id[1] == 's' && id[2] != '0') {
            uint64_t y0, y1;  // "rs" + up to 16 digits, SWAR
            line16(word_at, mis, len, L.field[2] + 2, &y0, &y1);
            bool ok;
            const uint64_t v = decimal16(y0, y1, idn - 2, &ok);
            L.ext_id = ok ? v : 0ull;
          } else {
            L.ext_id = rs_number(id, idn);
          }
          if (!L.ext_id) L.flags |= AVDB_VCF_EXT_HOST;
        } else {
          // INFO: last entry whose key is exactly "RS" (dict(...) keeps the last)
          const CP inf = s + L.field[7];
          const uint32_t f7 = L.field[7], e7 = fend(7);
          int64_t vs = -1, ve = -1;
          bool bare = false;
          // entries are [i, j) between ';' (INFO-relative), scanned 8 bytes at a time
          uint32_t i = 0;
          const uint32_t in = e7 >= f7 ? e7 - f7 : 0;
          for (uint32_t at = 0; at <= in;) {
            // next ';' at or after `at` (SWAR), or the INFO end
            uint32_t j = in;
            {
              const uint32_t from = f7 + at, to = e7;
              const uint32_t k1 = (to + mis + 7) >> 3;
              for (uint32_t k = (from + mis) >> 3; k < k1; ++k) {
                uint64_t m = zero_bytes_mask(word_at(k) ^ kSemi) & kHiBits;
                const int32_t lo = int32_t(from + mis) - int32_t(8 * k);
                if (lo > 0) m &= ~low_bytes_mask(uint32_t(lo));
                const uint32_t hi = to + mis - 8 * k;
                if (hi < 8) m &= low_bytes_mask(hi);
                if (m) {
                  j = 8 * k + (uint32_t(__builtin_ctzll(m)) >> 3) - mis - f7;
                  break;
                }
              }
            }
            if (j - i >= 2 && inf[i] == 'R' && inf[i + 1] == 'S') {
              if (j - i == 2) { bare = true; vs = ve = -1; }
              else if (inf[i + 2] == '=') { bare = false; vs = i + 3; ve = j; }
            }
            i = j + 1;
            at = j + 1;
          }
          if (vs >= 0 || bare) {
            L.flags |= AVDB_VCF_INFO_RS;
            uint64_t v = 0;
            bool ok = !bare && ve > vs && ve - vs <= 18;
            for (int64_t i = vs; ok && i < ve; ++i) {
              ok = is_digit(inf[i]);
              v = v * 10 + (inf[i] - '0');
            }
            if (ok && v >= 1) L.ext_id = v;  // 'rs' + str(int(value))
            else L.flags |= AVDB_VCF_EXT_HOST;
          }
        }
        // REF / ALT
        const uint32_t rlen = fend(3) - L.field[3];
        const CP alt = s + L.field[4];
        const uint32_t an = fend(4) - L.field[4];
        // SWAR: commas and '.' bytes of the ALT field; without a '.', every ALT is a
        // record and the counts follow from the comma count
        uint32_t commas = 0;
        bool dot = false;
        for (uint32_t b = 0; b < an; b += 16) {
          uint64_t y0, y1;
          line16(word_at, mis, len, L.field[4] + b, &y0, &y1);
          const uint32_t nb = an - b < 16u ? an - b : 16u;
          const uint64_t m0 = low_bytes_mask(nb < 8 ? nb : 8) & kHiBits;
          const uint64_t m1 = (nb > 8 ? low_bytes_mask(nb - 8) : 0ull) & kHiBits;
          commas += uint32_t(__popcll(bytes_eq_mask(y0, ',') & m0) + __popcll(bytes_eq_mask(y1, ',') & m1));
          dot = dot || ((bytes_eq_mask(y0, '.') & m0) | (bytes_eq_mask(y1, '.') & m1));
        }
        if (!dot) {
          L.n_alt = commas + 1;
          L.n_rec = L.n_alt;
          hbytes = uint64_t(L.n_rec) * rlen + (an - commas);
        }
        uint32_t a0 = 0;
        for (uint32_t i = 0; dot && i <= an; ++i) {
          if (i == an || alt[i] == ',') {
            const uint32_t al = i - a0;
            ++L.n_alt;
            if (!(al == 1 && alt[a0] == '.')) {
              ++L.n_rec;
              hbytes += rlen + al;
            }
            a0 = i + 1;
          }
        }
        recs = L.n_rec;
      }
    }
}

__global__ __launch_bounds__(kBlock) void k_vcf_parse(const uint8_t* __restrict__ text,
                                                      size_t text_bytes, size_t n_lines,
                                                      const uint64_t* __restrict__ starts,
                                                      avdb_vcf_line* __restrict__ lines,
                                                      unsigned long long* __restrict__ rec_cnt,
                                                      unsigned long long* __restrict__ heap_cnt) {
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
        parse_line((lds_cp)ls, [lw](uint32_t k) { return lw[k]; }, mis, raw, L, recs, hbytes);
      } else {
        const uintptr_t la = h.lo + L.start - mis;
        parse_line((glb_cp)(text + L.start), [la, h](uint32_t k) { return heap_word(la + 8 * size_t(k), h); },
                   mis, raw, L, recs, hbytes);
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
                      hipStream_t s) {
  char* w = static_cast<char*>(ws);
  auto* wave = reinterpret_cast<uint32_t*>(w + kCountWsWave);
  auto* blk = reinterpret_cast<unsigned long long*>(w + kCountWsBlkOff);
  hipLaunchKernelGGL(k_vcf_count, dim3(kVcfGrid), dim3(kBlock), 0, s, text, text_bytes, wave);
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
                                    void* stream) {
  if (!ctx || !lines || !rec_off || !heap_off) {
    avdb_set_error("avdb_vcf_parse_lines: null argument");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_vcf_workspace_size(text_bytes, n_lines, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_vcf_parse_lines: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  if (n_lines == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
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
                     lines, rc, hc);
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
