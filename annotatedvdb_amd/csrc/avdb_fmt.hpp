// Text sink and JSON / key / ltree-path renderers shared by the K5 (avdb_format.hip),
// K5a + K7 (avdb_keys.hip) and K8 (avdb_small.hip) kernels.
#pragma once

#include "avdb_internal.hpp"
#include "avdb_text.hpp"

#include <type_traits>

namespace avdb {


// ---------------------------------------------------------------------------
// output sink: SIZE pass counts, WRITE pass stores
// ---------------------------------------------------------------------------
// WRITE pass sink: each lane's bytes are packed into a 64-bit register word and
// stored 8 at a time (an unaligned global_store_dwordx2; gfx950 runs in
// unaligned mode), the tail (< 8 bytes) byte by byte at the end of the line.
// The lanes of a wave write 64 different lines, so every store instruction
// touches up to 64 cache lines: what costs is the number of lane-stores, not
// bytes.  A/B on MI355X, 8.39 M dbSNP-shaped lines, 5.25 GB written (write
// pass; size pass 5.1 ms; tools/k5_ab.sh):
//   byte stores, noinline helpers, 3 waves/SIMD            15.0 ms
//   same, stores made coalesced (wrong output; the floor)     4.6 ms
//   8-byte word, noinline helpers, 3 waves/SIMD             9.7 ms
//   8-byte word, inlined helpers, 3 waves/SIMD              9.3 ms
//   8-byte word, inlined helpers, 4 waves/SIMD (this)       8.1 ms
//   16-byte word (two u64), 2 waves/SIMD (VGPR-bound)      17.4 ms
//   per-lane LDS ring (32/64 B per stream) flushing 16-byte
//     chunks at convergent points, 2 waves/SIMD             13.4 / 17.7 ms
// Occupancy decides: the pass is latency-bound on LDS text reads and store
// back-pressure, so 4 waves/SIMD (launch bound; ~120 B of spills) beats every
// wider sink that costs registers or LDS.
// Round 2 (tools/k5_probe.py, same workload, A/B on one box each; the write pass
// was 5.73 ms before): sink variants, all byte-identical output —
//   32-byte sectors through 3 LDS slots/lane, 16-byte stores, 4 waves  11.5 ms
//     (3 waves, 36 KB text window: 8.1 ms; WRITE_SIZE 10.7 -> 8.0 GB)
//   aligned 8-byte words, byte-masked first/last word                  +32 %
//   16-byte pending word (two registers), 4 / 3 waves                  +17 / +31 %
//   32-bit span-relative positions                                     +4 %
//   pieces concatenated in registers before the sink (Dec-style)       +24 %
// and what helped: the variant-class strings as constant literals (a string
// chosen at run time was measured and copied a byte at a time from memory:
// write 5.43 -> 4.34 ms, size 2.80 -> 2.26 ms) and ranking each tile's lines
// by shape (-3 %).  SQ/TA counters put the remaining time in VALU issue
// (1.8e9 wave-instructions per launch) and the texture path (TD busy 90 %):
// the lanes' 8-byte stores touch 64 lines per instruction, but every
// alternative above that makes them wider or aligned costs more instructions
// than it saves.
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef __attribute__((address_space(1))) U64u* gw_u64u;
// per SIMD: the text window's LDS allows 4 workgroups per CU (re-checked after
// the append sink: 4 waves with ~100 B of spills 5.5 ms, 3 waves without 6.2 ms)
#ifndef AVDB_K5_WAVES
#define AVDB_K5_WAVES 4  // A/B knob
#endif
constexpr int kFormatWaves = AVDB_K5_WAVES;

// decimal digit count of v (compare chain: no division)
AVDB_HD uint32_t ndigits(uint32_t v) {
  return 1u + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) +
         (v >= 1000000u) + (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}

// v < 10^8 as exactly 8 ASCII digits (leading zeros), most significant digit in
// the lowest byte: SWAR in one 64-bit register — two 4-digit halves in 32-bit
// lanes, each split into 2-digit pairs (x/100 = x*5243 >> 19 for x < 10^4) in
// 16-bit lanes, each into tens / ones (x/10 = x*103 >> 10 for x < 100) in bytes.
// About 20 VALU instructions instead of a divide-by-10 loop per digit.
AVDB_HD uint64_t ascii8(uint32_t v) {
  const uint32_t a = v / 10000u, b = v - a * 10000u;
  uint64_t x = uint64_t(a) | (uint64_t(b) << 32);
  const uint64_t q = ((x * 5243ull) >> 19) & 0x0000007F0000007Full;
  x = q | ((x - q * 100ull) << 16);
  const uint64_t t = ((x * 103ull) >> 10) & 0x000F000F000F000Full;
  x = t | ((x - t * 10ull) << 8);
  return x + 0x3030303030303030ull;
}

// decimal digits of v as nibbles, most significant digit in the lowest nibble: a
// divide-by-10 loop with few live registers (the K5 write pass, which runs at its
// register limit, keeps this form: the SWAR form above spilled 124 -> 232 B/lane
// there and cost +7 %)
__device__ __forceinline__ uint64_t dec_nibbles(uint32_t v, uint32_t* ndig) {
  uint64_t d = 0;
  uint32_t k = 0;
  do { d = (d << 4) | (v % 10u); v /= 10u; ++k; } while (v);
  *ndig = k;
  return d;
}

__device__ __forceinline__ uint64_t nibbles_to_ascii(uint64_t d, uint32_t k) {  // k <= 8
  uint64_t y = d & 0xFFFFFFFFull;
  y = (y | (y << 16)) & 0x0000FFFF0000FFFFull;
  y = (y | (y << 8)) & 0x00FF00FF00FF00FFull;
  y = (y | (y << 4)) & 0x0F0F0F0F0F0F0F0Full;
  return (y + 0x3030303030303030ull) & low_bytes_mask(k);
}

// a decimal number as ASCII text in registers (up to 16 digits), so a value
// printed several times per line is converted once
struct Dec {
  uint64_t lo, hi;  // digits 0..7 and 8..15, little-endian bytes
  uint32_t n;
};

AVDB_HD Dec dec_text(uint32_t v) {
  // branch-free: the low 8 digits are converted either way, and the count of the
  // number's digits comes from them (the lowest nonzero digit byte is its first
  // digit: (d + 0x7F) sets bit 7 of each byte d >= 1, no carries for d <= 9)
  // instead of a chain of ten compares
  const uint32_t hi = v / 100000000u;  // 0..42
  const uint64_t b = ascii8(v - hi * 100000000u);
  const uint64_t nz = ((b - 0x3030303030303030ull) + 0x7F7F7F7F7F7F7F7Full) & kHiBits;
  const uint32_t nlo = nz ? 8u - (uint32_t(__builtin_ctzll(nz)) >> 3) : 1u;  // digits of v < 10^8
  const uint32_t nh = hi >= 10u ? 2u : 1u;
  const uint64_t a = hi < 10u ? uint64_t('0' + hi)
                              : (uint64_t('0' + hi / 10u) | (uint64_t('0' + hi % 10u) << 8));
  const uint64_t lo8 = b >> (8 * (8 - nlo));
  return hi ? Dec{a | (b << (8 * nh)), b >> (64 - 8 * nh), 8u + nh} : Dec{lo8, 0ull, nlo};
}

typedef __attribute__((address_space(3))) uint64_t lds_u64;
struct LdsImage {};  // constructor tag of the LDS sink

// LDS = true (WRITE only): the sink renders into a workgroup's LDS image of its
// output span instead of global memory, for a coalesced flush afterwards.  Every
// LDS access is an aligned 8-byte word: the words a lane shares with its
// neighbours (the first and the last of its span) must be merged, so every word
// goes to the zeroed image as a ds_or_b64 (plain ds_write_b64 inside a lane's span
// with a first-word branch measured slower, profiles/k7_ab/r04_sink_allor_ab.log).
template <bool WRITE, bool LDS = false>
struct Out {
  static constexpr bool kWrite = WRITE;
  using Counter = Out<false>;  // a sink of the same family that only counts bytes
  gbyte* base;
  uint64_t p, lo;
  bool bad;  // set by a formatter that cannot render its input (line goes to the host)
  __device__ __forceinline__ Out(uint8_t* b, uint64_t at)
      : base((gbyte*)b), p(at), lo(at), bad(false) {}
  // LDS sink: `at` is the byte offset in the image (same alignment mod 8 as the
  // global destination)
  __device__ __forceinline__ Out(LdsImage, lds_u64* img, uint64_t at) : base(nullptr), p(at), lo(at), bad(false) {
    if constexpr (LDS) {
      pend.img = img;
      pend.k = uint32_t(at & 7u);
      pend.wq = uint32_t(at >> 3);
    }
  }
  __device__ __forceinline__ uint32_t size() const { return uint32_t(p - lo); }
  struct Pending {  // WRITE: bytes [p-k, p) not yet stored
    uint64_t w = 0;
    uint32_t k = 0;
  };
  struct LPending {  // LDS: bytes [p-k, p) of the current aligned word (the first
    uint64_t w = 0;  // word's low bytes belong to the previous lane: zero here)
    uint32_t k = 0;
    uint32_t wq = 0;  // image word of byte p - k (32-bit: no 64-bit address math per append)
    lds_u64* img = nullptr;
  };
  struct None {};
  [[no_unique_address]] std::conditional_t<WRITE, std::conditional_t<LDS, LPending, Pending>, None> pend;
  // append t (1..8) bytes, little-endian in x (bytes of x at and above t are 0)
  __device__ __forceinline__ void append(uint64_t x, uint32_t t) {
    if constexpr (WRITE && LDS) {
      const uint32_t k = pend.k;  // 0..7
      pend.w |= x << (8 * k);
      if (k + t >= 8) {
        lds_u64* wp = pend.img + pend.wq;
        __hip_atomic_fetch_or(wp, pend.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ++pend.wq;
        pend.w = k ? x >> (64 - 8 * k) : 0ull;
        pend.k = k + t - 8;
      } else {
        pend.k = k + t;
      }
    } else if constexpr (WRITE) {
      const uint32_t k = pend.k;  // 0..7
      pend.w |= x << (8 * k);
      if (k + t >= 8) {
        reinterpret_cast<gw_u64u>(base + p - k)->v = pend.w;
        pend.w = k ? x >> (64 - 8 * k) : 0ull;
        pend.k = k + t - 8;
      } else {
        pend.k = k + t;
      }
    }
    p += t;
  }
  __device__ __forceinline__ void put(uint32_t c) { append(c & 0xFFu, 1); }
  // end of the line: store the buffered tail
  __device__ __forceinline__ void finish() {
    if constexpr (WRITE && LDS) {
      // the last (partial) word may be shared with the next lane (an empty text
      // ORs a zero word: harmless)
      if (pend.k)
        __hip_atomic_fetch_or(pend.img + pend.wq, pend.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      pend.w = 0;
      pend.k = 0;
    } else if constexpr (WRITE) {
      // the k < 8 buffered bytes as at most one 4-, one 2- and one 1-byte store
      // (unaligned: gfx950's unaligned-access mode) instead of k byte stores
      const uint32_t k = pend.k;
      gbyte* q = base + p - k;
      uint64_t w = pend.w;
      if (k & 4) {
        reinterpret_cast<__attribute__((address_space(1))) U32u*>(q)->v = uint32_t(w);
        q += 4;
        w >>= 32;
      }
      if (k & 2) {
        reinterpret_cast<__attribute__((address_space(1))) U16u*>(q)->v = uint16_t(w);
        q += 2;
        w >>= 16;
      }
      if (k & 1) *q = uint8_t(w);
      pend.w = 0;
      pend.k = 0;
    }
  }
  // (literal strings: the length and the 8-byte chunks fold at compile time)
  __device__ __forceinline__ void lit(const char* s) {
    uint32_t n = 0;
    while (s[n]) ++n;
    for (uint32_t i = 0; i < n; i += 8) {
      const uint32_t t = n - i < 8u ? n - i : 8u;
      uint64_t x = 0;
      for (uint32_t j = 0; j < t; ++j) x |= uint64_t(uint8_t(s[i + j])) << (8 * j);
      append(x, t);
    }
  }
  template <class CP>
  __device__ __forceinline__ void bytes(CP s, uint32_t n) {
    if constexpr (!WRITE) {
      p += n;
    } else if constexpr (std::is_same_v<CP, lds_cp> || std::is_same_v<CP, glb_cp>) {
      // aligned 8-byte text words, up to 8 bytes per append
      const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(s)) & 7u;
      const typename Word64<CP>::T w = reinterpret_cast<typename Word64<CP>::T>(s - mis);
      for (uint32_t i = 0; i < n;) {
        const uint32_t q = mis + i, o = q & 7u;
        const uint32_t t = (8u - o) < (n - i) ? 8u - o : n - i;
        append((w[q >> 3] >> (8 * o)) & low_bytes_mask(t), t);
        i += t;
      }
    } else {
      for (uint32_t k = 0; k < n; ++k) put(s[k]);
    }
  }
  __device__ __forceinline__ void dec(const Dec& t) {
    if constexpr (!WRITE) {
      p += t.n;
    } else {
      append(t.lo, t.n < 8 ? t.n : 8);
      if (t.n > 8) append(t.hi, t.n - 8);
    }
  }
  __device__ __forceinline__ void u32v(uint32_t v) {
    if constexpr (!WRITE) {
      p += ndigits(v);
      return;
    }
    if constexpr (LDS) {  // K7's LDS sink: SWAR conversion
      dec(dec_text(v));
    } else {
      uint32_t k;
      const uint64_t d = dec_nibbles(v, &k);
      if (k > 8) {
        append(nibbles_to_ascii(d, 8), 8);
        append(nibbles_to_ascii(d >> 32, k - 8), k - 8);
      } else {
        append(nibbles_to_ascii(d, k), k);
      }
    }
  }
  __device__ __forceinline__ void u64v(uint64_t v) {
    if (v <= 0xFFFFFFFFull) { u32v(uint32_t(v)); return; }
    const uint64_t q = v / 1000000000ull;
    if (q <= 0xFFFFFFFFull) {
      u32v(uint32_t(q));
    } else {
      u32v(uint32_t(q / 1000000000ull));
      dec9(uint32_t(q % 1000000000ull));
    }
    dec9(uint32_t(v % 1000000000ull));
  }
  __device__ __forceinline__ void dec9(uint32_t v) {  // exactly 9 digits, zero-padded
    if constexpr (!WRITE) {
      p += 9;
      return;
    }
    const uint32_t hi = v / 100000000u;  // 0..9
    append(uint64_t('0' + hi), 1);
    append(ascii8(v - hi * 100000000u), 8);
  }
};

// The sink interface of Out<> over a host byte buffer, for the library's per-call
// host entries (K8h avdb_small_prep_host, K5h avdb_vcf_line_host): the AVDB_HD
// renderers below run unchanged into it.  base == nullptr counts bytes only.
struct HostOut {
  static constexpr bool kWrite = true;
  using Counter = HostOut;
  uint8_t* base;
  uint64_t p, lo;
  bool bad;
  HostOut(uint8_t* b, uint64_t at) : base(b), p(at), lo(at), bad(false) {}
  uint32_t size() const { return uint32_t(p - lo); }
  void append(uint64_t x, uint32_t t) {
    if (base)
      for (uint32_t j = 0; j < t; ++j) base[p + j] = uint8_t(x >> (8 * j));
    p += t;
  }
  void put(uint32_t c) { append(c & 0xFFu, 1); }
  void finish() {}
  void lit(const char* s) {
    for (; *s; ++s) put(uint8_t(*s));
  }
  void bytes(const uint8_t* s, uint32_t n) {
    if (base)
      for (uint32_t j = 0; j < n; ++j) base[p + j] = s[j];
    p += n;
  }
  void dec(const Dec& t) {
    append(t.lo, t.n < 8 ? t.n : 8);
    if (t.n > 8) append(t.hi, t.n - 8);
  }
  void u32v(uint32_t v) { dec(dec_text(v)); }
  void u64v(uint64_t v) {
    char t[20];
    int k = 0;
    do { t[k++] = char('0' + v % 10u); v /= 10u; } while (v);
    while (k) put(uint8_t(t[--k]));
  }
};

// ---------------------------------------------------------------------------
// LDS-image spans (K7 keys / paths, K0 allele heap)
// ---------------------------------------------------------------------------
// bytes [lo, hi) (0 <= lo < hi <= 16) of the 16-byte value (v0, v1) to the
// 16-aligned global chunk at a, as naturally aligned 1/2/4/8-byte stores:
// straight-line and predicated (at most 8 stores), not a 16-step byte loop
__device__ __forceinline__ void store_part16(uint8_t* out, uint64_t a, uint32_t lo, uint32_t hi, uint64_t v0,
                                             uint64_t v1) {
  auto bytes_at = [&](uint32_t s) -> uint64_t {  // value bytes from s on (s < 16)
    return s == 0 ? v0 : (s < 8 ? (v0 >> (8 * s)) | (v1 << (64 - 8 * s)) : v1 >> (8 * (s - 8)));
  };
  uint32_t s = lo;
  if ((s & 1) && s < hi) { out[a + s] = uint8_t(bytes_at(s)); s += 1; }
  if ((s & 2) && s + 2 <= hi) { *reinterpret_cast<uint16_t*>(out + a + s) = uint16_t(bytes_at(s)); s += 2; }
  if ((s & 4) && s + 4 <= hi) { *reinterpret_cast<uint32_t*>(out + a + s) = uint32_t(bytes_at(s)); s += 4; }
  if ((s & 8) && s + 8 <= hi) { *reinterpret_cast<uint64_t*>(out + a + s) = bytes_at(s); s += 8; }
  if (s + 8 <= hi) { *reinterpret_cast<uint64_t*>(out + a + s) = bytes_at(s); s += 8; }
  if (s + 4 <= hi) { *reinterpret_cast<uint32_t*>(out + a + s) = uint32_t(bytes_at(s)); s += 4; }
  if (s + 2 <= hi) { *reinterpret_cast<uint16_t*>(out + a + s) = uint16_t(bytes_at(s)); s += 2; }
  if (s < hi) out[a + s] = uint8_t(bytes_at(s));
}

// A tile's output span [g0, g1) leaves its LDS image (image byte 0 = address
// g0 & ~15), written by `nt` threads (a wave or a workgroup; `t` = this thread's
// rank among them): full 16-byte chunks as coalesced nontemporal stores, then
// the partial head and tail chunks (shared with the neighbouring tiles) by ranks
// 0 and 1 together.  Every image word read is zeroed again.
__device__ __forceinline__ void flush_span(lds_u64* img, uint8_t* out, uint64_t g0, uint64_t g1, uint32_t lane,
                                           uint32_t nt) {
  const uint64_t a0 = g0 & ~uint64_t(15);
  const uint64_t f0 = (g0 + 15) & ~uint64_t(15), f1 = g1 & ~uint64_t(15);  // full chunks [f0, f1)
  if (f1 > f0) {
    for (uint64_t q = (f0 - a0) / 16 + lane; q < (f1 - a0) / 16; q += nt) {
      const uint64_t lo = img[2 * q], hi = img[2 * q + 1];
      img[2 * q] = 0;
      img[2 * q + 1] = 0;
      __builtin_nontemporal_store(u32x4{uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32)},
                                  reinterpret_cast<u32x4*>(out + a0 + 16 * q));
    }
  }
  // head: the chunk at a0 when g0 is not 16-aligned (it may also hold g1);
  // tail: the chunk at f1 when g1 is not 16-aligned and it is not the head's
  const bool head = g0 != f0 || f1 < f0;
  const bool tail = (g1 & 15) && f1 >= f0 && (f1 != a0 || !head);
  if ((lane == 0 && head) || (lane == 1 && tail)) {
    const uint64_t a = lane == 0 ? a0 : f1;
    const uint64_t q = (a - a0) / 16;
    const uint64_t v0 = img[2 * q], v1 = img[2 * q + 1];
    img[2 * q] = 0;
    img[2 * q + 1] = 0;
    const uint32_t lo = a < g0 ? uint32_t(g0 - a) : 0u;
    const uint32_t hi = a + 16 > g1 ? uint32_t(g1 - a) : 16u;
    store_part16(out, a, lo, hi, v0, v1);
  }
}

// contig label (Util/lib/python/enums/chromosomes.py:9-38 order)
template <class O>
AVDB_HD void chrom_name(O& o, uint32_t c) {
  if (c < 9) o.put('1' + c);
  else if (c < 22) o.append(uint64_t('0' + (c + 1) / 10u) | (uint64_t('0' + (c + 1) % 10u) << 8), 2);
  else if (c == 22) o.put('X');
  else if (c == 23) o.put('Y');
  else if (c == 24) o.put('M');
  else o.u32v(c);  // contigs beyond the human 25: numeric label (matches avdb_format_bin_path)
}

// ltree path of a bin code (generate_bin_index_references.py:54,60-61,74): one
// 6- or 7-byte append per level (".L<l>.B<b>").
// Helpers take and return the sink by value (never by reference: a sink whose
// address escapes lives in scratch memory); all are inlined (see the A/B above).
// A leaf (level-13) path of a labelled contig has a fixed shape: "chr" + a
// 1- or 2-byte label + 9 six-byte and 4 seven-byte level pieces (86 / 87
// bytes), each piece's bin digit '1' or '2' (L1: '1'..'4').  It is rendered as
// eleven compile-time template words with the label and the 13 digit bits added
// at constant byte positions (~40 instructions instead of a per-level loop).
// Leaves are what SNVs and short indels get: nearly every record.
template <uint32_t L>
struct LeafPath {
  static constexpr uint32_t kLen = 3 + L + 9 * 6 + 4 * 7;
  static constexpr uint32_t digit_pos(uint32_t l) {  // byte index of level l's bin digit
    return l < 10 ? 3 + L + 6 * (l - 1) + 5 : 3 + L + 54 + 7 * (l - 10) + 6;
  }
  static constexpr uint8_t byte(uint32_t i) {
    if (i < 3) return "chr"[i];
    if (i < 3 + L) return 0;  // label, added at run time
    uint32_t k = i - (3 + L);
    if (k < 54) {
      const uint32_t l = k / 6 + 1, off = k % 6;
      const char piece[6] = {'.', 'L', char('0' + l), '.', 'B', '1'};
      return uint8_t(piece[off]);
    }
    k -= 54;
    if (k >= 28) return 0;
    const uint32_t l = 10 + k / 7, off = k % 7;
    const char piece[7] = {'.', 'L', '1', char('0' + l - 10), '.', 'B', '1'};
    return uint8_t(piece[off]);
  }
  static constexpr uint64_t word(uint32_t j) {
    uint64_t w = 0;
    for (uint32_t b = 0; b < 8; ++b) w |= uint64_t(byte(8 * j + b)) << (8 * b);
    return w;
  }
};

// W32: the caller's choice (K7: 32-bit halves; K5's write pass keeps the 64-bit
// form: the 32-bit one moved its spills from SGPRs to scratch, 172 -> 288 B/lane)
template <uint32_t L, uint32_t J, bool W32 = false>
AVDB_HD uint64_t leaf_word(uint64_t label, uint32_t g) {  // word J of the path
  using P = LeafPath<L>;
  if constexpr (W32) {
    // Each half is its template literal plus the label / digit bytes (a digit
    // byte is '1' + 0..8: no carry between bytes, so two 32-bit adds).  A 32-bit
    // literal is an operand of the add itself; 64-bit template constants were
    // hoisted out of K7's tile loop into SGPR pairs, which ran out and spilled
    // to VGPR lanes (a v_readlane / v_writelane pair per word and tile).
    constexpr uint64_t T = P::word(J);
    uint32_t lo = 0, hi = 0;
    if constexpr (J == 0) {
      lo |= uint32_t(label << 24);
      hi |= uint32_t(label >> 8);
    }
    if constexpr (P::digit_pos(1) / 8 == J) {
      constexpr uint32_t p = P::digit_pos(1) % 8;
      if constexpr (p < 4) lo |= (g >> 12) << (8 * p); else hi |= (g >> 12) << (8 * (p - 4));
    }
#pragma unroll
    for (uint32_t l = 2; l <= 13; ++l)
      if (P::digit_pos(l) / 8 == J) {
        const uint32_t p = P::digit_pos(l) % 8, b = (g >> (13 - l)) & 1u;
        if (p < 4) lo |= b << (8 * p); else hi |= b << (8 * (p - 4));
      }
#if defined(__HIP_DEVICE_COMPILE__)
    // the literals are materialised where they are used (SALU moves, issued beside
    // the VALU): loop-invariant constants are otherwise hoisted out of the tile loop
    // into registers the loop does not have
    uint32_t tlo, thi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(tlo) : "n"(uint32_t(T)));
    asm volatile("s_mov_b32 %0, %1" : "=s"(thi) : "n"(uint32_t(T >> 32)));
    return (uint64_t(thi + hi) << 32) | uint32_t(tlo + lo);
#else
    return (uint64_t(uint32_t(T >> 32) + hi) << 32) | uint32_t(uint32_t(T) + lo);
#endif
  } else {
    uint64_t w = P::word(J);
    if constexpr (J == 0) w |= label << 24;
    if constexpr (P::digit_pos(1) / 8 == J) w += uint64_t(g >> 12) << (8 * (P::digit_pos(1) % 8));
#pragma unroll
    for (uint32_t l = 2; l <= 13; ++l)
      if (P::digit_pos(l) / 8 == J) w += uint64_t((g >> (13 - l)) & 1u) << (8 * (P::digit_pos(l) % 8));
    return w;
  }
}

// each word is built just before it is appended (one live word: the K5 write
// pass runs at its register limit)
template <uint32_t L, bool W32 = false, class O>
AVDB_HD O leaf_path(O o, uint64_t label, uint32_t g) {
  o.append(leaf_word<L, 0, W32>(label, g), 8);
  o.append(leaf_word<L, 1, W32>(label, g), 8);
  o.append(leaf_word<L, 2, W32>(label, g), 8);
  o.append(leaf_word<L, 3, W32>(label, g), 8);
  o.append(leaf_word<L, 4, W32>(label, g), 8);
  o.append(leaf_word<L, 5, W32>(label, g), 8);
  o.append(leaf_word<L, 6, W32>(label, g), 8);
  o.append(leaf_word<L, 7, W32>(label, g), 8);
  o.append(leaf_word<L, 8, W32>(label, g), 8);
  o.append(leaf_word<L, 9, W32>(label, g), 8);
  o.append(leaf_word<L, 10, W32>(label, g), LeafPath<L>::kLen - 80);
  return o;
}

template <bool W32 = false, class O>
AVDB_HD O bin_path(O o, uint32_t c, uint32_t code) {
  const uint32_t level = code >> 28, g = code & 0x0FFFFFFFu;
  if (level == 13 && c < 25 && (g >> 12) < 9) {
    if (c < 9) return leaf_path<1, W32>(o, uint64_t('1' + c), g);
    if (c < 22) return leaf_path<2, W32>(o, uint64_t('0' + (c + 1) / 10u) | (uint64_t('0' + (c + 1) % 10u) << 8), g);
    return leaf_path<1, W32>(o, c == 22 ? uint64_t('X') : (c == 23 ? uint64_t('Y') : uint64_t('M')), g);
  }
  o.lit("chr");
  chrom_name(o, c);
  for (uint32_t l = 1; l <= level; ++l) {
    const uint32_t gl = g >> (level - l);
    const uint32_t b = l == 1 ? gl + 1 : (gl & 1u) + 1;
    if (b >= 10) {  // L1 of a contig longer than 576 Mb (custom chromosome tables)
      o.lit(".L");
      o.u32v(l);
      o.lit(".B");
      o.u32v(b);
    } else if (l < 10) {
      o.append(0x000000422E004C2Eull | (uint64_t('0' + l) << 16) | (uint64_t('0' + b) << 40), 6);
    } else {
      o.append(0x00422E00314C2Eull | (uint64_t('0' + l - 10) << 24) | (uint64_t('0' + b) << 48), 7);
    }
  }
  return o;
}

// ---- K7 text sizes (shared by K7's group-totals pass and the keyed K2) ----
// bytes of bin_path(c, code) in closed form: "chr" + label + 6 bytes per level
// up to L9, 7 from L10 on, and the extra digits of an L1 bin number >= 10
AVDB_HD uint32_t bin_path_size(uint32_t c, uint32_t code) {
  const uint32_t level = code >> 28, g = code & 0x0FFFFFFFu;
  const uint32_t label = c < 9 ? 1u : (c < 22 ? 2u : (c < 25 ? 1u : ndigits(c)));
  uint32_t n = 3u + label + 6u * (level < 9u ? level : 9u) + 7u * (level > 9u ? level - 9u : 0u);
  if (level) n += ndigits((g >> (level - 1)) + 1u) - 1u;
  return n;
}

__device__ __forceinline__ uint32_t ndigits64(uint64_t v) {
  if (v <= 0xFFFFFFFFull) return ndigits(uint32_t(v));
  const uint64_t q = v / 1000000000ull;
  return 9u + (q <= 0xFFFFFFFFull ? ndigits(uint32_t(q)) : 9u + ndigits(uint32_t(q / 1000000000ull)));
}

// The key's layout, one definition for every kernel that needs it (the sizes, K7's
// "label:pos:" prefix, the digest fill): the contig label of code c (0..24:
// chromosomes.py:9-38 without "chr") is 1 or 2 bytes, and the body (ref:alt or
// the 32 digest characters) starts after "label:pos:".
__device__ __forceinline__ uint32_t key_label_width(uint32_t c) { return (c >= 9 && c < 22) ? 2u : 1u; }
__device__ __forceinline__ uint32_t key_body_at(uint32_t c, uint32_t p) { return key_label_width(c) + 2u + ndigits(p); }

// bytes of primary_key_generator.py:106-122's key for a labelled contig
__device__ __forceinline__ uint32_t key_size(uint32_t c, uint32_t p, uint32_t r, uint32_t a, uint64_t e, bool lng) {
  return key_body_at(c, p) + (lng ? uint32_t(AVDB_DIGEST_CHARS) : r + 1u + a) +
         ((e && !(e >> 63)) ? 3u + ndigits64(e) : 0u);
}

// the key and path sizes K7's write pass gives a record (SoA-decidable states only):
// n_key_chrom labelled contigs, keys of long records only with digests, paths only
// with bin codes
__device__ __forceinline__ void key_path_sizes(uint32_t c, uint32_t p, uint32_t r, uint32_t a, uint64_t e, uint32_t cd,
                                               uint32_t max_seq_len, uint32_t n_key_chrom, bool has_digest,
                                               bool has_code, uint32_t* ks, uint32_t* ps) {
  const bool lg = uint64_t(r) + a > max_seq_len;
  *ks = (c < n_key_chrom && !(e >> 63) && !(lg && !has_digest)) ? key_size(c, p, r, a, e, lg) : 0u;
  *ps = (has_code && cd != AVDB_BIN_NONE && c < n_key_chrom) ? bin_path_size(c, cd) : 0u;
}

// ---------------------------------------------------------------------------
// JSON strings (json.dumps, ensure_ascii): '"' '\\' and the short escapes,
// other bytes outside ' '..'~' as \u00XX (lowercase hex)
// ---------------------------------------------------------------------------
template <bool ESC, class O, class CP>
AVDB_HD void jstr(O& o, CP s, uint32_t n) {
  if constexpr (!ESC) {
    o.bytes(s, n);
  } else {
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t c = s[i];
      if (c >= 0x20 && c < 0x7F && c != '"' && c != '\\') { o.put(c); continue; }
      o.put('\\');
      switch (c) {
        case '"': o.put('"'); break;
        case '\\': o.put('\\'); break;
        case '\n': o.put('n'); break;
        case '\r': o.put('r'); break;
        case '\t': o.put('t'); break;
        case '\b': o.put('b'); break;
        case '\f': o.put('f'); break;
        default: {
          const char* hx = "0123456789abcdef";
          o.lit("u00");
          o.put(uint8_t(hx[c >> 4]));
          o.put(uint8_t(hx[c & 15]));
        }
      }
    }
  }
}

// an allele in its display form: bytes, or '-' for an empty normalized allele
// (variant_annotator.py:111-116, snvDivMinus=True)
template <class CP>
struct Al {
  CP p;
  uint32_t n;
  bool dash;
};

template <bool ESC, class O, class CP>
AVDB_HD void al_str(O& o, const Al<CP>& a) {
  if (a.dash) o.put('-');
  else jstr<ESC>(o, a.p, a.n);
}

// truncate(s, cap) = s if len(s) <= cap else s[:cap] + '...' (variant_annotator.py:8-10)
template <bool ESC, class O, class CP>
AVDB_HD void al_trunc(O& o, const Al<CP>& a, uint32_t cap) {
  if (a.dash) { o.put('-'); return; }
  jstr<ESC>(o, a.p, a.n < cap ? a.n : cap);
  if (a.n > cap) o.lit("...");
}

// ', "variant_class": .., "variant_class_abbrev": ..' of a display class
// (variant_annotator.py:150-239).  Constant literals per case: a string chosen
// at run time would be measured and copied a byte at a time from memory.
template <class O>
AVDB_HD void variant_class_text(O& o, int cls, bool dup) {
  switch (cls) {
    case 0: o.lit(", \"variant_class\": \"single nucleotide variant\", \"variant_class_abbrev\": \"SNV\""); break;
    case 1: o.lit(", \"variant_class\": \"inversion\", \"variant_class_abbrev\": \"MNV\""); break;
    case 2: o.lit(", \"variant_class\": \"substitution\", \"variant_class_abbrev\": \"MNV\""); break;
    case 3:
    case 4: o.lit(", \"variant_class\": \"indel\", \"variant_class_abbrev\": \"INDEL\""); break;
    case 5:
      if (dup) o.lit(", \"variant_class\": \"duplication\", \"variant_class_abbrev\": \"DUP\"");
      else o.lit(", \"variant_class\": \"insertion\", \"variant_class_abbrev\": \"INS\"");
      break;
    default: o.lit(", \"variant_class\": \"deletion\", \"variant_class_abbrev\": \"DEL\""); break;
  }
}

// The display class and coordinates of one record (variant_annotator.py:147-239):
// the common prefix l (__normalize_alleles :100-107; SNVs untouched, :97-98),
// cls 0 SNV, 1 inversion, 2 substitution, 3 indel, 4 indel (insertion downstream
// of POS), 5 insertion / duplication, 6 deletion; dup: the 'dup' prefix.
template <class CP>
struct DisplayShape {
  uint32_t l, ls, le;
  int cls;
  bool dup, snv;
  Al<CP> nref, nalt, orig;
};

template <class CP>
AVDB_HD DisplayShape<CP> display_shape(uint32_t pos, uint32_t end, CP ref, uint32_t r, CP alt, uint32_t a) {
  DisplayShape<CP> d;
  d.snv = r == 1u && a == 1u;
  uint32_t l = 0;
  if (!d.snv) {
    const uint32_t m = r < a ? r : a;
    while (l < m && ref[l] == alt[l]) ++l;
  }
  const uint32_t nr = r - l, na = a - l;
  d.l = l;
  d.nref = Al<CP>{ref + l, nr, l > 0 && nr == 0};
  d.nalt = Al<CP>{alt + l, na, l > 0 && na == 0};
  d.orig = Al<CP>{r ? ref + 1 : ref, r ? r - 1 : 0, false};
  d.ls = pos;
  d.le = pos;
  d.dup = false;
  if (d.snv) {
    d.cls = 0;
  } else if (r == a) {  // MNV (:171-189)
    bool inv = true;
    for (uint32_t i = 0; i < r && inv; ++i) inv = ref[i] == alt[r - 1 - i];
    d.cls = inv ? 1 : 2;
    d.le = end;
  } else if (na >= 1) {  // insertion (:192-229)
    d.ls = pos + 1;
    // originalRef.count(normAlt) non-overlapping and len/count == len(normAlt)
    // <=> originalRef == normAlt * k, k >= 1
    if (d.orig.n > 0 && d.orig.n % na == 0) {
      d.dup = true;
      for (uint32_t i = 0, j = 0; i < d.orig.n && d.dup; ++i) {
        d.dup = d.orig.p[i] == d.nalt.p[j];
        if (++j == na) j = 0;
      }
    }
    if (nr >= 1) { d.cls = 3; d.le = end; }
    else if (end != pos + 1) { d.cls = 4; d.le = end; }
    else { d.cls = 5; d.le = pos + 1; }
  } else {  // deletion (:231-239)
    d.cls = 6;
    d.ls = pos + 1;
    d.le = end;
  }
  return d;
}

// the 'display_allele' value of a display shape (:167-237)
template <bool ESC, class O, class CP>
AVDB_HD void display_allele_text(O& o, const DisplayShape<CP>& d, CP ref, uint32_t r, CP alt, uint32_t a) {
  const uint64_t pre = d.dup ? 0x707564ull : 0x736E69ull;  // "dup" / "ins"
  const Al<CP> raw_ref{ref, r, false}, raw_alt{alt, a, false};
  switch (d.cls) {
    case 0: al_str<ESC>(o, raw_ref); o.put('>'); al_str<ESC>(o, raw_alt); break;
    case 1: o.lit("inv"); al_str<ESC>(o, raw_ref); break;
    case 2: al_str<ESC>(o, d.nref); o.put('>'); al_str<ESC>(o, d.nalt); break;
    case 3: o.lit("del"); al_trunc<ESC>(o, d.nref, 100); o.append(pre, 3); al_trunc<ESC>(o, d.nalt, 100); break;
    case 4: o.lit("del"); al_trunc<ESC>(o, d.orig, 100); o.append(pre, 3); al_trunc<ESC>(o, d.nalt, 100); break;
    case 5: o.append(pre, 3); al_trunc<ESC>(o, d.nalt, 100); break;
    default: o.lit("del"); al_trunc<ESC>(o, d.nref, 100); break;
  }
}

// the 'sequence_allele' value of a display shape (:168-238)
template <bool ESC, class O, class CP>
AVDB_HD void sequence_allele_text(O& o, const DisplayShape<CP>& d, CP ref, uint32_t r, CP alt, uint32_t a) {
  const uint64_t pre = d.dup ? 0x707564ull : 0x736E69ull;
  const Al<CP> raw_ref{ref, r, false}, raw_alt{alt, a, false};
  switch (d.cls) {
    case 0: al_str<ESC>(o, raw_ref); o.put('/'); al_str<ESC>(o, raw_alt); break;
    case 1: al_trunc<ESC>(o, raw_ref, 8); o.put('/'); al_trunc<ESC>(o, raw_alt, 8); break;
    case 5: o.append(pre, 3); al_trunc<ESC>(o, d.nalt, 8); break;
    case 6: al_trunc<ESC>(o, d.nref, 8); o.lit("/-"); break;
    default: al_trunc<ESC>(o, d.nref, 8); o.put('/'); al_trunc<ESC>(o, d.nalt, 8); break;
  }
}

// ---------------------------------------------------------------------------
// get_display_attributes (variant_annotator.py:134-241) as json.dumps text.
// Keys in the reference's dict insertion order: location_start, location_end,
// [normalized_metaseq_id], then variant_class, variant_class_abbrev,
// display_allele, sequence_allele — except the insertion branch (:192-229),
// whose update() lists display_allele and sequence_allele first.
// chrom >= 25 writes no label in normalized_metaseq_id (the caller prepends it).
// ---------------------------------------------------------------------------
template <bool ESC, class O, class CP>
AVDB_HD O display_json(O o, uint32_t chrom, uint32_t pos, uint32_t end, CP ref, uint32_t r,
                                       CP alt, uint32_t a, Dec posd = Dec{0, 0, 0}) {
  const DisplayShape<CP> d = display_shape(pos, end, ref, r, alt, a);
  o.lit("{\"location_start\": ");
  if (posd.n && d.ls == pos) o.dec(posd);  // posd: POS as text, when the caller has it
  else o.u32v(d.ls);
  o.lit(", \"location_end\": ");
  if (posd.n && d.le == pos) o.dec(posd);
  else o.u32v(d.le);
  if (!d.snv && d.l > 0) {  // normalized id differs from the metaseq id iff a prefix was trimmed
    o.lit(", \"normalized_metaseq_id\": \"");
    if (chrom < 25) chrom_name(o, chrom);
    o.put(':');
    if (posd.n) o.dec(posd);
    else o.u32v(pos);
    o.put(':');
    al_str<ESC>(o, d.nref);
    o.put(':');
    al_str<ESC>(o, d.nalt);
    o.put('"');
  }
  const bool order_b = d.cls >= 3 && d.cls <= 5;
  if (!order_b) variant_class_text(o, d.cls, d.dup);
  o.lit(", \"display_allele\": \"");
  display_allele_text<ESC>(o, d, ref, r, alt, a);
  o.lit("\", \"sequence_allele\": \"");
  sequence_allele_text<ESC>(o, d, ref, r, alt, a);
  o.put('"');
  if (order_b) variant_class_text(o, d.cls, d.dup);
  o.put('}');
  return o;
}

// ---------------------------------------------------------------------------
// to_numeric(str) as json.dumps prints it, for the canonical subset:
//   [0-9]+            int()   -> digits without leading zeros
//   [0-9]*.[0-9]*     float() -> repr(): <= 15 significant digits round-trip to
//                     exactly those digits, fixed notation for decimal exponent
//                     -4..15, else d.ddde[+-]XX
// Anything else (signs, exponents, '_', spaces, nan/inf, > 15 significant
// digits) returns false: the line is rendered by the host.
// ---------------------------------------------------------------------------
template <class CP>
AVDB_HD bool number_plain(CP f, uint32_t n) {
  if (n == 0 || n > 40) return false;
  uint32_t dot = n, f0 = n, l0 = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (f[i] == '.') {
      if (dot != n) return false;
      dot = i;
    } else if (!is_digit(f[i])) {
      return false;
    } else if (f[i] != '0') {
      if (f0 == n) f0 = i;
      l0 = i;
    }
  }
  if (dot == n) return true;                  // int
  if (n == 1) return false;                   // "." alone
  if (f0 == n) return true;                   // 0.0
  const uint32_t nd = l0 - f0 + 1 - (f0 < dot && dot < l0 ? 1u : 0u);
  return nd <= 15;                            // repr == these digits
}


// n <= 16 text bytes at s as two registers (independent aligned word reads; the
// words hold only bytes of the text's own window, bytes past n are 0)
template <class CP>
AVDB_HD void load16(CP s, uint32_t n, uint64_t* x0, uint64_t* x1) {
  const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(s)) & 7u;
  const typename Word64<CP>::T w = reinterpret_cast<typename Word64<CP>::T>(s - mis);
  const uint32_t nw = (mis + n + 7) >> 3;
  const uint64_t w0 = nw > 0 ? w[0] : 0ull, w1 = nw > 1 ? w[1] : 0ull, w2 = nw > 2 ? w[2] : 0ull;
  const uint32_t sh = 8 * mis;
  uint64_t y0 = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  uint64_t y1 = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  y0 &= low_bytes_mask(n < 8 ? n : 8);
  y1 &= n > 8 ? low_bytes_mask(n - 8) : 0ull;
  *x0 = y0;
  *x1 = y1;
}

// bytes [a, b) (b <= 16) of the register pair (x0, x1) to the sink
template <class O>
AVDB_HD void append_pair(O& o, uint64_t x0, uint64_t x1, uint32_t a, uint32_t b) {
  if (b <= a) return;
  const uint32_t n = b - a;
  uint64_t y0, y1;
  if (a == 0) { y0 = x0; y1 = x1; }
  else if (a < 8) { y0 = (x0 >> (8 * a)) | (x1 << (64 - 8 * a)); y1 = x1 >> (8 * a); }
  else { y0 = x1 >> (8 * (a - 8)); y1 = 0; }
  o.append(y0 & low_bytes_mask(n < 8 ? n : 8), n < 8 ? n : 8);
  if (n > 8) o.append(y1 & low_bytes_mask(n - 8), n - 8);
}

// lowest / highest flagged byte index of a 16-byte mask pair (bit 7 per byte), 16 if none
AVDB_HD uint32_t first_byte16(uint64_t m0, uint64_t m1) {
  return m0 ? uint32_t(__builtin_ctzll(m0)) >> 3 : (m1 ? 8 + (uint32_t(__builtin_ctzll(m1)) >> 3) : 16u);
}
AVDB_HD uint32_t last_byte16(uint64_t m0, uint64_t m1) {
  return m1 ? 15 - (uint32_t(__builtin_clzll(m1)) >> 3) : (m0 ? 7 - (uint32_t(__builtin_clzll(m0)) >> 3) : 16u);
}

template <class O, class CP>
AVDB_HD O json_number(O o, CP f, uint32_t n) {
  // SWAR form for fields of <= 16 bytes in fixed notation (repr's decimal
  // exponent -4..15): the canonical text is the integer digits without leading
  // zeros (or "0"), '.', the fraction without trailing zeros (or "0") — two byte
  // ranges of the field, read once into registers.  Exponent forms and longer
  // fields take the digit-by-digit path below.
  constexpr bool swar = !O::kWrite;  // size pass only: in the write pass its registers spill (4.37 -> 4.86 ms)
  if (swar && n >= 1 && n <= 16) {
    uint64_t x0, x1;
    load16(f, n, &x0, &x1);
    const uint64_t m0 = low_bytes_mask(n < 8 ? n : 8) & kHiBits, m1 = (n > 8 ? low_bytes_mask(n - 8) : 0ull) & kHiBits;
    const uint64_t d0 = bytes_eq_mask(x0, '.') & m0, d1 = bytes_eq_mask(x1, '.') & m1;
    const uint64_t nd0 = nondigit_mask(x0) & m0 & ~d0, nd1 = nondigit_mask(x1) & m1 & ~d1;
    const uint32_t ndots = uint32_t(__builtin_popcountll(d0) + __builtin_popcountll(d1));
    if (nd0 | nd1 || ndots > 1 || (ndots == 1 && n == 1)) {
      o.bad = true;
      return o;
    }
    const uint64_t z0 = ~bytes_eq_mask(x0, '0') & m0 & ~d0, z1 = ~bytes_eq_mask(x1, '0') & m1 & ~d1;  // nonzero digits
    const uint32_t f0 = first_byte16(z0, z1), l0 = last_byte16(z0, z1);
    if (ndots == 0) {  // int: leading zeros stripped, at least one digit
      append_pair(o, x0, x1, f0 < n ? f0 : n - 1, n);
      return o;
    }
    const uint32_t dot = first_byte16(d0, d1);
    if (f0 == 16) {  // all zeros
      o.lit("0.0");
      return o;
    }
    const uint32_t nsig = l0 - f0 + 1 - (f0 < dot && dot < l0 ? 1u : 0u);
    if (nsig > 15) {  // repr would not be these digits
      o.bad = true;
      return o;
    }
    const int32_t k = f0 < dot ? int32_t(f0) : int32_t(f0) - 1;  // index in the digits without the dot
    const int32_t e = int32_t(dot) - 1 - k;
    if (e >= -4 && e < 16) {
      if (f0 < dot) append_pair(o, x0, x1, f0, dot);
      else o.put('0');
      o.put('.');
      if (l0 > dot) append_pair(o, x0, x1, dot + 1, l0 + 1);
      else o.put('0');
      return o;
    }
  }
  o.bad = !number_plain(f, n);
  if (o.bad) return o;
  uint32_t dot = n;
  for (uint32_t i = 0; i < n; ++i)
    if (f[i] == '.') dot = i;
  if (dot == n) {  // int
    uint32_t i = 0;
    while (i + 1 < n && f[i] == '0') ++i;
    o.bytes(f + i, n - i);
    return o;
  }
  // digits without the dot: S[k] = f[k < dot ? k : k + 1], ns = n - 1
  const uint32_t ns = n - 1;
  auto S = [&](uint32_t k) -> uint8_t { return f[k < dot ? k : k + 1]; };
  int32_t f0 = -1, l0 = -1;
  for (uint32_t k = 0; k < ns; ++k) {
    if (S(k) != '0') {
      if (f0 < 0) f0 = int32_t(k);
      l0 = int32_t(k);
    }
  }
  if (f0 < 0) { o.lit("0.0"); return o; }
  const int32_t nd = l0 - f0 + 1;
  const int32_t e = int32_t(dot) - 1 - f0;  // decimal exponent of the first significant digit
  if (e >= -4 && e < 16) {
    if (e >= 0) {
      for (int32_t k = 0; k <= e; ++k) o.put(k < nd ? S(uint32_t(f0 + k)) : '0');
      o.put('.');
      if (nd > e + 1) {
        for (int32_t k = e + 1; k < nd; ++k) o.put(S(uint32_t(f0 + k)));
      } else {
        o.put('0');
      }
    } else {
      o.lit("0.");
      for (int32_t k = 0; k < -e - 1; ++k) o.put('0');
      for (int32_t k = 0; k < nd; ++k) o.put(S(uint32_t(f0 + k)));
    }
  } else {
    o.put(S(uint32_t(f0)));
    if (nd > 1) {
      o.put('.');
      for (int32_t k = 1; k < nd; ++k) o.put(S(uint32_t(f0 + k)));
    }
    o.put('e');
    o.put(e < 0 ? '-' : '+');
    const uint32_t ae = uint32_t(e < 0 ? -e : e);
    if (ae < 10) o.put('0');
    o.u32v(ae);
  }
  return o;
}

// ':' in an allele (the reference's metaseq split raises ValueError,
// primary_key_generator.py:106) or a non-ASCII byte (outside the contract)
template <class CP>
AVDB_HD bool key_allele_ok(CP s, uint32_t n) {
  return swar_find(s, n, [](uint64_t x) { return (x & kHiBits) | bytes_eq_mask(x, ':'); }) == n;
}

}  // namespace avdb
