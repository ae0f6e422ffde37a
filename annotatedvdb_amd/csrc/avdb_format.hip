// K5 — the load driver's text outputs on the GPU (gfx950).
//
// K5b avdb_vcf_format_{size,write}: for VCF lines tokenized by K0 and processed
//   by K2 (end, bin), K4 (long-key digests) and optionally K3 (keep), writes
//   byte-exact what Load/bin/load_vcf_file.py:101-119 produces per line:
//   * COPY rows of VCFVariantLoader.__parse_alt_alleles
//     (Util/lib/python/loaders/vcf_variant_loader.py:320-343): 'chr'+chrom, primary
//     key (primary_key_generator.py:99-122), position, metaseq id
//     (variant_annotator.py:124-126), bin path (bin_index.py:75), algorithm id,
//     refSNP | NULL, True | NULL (is_multi_allelic), display attributes
//     (variant_annotator.py:134-241) and INFO FREQ allele frequencies
//     (vcf_parser.py:200-222), both as json.dumps text;
//   * the .mapping line: variant id TAB str([{'primary_key': .., 'bin_index': ..}, ..])
//     (load_vcf_file.py:116-117).
//   SIZE pass (bytes per line) -> hipCUB exclusive scans -> WRITE pass, both the
//   same templated code.  One lane per line, 256 consecutive lines per workgroup
//   with their text staged in LDS (as K0); each lane writes its own contiguous
//   span of both outputs (sink and alternatives measured: see Out below).  A
//   line the GPU does not render byte-exact (non-ASCII text,
//   allele bytes that need escaping, an unmappable record (TypeError), a key the
//   reference cannot build (':' in an allele), malformed or non-canonical FREQ
//   numbers, K0 host-resolved fields) is marked HOST and gets zero bytes; the
//   host renders it between its neighbours.
// K5a avdb_display_attributes: display-attribute JSON for any record batch
//   (allele heap), json.dumps escaping included (ASCII alleles).
#include "avdb_internal.hpp"
#include "avdb_text.hpp"

#include <hipcub/hipcub.hpp>
#include <string.h>
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
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef __attribute__((address_space(1))) U64u* gw_u64u;
// per SIMD: the text window's LDS allows 4 workgroups per CU (re-checked after
// the append sink: 4 waves with ~100 B of spills 5.5 ms, 3 waves without 6.2 ms)
constexpr int kFormatWaves = 4;

// decimal digits of v as nibbles, most significant digit in the lowest nibble
// (registers only: a local char array would live in scratch memory)
__device__ __forceinline__ uint64_t dec_nibbles(uint32_t v, uint32_t* ndig) {
  uint64_t d = 0;
  uint32_t k = 0;
  do { d = (d << 4) | (v % 10u); v /= 10u; ++k; } while (v);
  *ndig = k;
  return d;
}

__device__ __forceinline__ uint32_t ndigits(uint32_t v) {  // decimal digits
  uint32_t k = 1;
  while (v >= 10u) { v /= 10u; ++k; }
  return k;
}

// a decimal number as ASCII text in registers (up to 16 digits), so a value
// printed several times per line is converted once
struct Dec {
  uint64_t lo, hi;  // digits 0..7 and 8..15, little-endian bytes
  uint32_t n;
};

__device__ __forceinline__ uint64_t nibbles_to_ascii(uint64_t d, uint32_t k) {  // k <= 8
  uint64_t y = d & 0xFFFFFFFFull;
  y = (y | (y << 16)) & 0x0000FFFF0000FFFFull;
  y = (y | (y << 8)) & 0x00FF00FF00FF00FFull;
  y = (y | (y << 4)) & 0x0F0F0F0F0F0F0F0Full;
  return (y + 0x3030303030303030ull) & low_bytes_mask(k);
}

__device__ __forceinline__ Dec dec_text(uint32_t v) {
  uint32_t k;
  const uint64_t d = dec_nibbles(v, &k);
  return Dec{nibbles_to_ascii(d, k < 8 ? k : 8), k > 8 ? nibbles_to_ascii(d >> 32, k - 8) : 0ull, k};
}

typedef __attribute__((address_space(3))) uint64_t lds_u64;
struct LdsImage {};  // constructor tag of the LDS sink

// LDS = true (WRITE only): the sink renders into a workgroup's LDS image of its
// output span instead of global memory, for a coalesced flush afterwards.  Every
// LDS access is an aligned 8-byte word: the words a lane shares with its
// neighbours (the first and the last of its span) are merged with ds_or_b64 into
// the zeroed image, the words wholly inside its span are plain ds_write_b64.
template <bool WRITE, bool LDS = false>
struct Out {
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
    bool first = true;
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
        lds_u64* wp = pend.img + ((p - k) >> 3);
        if (pend.first) __hip_atomic_fetch_or(wp, pend.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else *wp = pend.w;
        pend.first = false;
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
      // the last (partial) word may be shared with the next lane
      if (pend.k && (p > lo || !pend.first))
        __hip_atomic_fetch_or(pend.img + ((p - pend.k) >> 3), pend.w, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
      pend.w = 0;
      pend.k = 0;
    } else if constexpr (WRITE) {
      for (uint32_t j = 0; j < pend.k; ++j) base[p - pend.k + j] = uint8_t(pend.w >> (8 * j));
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
  // up to 8 decimal digits given as nibbles (most significant lowest) -> ASCII
  __device__ __forceinline__ void digits8(uint64_t d, uint32_t k) { append(nibbles_to_ascii(d, k), k); }
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
    uint32_t k;
    const uint64_t d = dec_nibbles(v, &k);
    if (k > 8) {
      digits8(d, 8);
      digits8(d >> 32, k - 8);
    } else {
      digits8(d, k);
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
    uint64_t d = 0;
    for (int i = 0; i < 9; ++i) { d = (d << 4) | (v % 10u); v /= 10u; }
    digits8(d, 8);
    digits8(d >> 32, 1);
  }
};

// contig label (Util/lib/python/enums/chromosomes.py:9-38 order)
template <class O>
__device__ __forceinline__ void chrom_name(O& o, uint32_t c) {
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
template <class O>
__device__ __forceinline__ O bin_path(O o, uint32_t c, uint32_t code) {
  o.lit("chr");
  chrom_name(o, c);
  const uint32_t level = code >> 28, g = code & 0x0FFFFFFFu;
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

// ---------------------------------------------------------------------------
// JSON strings (json.dumps, ensure_ascii): '"' '\\' and the short escapes,
// other bytes outside ' '..'~' as \u00XX (lowercase hex)
// ---------------------------------------------------------------------------
template <bool ESC, class O, class CP>
__device__ __forceinline__ void jstr(O& o, CP s, uint32_t n) {
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
__device__ __forceinline__ void al_str(O& o, const Al<CP>& a) {
  if (a.dash) o.put('-');
  else jstr<ESC>(o, a.p, a.n);
}

// truncate(s, cap) = s if len(s) <= cap else s[:cap] + '...' (variant_annotator.py:8-10)
template <bool ESC, class O, class CP>
__device__ __forceinline__ void al_trunc(O& o, const Al<CP>& a, uint32_t cap) {
  if (a.dash) { o.put('-'); return; }
  jstr<ESC>(o, a.p, a.n < cap ? a.n : cap);
  if (a.n > cap) o.lit("...");
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
__device__ __forceinline__ O display_json(O o, uint32_t chrom, uint32_t pos, uint32_t end, CP ref, uint32_t r,
                                       CP alt, uint32_t a, Dec posd = Dec{0, 0, 0}) {
  const bool snv = r == 1u && a == 1u;
  uint32_t l = 0;  // common prefix (__normalize_alleles :100-107); SNVs untouched (:97-98)
  if (!snv) {
    const uint32_t m = r < a ? r : a;
    while (l < m && ref[l] == alt[l]) ++l;
  }
  const uint32_t nr = r - l, na = a - l;
  const Al<CP> nref{ref + l, nr, l > 0 && nr == 0}, nalt{alt + l, na, l > 0 && na == 0};
  uint32_t ls = pos, le = pos;
  int cls;  // 0 SNV, 1 inversion, 2 substitution, 3 indel, 4 indel (ins downstream), 5 ins/dup, 6 deletion
  bool dup = false;
  const Al<CP> orig{r ? ref + 1 : ref, r ? r - 1 : 0, false};
  if (snv) {
    cls = 0;
  } else if (r == a) {  // MNV (:171-189)
    bool inv = true;
    for (uint32_t i = 0; i < r && inv; ++i) inv = ref[i] == alt[r - 1 - i];
    cls = inv ? 1 : 2;
    le = end;
  } else if (na >= 1) {  // insertion (:192-229)
    ls = pos + 1;
    // originalRef.count(normAlt) non-overlapping and len/count == len(normAlt)
    // <=> originalRef == normAlt * k, k >= 1
    if (orig.n > 0 && orig.n % na == 0) {
      dup = true;
      for (uint32_t i = 0, j = 0; i < orig.n && dup; ++i) {
        dup = orig.p[i] == nalt.p[j];
        if (++j == na) j = 0;
      }
    }
    if (nr >= 1) { cls = 3; le = end; }
    else if (end != pos + 1) { cls = 4; le = end; }
    else { cls = 5; le = pos + 1; }
  } else {  // deletion (:231-239)
    cls = 6;
    ls = pos + 1;
    le = end;
  }
  o.lit("{\"location_start\": ");
  if (posd.n && ls == pos) o.dec(posd);  // posd: POS as text, when the caller has it
  else o.u32v(ls);
  o.lit(", \"location_end\": ");
  if (posd.n && le == pos) o.dec(posd);
  else o.u32v(le);
  if (!snv && l > 0) {  // normalized id differs from the metaseq id iff a prefix was trimmed
    o.lit(", \"normalized_metaseq_id\": \"");
    if (chrom < 25) chrom_name(o, chrom);
    o.put(':');
    if (posd.n) o.dec(posd);
    else o.u32v(pos);
    o.put(':');
    al_str<ESC>(o, nref);
    o.put(':');
    al_str<ESC>(o, nalt);
    o.put('"');
  }
  const char* vc;
  const char* vca;
  switch (cls) {
    case 0: vc = "single nucleotide variant"; vca = "SNV"; break;
    case 1: vc = "inversion"; vca = "MNV"; break;
    case 2: vc = "substitution"; vca = "MNV"; break;
    case 3:
    case 4: vc = "indel"; vca = "INDEL"; break;
    case 5: vc = dup ? "duplication" : "insertion"; vca = dup ? "DUP" : "INS"; break;
    default: vc = "deletion"; vca = "DEL"; break;
  }
  const bool order_b = cls >= 3 && cls <= 5;
  if (!order_b) {
    o.lit(", \"variant_class\": \"");
    o.lit(vc);
    o.lit("\", \"variant_class_abbrev\": \"");
    o.lit(vca);
    o.put('"');
  }
  const char* pre = dup ? "dup" : "ins";
  const Al<CP> raw_ref{ref, r, false}, raw_alt{alt, a, false};
  o.lit(", \"display_allele\": \"");
  switch (cls) {
    case 0: al_str<ESC>(o, raw_ref); o.put('>'); al_str<ESC>(o, raw_alt); break;
    case 1: o.lit("inv"); al_str<ESC>(o, raw_ref); break;
    case 2: al_str<ESC>(o, nref); o.put('>'); al_str<ESC>(o, nalt); break;
    case 3: o.lit("del"); al_trunc<ESC>(o, nref, 100); o.lit(pre); al_trunc<ESC>(o, nalt, 100); break;
    case 4: o.lit("del"); al_trunc<ESC>(o, orig, 100); o.lit(pre); al_trunc<ESC>(o, nalt, 100); break;
    case 5: o.lit(pre); al_trunc<ESC>(o, nalt, 100); break;
    default: o.lit("del"); al_trunc<ESC>(o, nref, 100); break;
  }
  o.lit("\", \"sequence_allele\": \"");
  switch (cls) {
    case 0: al_str<ESC>(o, raw_ref); o.put('/'); al_str<ESC>(o, raw_alt); break;
    case 1: al_trunc<ESC>(o, raw_ref, 8); o.put('/'); al_trunc<ESC>(o, raw_alt, 8); break;
    case 5: o.lit(pre); al_trunc<ESC>(o, nalt, 8); break;
    case 6: al_trunc<ESC>(o, nref, 8); o.lit("/-"); break;
    default: al_trunc<ESC>(o, nref, 8); o.put('/'); al_trunc<ESC>(o, nalt, 8); break;
  }
  o.put('"');
  if (order_b) {
    o.lit(", \"variant_class\": \"");
    o.lit(vc);
    o.lit("\", \"variant_class_abbrev\": \"");
    o.lit(vca);
    o.put('"');
  }
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
__device__ __forceinline__ bool number_plain(CP f, uint32_t n) {
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

template <class O, class CP>
__device__ __forceinline__ O json_number(O o, CP f, uint32_t n) {
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

// ---------------------------------------------------------------------------
// K5b: one VCF line
// ---------------------------------------------------------------------------
enum : uint8_t { kLineGpu = 0, kLineHost = 1, kLineSkip = 2 };

constexpr uint32_t kHostFlags = AVDB_VCF_FEW_FIELDS | AVDB_VCF_BAD_POS | AVDB_VCF_EXT_HOST |
                                AVDB_VCF_CHROM_HOST | AVDB_VCF_EMPTY | AVDB_VCF_ID_HOST;
constexpr int kMaxPops = 64;

struct FormatArgs {
  const uint8_t* text;
  size_t text_bytes;
  size_t n_lines;
  const avdb_vcf_line* lines;
  const uint64_t* rec_off;
  const uint32_t* end;
  const uint32_t* code;
  const uint8_t* status;
  const char* digest;
  const uint8_t* keep;
  uint64_t* copy_off;  // SIZE: bytes per line; WRITE: offsets
  uint64_t* map_off;
  uint8_t* line_state;
  uint8_t* copy_out;
  uint8_t* map_out;
  unsigned long long* counters;
  uint32_t max_seq_len;
  uint32_t alg_len;
  char alg[AVDB_MAX_ALG_ID];
  const int32_t* match;  // --skipExisting (K6), optional
  const uint8_t* match_kind;
  const uint8_t* frag;
  const uint64_t* frag_off;
  const uint8_t* adsp_dup;  // ADSP: per record, its primary key is already loaded (optional)
  bool adsp_col;            // ADSP: COPY rows end with is_adsp_variant = True
};

// allele bytes the GPU writes verbatim into JSON and Python repr text: printable
// ASCII except '"' '\\' '\'' (escaped by json.dumps / repr) and ':' (breaks
// metaseqId.split(':'), primary_key_generator.py:106)
// (SWAR, 8 bytes per step: bytes >= 0x80, < 0x20, 0x7F and the four specials)
template <class CP>
__device__ __forceinline__ bool plain_allele(CP s, uint32_t n) {
  return swar_find(s, n, [](uint64_t x) {
           const uint64_t lt20 = ~((x & 0x7F7F7F7F7F7F7F7Full) + 0x6060606060606060ull) & kHiBits;
           return (x & kHiBits) | lt20 | bytes_eq_mask(x, 0x7F) | bytes_eq_mask(x, '"') |
                  bytes_eq_mask(x, '\\') | bytes_eq_mask(x, '\'') | bytes_eq_mask(x, ':');
         }) == n;
}

template <class CP>
__device__ __forceinline__ bool bytes_eq(CP a, CP b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// next separator at or after i in [i, e), or e
template <class CP>
__device__ __forceinline__ uint32_t find_byte(CP s, uint32_t i, uint32_t e, uint8_t c) {
  if (i >= e) return i;
  return i + swar_find(s + i, e - i, [c](uint64_t x) { return bytes_eq_mask(x, c); });
}

// FREQ value [v0, v1) of the line: is it one the GPU renders?  Every population
// needs a ':' (pop.split(':')[1]), a JSON-plain name, and names must be unique
// (the reference's dict comprehension keeps the last value at the first
// position).
template <class CP>
__device__ bool freq_plain(CP s, uint32_t v0, uint32_t v1) {
  uint32_t np = 0;
  for (uint32_t p0 = v0; p0 <= v1; ++np) {
    const uint32_t p1 = find_byte(s, p0, v1, '|');
    const uint32_t c1 = find_byte(s, p0, p1, ':');
    if (c1 == p1 || np >= kMaxPops) return false;
    for (uint32_t i = p0; i < c1; ++i) {
      const uint8_t c = s[i];
      if (c < 0x20 || c > 0x7E || c == '"' || c == '\\') return false;
    }
    // duplicate name among the earlier populations
    for (uint32_t q0 = v0; q0 < p0;) {
      const uint32_t q1 = find_byte(s, q0, v1, '|');
      const uint32_t d1 = find_byte(s, q0, q1, ':');
      if (d1 - q0 == c1 - p0 && bytes_eq(s + q0, s + p0, c1 - p0)) return false;
      q0 = q1 + 1;
    }
    p0 = p1 + 1;
  }
  return true;
}

// allele_frequencies of ALT index k (1-based, altAlleles.index(allele) + 1) as
// json.dumps text or NULL; false when the reference would raise or print a
// number the GPU does not format
template <class O, class CP>
__device__ __forceinline__ O freq_json(O o, CP s, uint32_t v0, uint32_t v1, uint32_t k) {
  bool any = false;
  for (uint32_t p0 = v0; p0 <= v1;) {
    const uint32_t p1 = find_byte(s, p0, v1, '|');
    const uint32_t c1 = find_byte(s, p0, p1, ':');
    const uint32_t c2 = find_byte(s, c1 + 1, p1, ':');  // pop.split(':')[1]
    // item k of the comma list [c1+1, c2)
    uint32_t f0 = c1 + 1, idx = 0;
    while (idx < k) {
      const uint32_t cm = find_byte(s, f0, c2, ',');
      if (cm == c2) { o.bad = true; return o; }  // IndexError in the reference
      f0 = cm + 1;
      ++idx;
    }
    const uint32_t f1 = find_byte(s, f0, c2, ',');
    const uint32_t fn = f1 - f0;
    const bool zero = fn == 1 && (s[f0] == '.' || s[f0] == '0');
    if (!zero) {
      o.put(any ? ',' : '{');
      if (any) o.put(' ');
      o.put('"');
      o.bytes(s + p0, c1 - p0);
      o.lit("\": {\"gmaf\": ");
      o = json_number(o, s + f0, fn);
      if (o.bad) return o;
      o.put('}');
      any = true;
    }
    p0 = p1 + 1;
  }
  if (any) o.put('}');
  else o.lit("NULL");
  return o;
}

template <bool WRITE, class O, class CP>
__device__ __forceinline__ uint8_t format_line(const FormatArgs& A, const avdb_vcf_line& L, CP s, size_t li,
                               O& oc, O& om, uint32_t* n_rows, uint32_t* n_skip,
                               uint32_t* n_dup, uint32_t* n_upd) {
  if (L.flags & AVDB_VCF_COMMENT) return kLineSkip;
  if ((L.flags & kHostFlags) || L.chrom >= 25) return kLineHost;
  // Checks that only decide GPU vs HOST run in the SIZE pass; the WRITE pass
  // only visits lines that passed them (line_state == GPU).
  // the reference decodes every line as UTF-8 (load_vcf_file.py:102): ASCII only here
  if constexpr (!WRITE) {
    if (swar_find(s, L.len, [](uint64_t x) { return x & kHiBits; }) != L.len) return kLineHost;
  }
  const uint32_t c = L.chrom;
  const uint32_t ref0 = L.field[3], rl = L.field[4] - 1 - ref0;
  const uint32_t alt0 = L.field[4], alt1 = L.field[5] - 1;
  const CP ref = s + ref0;
  if (!WRITE && !plain_allele(ref, rl)) return kLineHost;
  // INFO: the last FREQ entry (dict keeps the last key); '#' or '\' in INFO are
  // rewritten by the reference before it splits (vcf_parser.py:101-103)
  const uint32_t i0 = L.field[7], i1 = L.field_end8;
  int64_t fq0 = -1, fq1 = -1;
  if constexpr (!WRITE) {
    if (i1 > i0 && swar_find(s + i0, i1 - i0, [](uint64_t x) {
          return bytes_eq_mask(x, '#') | bytes_eq_mask(x, '\\');
        }) != i1 - i0)
      return kLineHost;
  }
  for (uint32_t e0 = i0; e0 <= i1;) {
    const uint32_t e1 = find_byte(s, e0, i1, ';');
    if (e1 - e0 >= 4 && s[e0] == 'F' && s[e0 + 1] == 'R' && s[e0 + 2] == 'E' && s[e0 + 3] == 'Q') {
      if (e1 - e0 == 4) return kLineHost;  // bare flag -> True.split: AttributeError
      if (s[e0 + 4] == '=') { fq0 = e0 + 5; fq1 = e1; }
    }
    e0 = e1 + 1;
  }
  if (!WRITE && fq0 >= 0 && !freq_plain(s, uint32_t(fq0), uint32_t(fq1))) return kLineHost;
  const bool has_rs = (L.flags & (AVDB_VCF_ID_RS | AVDB_VCF_INFO_RS)) != 0;
  Dec posd;  // POS is printed up to 7 times per ALT
  if constexpr (WRITE) posd = dec_text(L.pos);
  else posd = Dec{0, 0, ndigits(L.pos)};
  // .mapping: variant id (vcf_parser.py:140-142) TAB '['
  if (L.flags & AVDB_VCF_ID_METASEQ) {
    chrom_name(om, c);
    om.put(':');
    om.dec(posd);
    om.put(':');
    om.bytes(ref, rl);
    om.put(':');
    om.bytes(s + alt0, alt1 - alt0);
  } else {
    om.bytes(s + L.field[2], L.field[3] - 1 - L.field[2]);
  }
  om.lit("\t[");
  uint64_t r = A.rec_off[li];
  uint32_t nrec = 0, rows = 0, skip = 0, dups = 0, upd = 0;
  for (uint32_t a0 = alt0, ai = 0; a0 <= alt1; ++ai) {
    const uint32_t a1 = find_byte(s, a0, alt1, ',');
    const CP alt = s + a0;
    const uint32_t al = a1 - a0;
    if (al == 1 && alt[0] == '.') {  // vcf_variant_loader.py:277-280
      ++skip;
      a0 = a1 + 1;
      continue;
    }
    if (!WRITE && !plain_allele(alt, al)) return kLineHost;
    const bool lng = rl + al > A.max_seq_len;
    if (lng && !A.digest) return kLineHost;
    if (A.match) {  // --skipExisting: after the key (:282), before the bin (:310)
      if (A.match_kind[r] == AVDB_MATCH_HOST) return kLineHost;
      if (A.match[r] >= 0) {  // primaryKeyMapping += matchedVariant; skipped (:287-291)
        const int32_t m = A.match[r];
        if (nrec) om.lit(", ");
        om.bytes(A.frag + A.frag_off[m], uint32_t(A.frag_off[m + 1] - A.frag_off[m]));
        ++nrec;
        ++skip;
        ++r;
        a0 = a1 + 1;
        continue;
      }
    }
    if (A.adsp_dup && A.adsp_dup[r]) {  // ADSP: key already loaded -> an is_adsp_variant UPDATE,
      ++upd;                              // no COPY row, no mapping entry (vcf_variant_loader.py:303-307)
      ++r;
      a0 = a1 + 1;
      continue;
    }
    const uint32_t st = A.status[r];
    if (st == AVDB_STATUS_UNKNOWN_CHROM || st == AVDB_STATUS_OUT_OF_RANGE) return kLineHost;
    const uint32_t code = A.code[r];
    const bool keep = !A.keep || A.keep[r];
    // altIndex = altAlleles.index(allele) + 1: the first equal ALT
    uint32_t k = ai + 1;
    for (uint32_t b0 = alt0, bi = 0; bi < ai; ++bi) {
      const uint32_t b1 = find_byte(s, b0, alt1, ',');
      if (b1 - b0 == al && bytes_eq(s + b0, alt, al)) { k = bi + 1; break; }
      b0 = b1 + 1;
    }
    // primary key (primary_key_generator.py:106-122)
    auto pk = [&](O& o) {
      chrom_name(o, c);
      o.put(':');
      o.dec(posd);
      o.put(':');
      if (lng) {
        o.bytes(reinterpret_cast<const uint8_t*>(A.digest) + 32 * r, AVDB_DIGEST_CHARS);
      } else {
        o.bytes(ref, rl);
        o.put(':');
        o.bytes(alt, al);
      }
      if (has_rs) {
        o.lit(":rs");
        o.u64v(L.ext_id);
      }
    };
    if (keep) {
      // COPY row (vcf_variant_loader.py:320-343)
      oc.lit("chr");
      chrom_name(oc, c);
      oc.put('#');
      pk(oc);
      oc.put('#');
      oc.dec(posd);
      oc.put('#');
      chrom_name(oc, c);
      oc.put(':');
      oc.dec(posd);
      oc.put(':');
      oc.bytes(ref, rl);
      oc.put(':');
      oc.bytes(alt, al);
      oc.put('#');
      oc = bin_path(oc, c, code);
      oc.put('#');
      oc.bytes(reinterpret_cast<const uint8_t*>(A.alg), A.alg_len);
      oc.put('#');
      if (has_rs) {
        oc.lit("rs");
        oc.u64v(L.ext_id);
      } else {
        oc.lit("NULL");
      }
      oc.put('#');
      oc.lit(L.n_alt > 1 ? "True" : "NULL");
      oc.put('#');
      oc = display_json<false>(oc, c, L.pos, A.end[r], ref, rl, alt, al, posd);
      oc.put('#');
      if (fq0 >= 0) {
        oc = freq_json(oc, s, uint32_t(fq0), uint32_t(fq1), k);
        if (oc.bad) return kLineHost;
      } else {
        oc.lit("NULL");
      }
      if (A.adsp_col) oc.lit("#True");  // is_adsp_variant (vcf_variant_loader.py:336-337)
      oc.put('\n');
      ++rows;
    } else {
      // no COPY row, but the reference would still have evaluated FREQ
      if (fq0 >= 0) {
        if (freq_json(Out<false>(nullptr, 0), s, uint32_t(fq0), uint32_t(fq1), k).bad) return kLineHost;
      }
      ++dups;
    }
    // .mapping entry
    if (nrec) om.lit(", ");
    om.lit("{'primary_key': '");
    pk(om);
    om.lit("', 'bin_index': '");
    om = bin_path(om, c, code);
    om.lit("'}");
    ++nrec;
    ++r;
    a0 = a1 + 1;
  }
  om.lit("]\n");
  *n_rows += rows;
  *n_skip += skip;
  *n_dup += dups;
  *n_upd += upd;
  return kLineGpu;
}

template <bool WRITE>
__global__ __launch_bounds__(kBlock, kFormatWaves) void k_vcf_format(FormatArgs A) {
  __shared__ u32x4 s_text[kStage / 16];
  const Heap h = make_heap(A.text, A.text_bytes);
  uint32_t rows = 0, skip = 0, dups = 0, hosts = 0, upds = 0;
  for (size_t base = size_t(blockIdx.x) * kBlock; base < A.n_lines; base += size_t(gridDim.x) * kBlock) {
    const size_t last = base + kBlock < A.n_lines ? base + kBlock : A.n_lines;
    const avdb_vcf_line& Z = A.lines[last - 1];
    const Window w = stage_window(h, A.lines[base].start, Z.start + Z.len, s_text);
    const size_t li = base + threadIdx.x;
    if (li < A.n_lines) {
      const avdb_vcf_line L = A.lines[li];
      // the same formatter on the LDS window (ds_read) or, for an oversized
      // window, on global memory
      auto run = [&](auto s) {
        if constexpr (WRITE) {
          const uint8_t st = A.line_state[li];
          if (st == kLineGpu) {
            Out<true> oc(A.copy_out, A.copy_off[li]), om(A.map_out, A.map_off[li]);
            format_line<true>(A, L, s, li, oc, om, &rows, &skip, &dups, &upds);
            oc.finish();
            om.finish();
          } else if (st == kLineHost) {
            ++hosts;
          }
        } else {
          Out<false> oc(nullptr, 0), om(nullptr, 0);
          const uint8_t st = format_line<false>(A, L, s, li, oc, om, &rows, &skip, &dups, &upds);
          A.line_state[li] = st;
          A.copy_off[li] = st == kLineGpu ? oc.size() : 0;
          A.map_off[li] = st == kLineGpu ? om.size() : 0;
        }
      };
      if (w.staged)
        run((lds_cp)(reinterpret_cast<const uint8_t*>(s_text) + (h.lo + L.start - w.a0)));
      else
        run((glb_cp)(A.text + L.start));
    }
    __syncthreads();  // the window is reused by the next trip
  }
  if (WRITE && A.counters) {
    for (int d = 32; d > 0; d >>= 1) {
      rows += __shfl_down(rows, d, kWave);
      skip += __shfl_down(skip, d, kWave);
      dups += __shfl_down(dups, d, kWave);
      hosts += __shfl_down(hosts, d, kWave);
      upds += __shfl_down(upds, d, kWave);
    }
    if (__lane_id() == 0) {
      if (rows) atomicAdd(&A.counters[AVDB_CTR_COPY_ROWS], (unsigned long long)rows);
      if (skip) atomicAdd(&A.counters[AVDB_CTR_SKIPPED_ALTS], (unsigned long long)skip);
      if (dups) atomicAdd(&A.counters[AVDB_CTR_DUP_ROWS], (unsigned long long)dups);
      if (hosts) atomicAdd(&A.counters[AVDB_CTR_HOST_LINES], (unsigned long long)hosts);
      if (upds) atomicAdd(&A.counters[AVDB_CTR_ADSP_UPDATES], (unsigned long long)upds);
    }
  }
}

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
// K7: primary keys (+ ltree bin paths) of a record batch; one lane per record.
// SIZE needs only the SoA (lengths, pos, ext): it never reads the heap, so it
// is a cheap streaming pass; WRITE renders the text and checks the allele bytes.
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
  const char* digest;     // nullable: long records get state NEED_DIGEST
  size_t heap_bytes, n, key_cap, path_cap;
  uint32_t max_seq_len;
  int32_t n_chrom;
  uint64_t* key_off;
  uint64_t* path_off;
  uint8_t* key_out;
  uint8_t* path_out;
  uint8_t* state;
};

// ':' in an allele (the reference's metaseq split raises ValueError,
// primary_key_generator.py:106) or a non-ASCII byte (outside the contract)
template <class CP>
__device__ __forceinline__ bool key_allele_ok(CP s, uint32_t n) {
  return swar_find(s, n, [](uint64_t x) { return (x & kHiBits) | bytes_eq_mask(x, ':'); }) == n;
}

// One stream's span of a 256-record tile is staged in LDS when it fits (always
// for keys <= ~90 B and ltree paths <= 87 B; else the lanes write global memory
// directly), then flushed with coalesced 16-byte stores: the lanes' texts are
// adjacent, so a wave of per-lane 8-byte stores would touch 64 partly written
// lines per instruction.
constexpr uint32_t kKeyStage = 24 * 1024;  // bytes per workgroup (6 workgroups per CU)

__device__ __forceinline__ void flush_tile(const lds_u64* img, uint8_t* out, uint64_t g0, uint64_t g1) {
  const uint64_t a0 = g0 & ~uint64_t(15);
  const uint64_t nchunks = (g1 - a0 + 15) / 16;
  for (uint64_t q = threadIdx.x; q < nchunks; q += blockDim.x) {
    const uint64_t a = a0 + 16 * q;
    const uint64_t lo = img[2 * q], hi = img[2 * q + 1];
    if (a >= g0 && a + 16 <= g1) {
      __builtin_nontemporal_store(u32x4{uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32)},
                                  reinterpret_cast<u32x4*>(out + a));
    } else {  // a chunk shared with the neighbouring tiles: only this tile's bytes
      for (uint32_t k = 0; k < 16; ++k) {
        if (a + k >= g0 && a + k < g1) out[a + k] = uint8_t((k < 8 ? lo : hi) >> (8 * (k & 7)));
      }
    }
  }
}

template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_record_keys(KeyArgs A) {
  __shared__ uint64_t s_img[WRITE ? kKeyStage / 8 : 1];
  lds_u64* img = (lds_u64*)s_img;
  for (size_t t0 = size_t(blockIdx.x) * blockDim.x; t0 < A.n; t0 += size_t(gridDim.x) * blockDim.x) {
    const size_t i = t0 + threadIdx.x;
    const bool live = i < A.n;
    uint32_t c = 0, p = 0, r = 0, a = 0;
    uint64_t e = 0;
    bool lng = false;
    uint8_t st = AVDB_KEY_HOST;
    if (live) {
      c = A.chrom[i];
      p = A.pos[i];
      r = A.rl[i];
      a = A.al[i];
      e = A.ext ? A.ext[i] : 0ull;
      lng = uint64_t(r) + a > A.max_seq_len;
      // SoA-decidable states; the WRITE pass adds the allele-byte checks
      st = AVDB_KEY_OK;
      if (c >= uint32_t(A.n_chrom) || (e >> 63)) st = AVDB_KEY_HOST;  // no label / interned external id
      else if (lng && !A.digest) st = AVDB_KEY_NEED_DIGEST;
    }
    auto key = [&](auto o) {  // primary_key_generator.py:106-122
      chrom_name(o, c);
      o.put(':');
      o.u32v(p);
      o.put(':');
      if (lng) {  // only reached with a digest array (st == OK)
        o.bytes((glb_cp)(A.digest + 32 * i), AVDB_DIGEST_CHARS);
      } else {
        const uint64_t off = A.off[i];
        o.bytes((glb_cp)(A.heap + off), r);
        o.put(':');
        o.bytes((glb_cp)(A.heap + off + r), a);
      }
      if (e && !(e >> 63)) {
        o.lit(":rs");
        o.u64v(e);
      }
      return o;
    };
    if constexpr (WRITE) {
      if (live && st == AVDB_KEY_OK && !lng) {
        const uint64_t off = A.off[i];
        if (off + r + a > A.heap_bytes || !key_allele_ok((glb_cp)(A.heap + off), r + a)) st = AVDB_KEY_HOST;
      }
      const size_t last = t0 + blockDim.x < A.n ? t0 + blockDim.x : A.n;
      // stream 0: keys, stream 1: paths; each staged in LDS when its span fits
      for (int sidx = 0; sidx < (A.code ? 2 : 1); ++sidx) {
        const uint64_t* offs = sidx ? A.path_off : A.key_off;
        uint8_t* out = sidx ? A.path_out : A.key_out;
        const uint64_t cap = sidx ? A.path_cap : A.key_cap;
        const uint64_t g0 = offs[t0], g1 = offs[last];
        const uint64_t a0 = g0 & ~uint64_t(15);
        const bool staged = g1 - a0 + 16 <= kKeyStage && g1 <= cap;
        uint32_t cd = AVDB_BIN_NONE;
        bool emit = false;
        if (live) {
          if (sidx == 0) {
            emit = st == AVDB_KEY_OK && offs[i + 1] <= cap;  // (cap: never write past the buffer)
          } else {
            cd = A.code[i];
            emit = cd != AVDB_BIN_NONE && c < uint32_t(A.n_chrom) && offs[i + 1] <= cap;
          }
        }
        if (staged) {
          for (uint64_t q = threadIdx.x; q < (g1 - a0 + 15) / 16; q += blockDim.x) {
            img[2 * q] = 0;
            img[2 * q + 1] = 0;
          }
          __syncthreads();
          if (emit) {
            Out<true, true> o(LdsImage{}, img, offs[i] - a0);
            if (sidx == 0) o = key(o);
            else o = bin_path(o, c, cd);
            o.finish();
          }
          __syncthreads();
          flush_tile(img, out, g0, g1);
          __syncthreads();
        } else if (emit) {
          Out<true> o(out, offs[i]);
          if (sidx == 0) o = key(o);
          else o = bin_path(o, c, cd);
          o.finish();
        }
      }
      if (live) A.state[i] = st;
    } else if (live) {
      A.key_off[i] = st == AVDB_KEY_OK ? key(Out<false>(nullptr, 0)).size() : 0;
      if (A.code) {
        const uint32_t cd = A.code[i];
        A.path_off[i] = (cd != AVDB_BIN_NONE && c < uint32_t(A.n_chrom))
                            ? bin_path(Out<false>(nullptr, 0), c, cd).size() : 0;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K8: the per-record / per-line drop-in path in ONE launch.  The reference
// calls its per-record API once per alt allele (vcf_variant_loader.py:
// 282-311): the drop-in's parse_variant / find_bin_index must not pay a chain of
// launches, scans and host syncs per call.  One workgroup takes a small batch
// (records in host-mapped pinned memory, read over PCIe): end inference + bin
// (K2), ltree path, primary key (K7) and display-attribute JSON (K5a) per lane,
// sizes -> LDS scan -> text written straight into host-mapped output buffers.
// A stream over its capacity sets *overflow and is not written (the caller
// then takes the multi-kernel path).
// ---------------------------------------------------------------------------
struct SmallArgs {
  const uint8_t* chrom;
  const uint32_t* pos;
  const uint32_t* end_in;  // nullable: infer from the alleles
  const uint64_t* off;
  const uint32_t* rl;
  const uint32_t* al;
  const uint8_t* heap;
  const uint64_t* ext;     // nullable
  size_t heap_bytes;
  uint32_t n, max_seq_len, want, n_chrom;  // want: AVDB_SMALL_* bits
  ChromTable tab;
  uint32_t* end_out;
  uint32_t* code;
  uint8_t* status;
  uint8_t* key_state;
  uint8_t* disp_state;
  uint32_t* off_out;       // [3][n+1]: path, key, display offsets
  uint8_t* text_out[3];
  uint32_t cap[3];
  uint32_t* overflow;
};

constexpr int kSmallBlock = 256;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t* total) {
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t u = __shfl_up(x, d, kWave);
    if (lane >= d) x += u;
  }
  if (lane == kWave - 1) s_tmp[wv] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int w = 0; w < kSmallBlock / kWave; ++w) {
    if (w < wv) base += s_tmp[w];
    tot += s_tmp[w];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ __launch_bounds__(kSmallBlock) void k_small_prep(SmallArgs A) {
  __shared__ uint32_t s_tmp[kSmallBlock / kWave];
  __shared__ uint32_t s_len[AVDB_MAX_CHROM];
  if (threadIdx.x < AVDB_MAX_CHROM) s_len[threadIdx.x] = A.tab.len[threadIdx.x];
  __syncthreads();
  const Heap hp = make_heap(A.heap, A.heap_bytes);
  uint32_t run[3] = {0, 0, 0};
  bool over[3] = {false, false, false};
  for (uint32_t t0 = 0; t0 < A.n; t0 += kSmallBlock) {
    const uint32_t i = t0 + threadIdx.x;
    const bool live = i < A.n;
    uint32_t c = 0, p = 0, e = 0, cd = AVDB_BIN_NONE, r = 0, a = 0;
    uint64_t o = 0, x = 0;
    uint8_t kst = AVDB_KEY_HOST, dst = 1;
    bool lng = false;
    if (live) {
      c = A.chrom[i];
      p = A.pos[i];
      uint8_t st;
      if (A.rl) {
        o = A.off[i];
        r = A.rl[i];
        a = A.al[i];
        x = A.ext ? A.ext[i] : 0ull;
        lng = uint64_t(r) + a > A.max_seq_len;
      }
      if (A.end_in) {
        e = A.end_in[i];
      } else {
        const bool snv = r == 1u && a == 1u;
        uint32_t l;
        e = infer_end(hp, o, r, a, p, snv ? 0 : heap_u64(hp, o), snv ? 0 : heap_u64(hp, o + r), &l);
      }
      st = uint8_t(classify(c, p, e, int(A.n_chrom), s_len, &cd));
      A.end_out[i] = e;
      A.code[i] = cd;
      A.status[i] = st;
      if (A.rl) {
        const bool fits = o + r + a <= A.heap_bytes;
        const bool ascii = fits && swar_find((glb_cp)(A.heap + o), r + a,
                                             [](uint64_t w) { return w & kHiBits; }) == r + a;
        dst = fits ? (ascii ? 0 : 1) : 2;
        if (c >= 25 || (x >> 63) || !ascii) kst = AVDB_KEY_HOST;  // no label / interned id / non-ASCII
        else if (lng) kst = AVDB_KEY_NEED_DIGEST;                  // the VRS digest path (K4)
        else if (!key_allele_ok((glb_cp)(A.heap + o), r + a)) kst = AVDB_KEY_HOST;  // ':' -> ValueError
        else kst = AVDB_KEY_OK;
        A.key_state[i] = kst;
        A.disp_state[i] = dst;
      }
    }
    // three text streams: 0 ltree path, 1 primary key, 2 display-attribute JSON
    auto render = [&](int sidx, auto o_) {
      if (sidx == 0) return bin_path(o_, c, cd);
      if (sidx == 1) {
        chrom_name(o_, c);
        o_.put(':');
        o_.u32v(p);
        o_.put(':');
        o_.bytes((glb_cp)(A.heap + o), r);
        o_.put(':');
        o_.bytes((glb_cp)(A.heap + o + r), a);
        if (x) {
          o_.lit(":rs");
          o_.u64v(x);
        }
        return o_;
      }
      return display_json<true>(o_, c, p, e, (glb_cp)(A.heap + o), r, (glb_cp)(A.heap + o + r), a);
    };
#pragma unroll
    for (int sidx = 0; sidx < 3; ++sidx) {
      if (!(A.want & (1u << sidx))) continue;
      bool emit = live;
      if (sidx == 0) emit = emit && cd != AVDB_BIN_NONE && c < 25;
      if (sidx == 1) emit = emit && kst == AVDB_KEY_OK;
      if (sidx == 2) emit = emit && dst == 0;
      const uint32_t len = emit ? render(sidx, Out<false>(nullptr, 0)).size() : 0u;
      uint32_t tot;
      const uint32_t at = run[sidx] + block_excl_scan(len, s_tmp, &tot);
      uint32_t* offs = A.off_out + size_t(sidx) * (A.n + 1);
      if (live) offs[i] = at;
      if (run[sidx] + tot > A.cap[sidx]) over[sidx] = true;
      if (emit && !over[sidx]) {
        auto w = render(sidx, Out<true>(A.text_out[sidx], at));
        w.finish();
      }
      run[sidx] += tot;
    }
  }
  if (threadIdx.x == 0) {
    uint32_t ov = 0;
    for (int sidx = 0; sidx < 3; ++sidx) {
      if (!(A.want & (1u << sidx))) continue;
      A.off_out[size_t(sidx) * (A.n + 1) + A.n] = run[sidx];
      ov |= uint32_t(over[sidx]) << sidx;
    }
    *A.overflow = ov;
  }
}

}  // namespace avdb

using namespace avdb;

static size_t scan_bytes(size_t n) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, static_cast<const unsigned long long*>(nullptr),
                                         static_cast<unsigned long long*>(nullptr), n);
  return (t + 255) & ~size_t(255);
}

extern "C" int avdb_format_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = scan_bytes(n + 1) + 256;
  return AVDB_OK;
}

static int fill_args(FormatArgs* A, avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                     const avdb_vcf_line* lines, const uint64_t* rec_off, const uint32_t* end,
                     const uint32_t* bin_code, const uint8_t* status, const char* digest,
                     const uint8_t* keep, const avdb_format_opts* opts) {
  if (!ctx || !lines || !rec_off || !end || !bin_code || !status || (text_bytes && !text)) {
    avdb_set_error("avdb_vcf_format: null argument");
    return AVDB_EINVAL;
  }
  memset(A, 0, sizeof(*A));
  A->text = text;
  A->text_bytes = text_bytes;
  A->n_lines = n_lines;
  A->lines = lines;
  A->rec_off = rec_off;
  A->end = end;
  A->code = bin_code;
  A->status = status;
  A->digest = digest;
  A->keep = keep;
  A->max_seq_len = opts ? opts->max_seq_len : 50u;
  const char* alg = opts && opts->alg_id ? opts->alg_id : "";
  const size_t n = strlen(alg);
  if (n >= AVDB_MAX_ALG_ID) {
    avdb_set_error("avdb_vcf_format: algorithm id longer than %d bytes", AVDB_MAX_ALG_ID - 1);
    return AVDB_EINVAL;
  }
  memcpy(A->alg, alg, n);
  A->alg_len = uint32_t(n);
  if (opts && opts->match) {
    if (!opts->match_kind || !opts->frag_off) {
      avdb_set_error("avdb_vcf_format: match needs match_kind and frag_off");
      return AVDB_EINVAL;
    }
    A->match = opts->match;
    A->match_kind = opts->match_kind;
    A->frag = opts->frag;
    A->frag_off = opts->frag_off;
  }
  if (opts) {
    A->adsp_dup = opts->adsp_dup;
    A->adsp_col = (opts->flags & AVDB_FORMAT_ADSP) != 0;
  }
  return AVDB_OK;
}

extern "C" int avdb_vcf_format_size(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                                    const avdb_vcf_line* lines, const uint64_t* rec_off,
                                    const uint32_t* end, const uint32_t* bin_code, const uint8_t* status,
                                    const char* digest, const uint8_t* keep,
                                    const avdb_format_opts* opts, void* workspace,
                                    size_t workspace_bytes, uint64_t* copy_off, uint64_t* map_off,
                                    uint8_t* line_state, void* stream) {
  FormatArgs A;
  if (int rc = fill_args(&A, ctx, text, text_bytes, n_lines, lines, rec_off, end, bin_code, status,
                         digest, keep, opts))
    return rc;
  if (!copy_off || !map_off || !line_state) {
    avdb_set_error("avdb_vcf_format_size: null output");
    return AVDB_EINVAL;
  }
  size_t need = 0;
  avdb_format_workspace_size(n_lines, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_vcf_format_size: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* co = reinterpret_cast<unsigned long long*>(copy_off);
  auto* mo = reinterpret_cast<unsigned long long*>(map_off);
  AVDB_HIP_TRY(hipMemsetAsync(co + n_lines, 0, 8, s));
  AVDB_HIP_TRY(hipMemsetAsync(mo + n_lines, 0, 8, s));
  if (n_lines == 0) return AVDB_OK;
  A.copy_off = copy_off;
  A.map_off = map_off;
  A.line_state = line_state;
  const unsigned grid = stream_grid(n_lines, kBlock, 4096);
  hipLaunchKernelGGL(k_vcf_format<false>, dim3(grid), dim3(kBlock), 0, s, A);
  AVDB_LAUNCH_CHECK("k_vcf_format<size>");
  size_t tb = scan_bytes(n_lines + 1);
  AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(workspace, tb, co, co, n_lines + 1, s));
  AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(workspace, tb, mo, mo, n_lines + 1, s));
  return AVDB_OK;
}

extern "C" int avdb_vcf_format_write(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                                     const avdb_vcf_line* lines, const uint64_t* rec_off,
                                     const uint32_t* end, const uint32_t* bin_code, const uint8_t* status,
                                     const char* digest, const uint8_t* keep,
                                     const avdb_format_opts* opts, const uint64_t* copy_off,
                                     const uint64_t* map_off, const uint8_t* line_state,
                                     uint8_t* copy_out, uint8_t* map_out, uint64_t* counters,
                                     void* stream) {
  FormatArgs A;
  if (int rc = fill_args(&A, ctx, text, text_bytes, n_lines, lines, rec_off, end, bin_code, status,
                         digest, keep, opts))
    return rc;
  if (!copy_off || !map_off || !line_state || !copy_out || !map_out) {
    avdb_set_error("avdb_vcf_format_write: null output");
    return AVDB_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(copy_out) % 8 || reinterpret_cast<uintptr_t>(map_out) % 8) {
    avdb_set_error("avdb_vcf_format_write: outputs must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  if (n_lines == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  A.copy_off = const_cast<uint64_t*>(copy_off);
  A.map_off = const_cast<uint64_t*>(map_off);
  A.line_state = const_cast<uint8_t*>(line_state);
  A.copy_out = copy_out;
  A.map_out = map_out;
  A.counters = reinterpret_cast<unsigned long long*>(counters);
  const unsigned grid = stream_grid(n_lines, kBlock, 4096);
  hipLaunchKernelGGL(k_vcf_format<true>, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), A);
  AVDB_LAUNCH_CHECK("k_vcf_format<write>");
  return AVDB_OK;
}

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
    AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(workspace, tb, oo, oo, n + 1, s));
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
  auto* ko = reinterpret_cast<unsigned long long*>(key_off);
  auto* po = reinterpret_cast<unsigned long long*>(path_off);
  if (!key_out) {  // size pass + scans
    AVDB_HIP_TRY(hipMemsetAsync(ko + n, 0, 8, s));
    if (bin_code) AVDB_HIP_TRY(hipMemsetAsync(po + n, 0, 8, s));
    if (n == 0) return AVDB_OK;
    if (!chrom || !pos || !allele_off || !ref_len || !alt_len || !heap) {
      avdb_set_error("avdb_primary_keys: null array");
      return AVDB_EINVAL;
    }
    size_t need = 0;
    avdb_format_workspace_size(n, &need);
    if (!workspace || workspace_bytes < need) {
      avdb_set_error("avdb_primary_keys: workspace of %zu bytes required", need);
      return AVDB_ERANGE;
    }
    const unsigned grid = stream_grid(n, kBlock, 4096);
    hipLaunchKernelGGL(k_record_keys<false>, dim3(grid), dim3(kBlock), 0, s, A);
    AVDB_LAUNCH_CHECK("k_record_keys<size>");
    size_t tb = scan_bytes(n + 1);
    AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(workspace, tb, ko, ko, n + 1, s));
    if (bin_code) AVDB_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(workspace, tb, po, po, n + 1, s));
    return AVDB_OK;
  }
  if (n == 0) return AVDB_OK;
  if (!key_state || (bin_code && !path_out)) {
    avdb_set_error("avdb_primary_keys: null output");
    return AVDB_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(key_out) % 8 || (path_out && reinterpret_cast<uintptr_t>(path_out) % 8)) {
    avdb_set_error("avdb_primary_keys: outputs must be 8-byte aligned");
    return AVDB_EINVAL;
  }
  const unsigned grid = stream_grid(n, kBlock, 4096);
  hipLaunchKernelGGL(k_record_keys<true>, dim3(grid), dim3(kBlock), 0, s, A);
  AVDB_LAUNCH_CHECK("k_record_keys<write>");
  return AVDB_OK;
}

extern "C" int avdb_small_prep(avdb_ctx* ctx, const avdb_small_batch* b, void* stream) {
  if (!ctx || !b || !b->chrom || !b->pos || !b->end_out || !b->code || !b->status || !b->off_out ||
      !b->overflow || (!b->end_in && !b->ref_len)) {
    avdb_set_error("avdb_small_prep: null argument");
    return AVDB_EINVAL;
  }
  if (b->ref_len && (!b->allele_off || !b->alt_len || !b->heap || !b->key_state || !b->disp_state)) {
    avdb_set_error("avdb_small_prep: alleles need allele_off, alt_len, heap, key_state and disp_state");
    return AVDB_EINVAL;
  }
  if ((b->want & (AVDB_SMALL_KEY | AVDB_SMALL_DISPLAY)) && !b->ref_len) {
    avdb_set_error("avdb_small_prep: keys and display attributes need alleles");
    return AVDB_EINVAL;
  }
  for (int k = 0; k < 3; ++k)
    if ((b->want & (1u << k)) && !b->text_out[k]) {
      avdb_set_error("avdb_small_prep: text stream %d requested without a buffer", k);
      return AVDB_EINVAL;
    }
  if (b->n > AVDB_SMALL_MAX) {
    avdb_set_error("avdb_small_prep: at most %d records", AVDB_SMALL_MAX);
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  SmallArgs A;
  memset(&A, 0, sizeof(A));
  A.chrom = b->chrom;
  A.pos = b->pos;
  A.end_in = b->end_in;
  A.off = b->allele_off;
  A.rl = b->ref_len;
  A.al = b->alt_len;
  A.heap = b->heap;
  A.ext = b->ext_id;
  A.heap_bytes = b->heap_bytes;
  A.n = b->n;
  A.max_seq_len = b->max_seq_len;
  A.want = b->want;
  A.n_chrom = uint32_t(ctx->tab.n);
  A.tab = ctx->tab;
  A.end_out = b->end_out;
  A.code = b->code;
  A.status = b->status;
  A.key_state = b->key_state;
  A.disp_state = b->disp_state;
  A.off_out = b->off_out;
  A.overflow = b->overflow;
  for (int k = 0; k < 3; ++k) {
    A.text_out[k] = b->text_out[k];
    A.cap[k] = b->text_cap[k];
  }
  hipLaunchKernelGGL(k_small_prep, dim3(1), dim3(kSmallBlock), 0, static_cast<hipStream_t>(stream), A);
  AVDB_LAUNCH_CHECK("k_small_prep");
  return AVDB_OK;
}
