// K0's per-line VCF parse (VcfEntryParser, Util/lib/python/parsers/vcf_parser.py:
// 76-169): one line's fields, contig code, POS, refSNP key, ALT and record counts.
// Shared by the tokenizer kernel (avdb_vcf.hip, lines staged in LDS) and the
// library's per-line host entry (avdb_line_host.hip): one definition, compiled
// for both sides.
#pragma once

#include "avdb_text.hpp"

#include <vector>

namespace avdb {

// contig code of a CHROM field (vcf_parser.py:133-150 + bin_index.py:64): plain
// digits go through int(); 'MT' -> 'M'; every 'chr' removed in one left-to-right
// pass (str.replace); then chr1..22, X, Y, M.  *host set for non-alphanumeric bytes.
template <class CP>
AVDB_HD uint8_t chrom_code_of(CP p, uint32_t n, bool* host) {
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

// ---- chromosome map (ChromosomeMap.get, chromosome_map_parser.py:84-91, applied
// by VcfEntryParser.update_chromosome, vcf_parser.py:117-124): CHROM bytes ->
// contig code through an open-addressing table built by avdb_chrom_map_create.
// Slot = (FNV-1a hash high 40 bits << 24) | (key index + 1); 0 = empty.  code[k]
// is the contig code of the mapped chromosome, or 0xFF when the line must be
// rendered by the host (a key Python would coerce to a number never matches a
// CHROM string: the reference's KeyError).  A CHROM not in the map is host too.
struct ChromMapView {
  const uint64_t* slot;
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint8_t* code;
  uint32_t mask;  // slots - 1; 0 (with slot == nullptr): no map
};

AVDB_HD uint64_t fnv1a(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return h;
}

template <class CP>
AVDB_HD uint64_t fnv1a_cp(CP p, uint32_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return h;
}

// contig code of the mapped CHROM, or 255 with *host set
template <class CP>
AVDB_HD uint8_t chrom_map_code(const ChromMapView& cm, CP p, uint32_t n, bool* host) {
  const uint64_t h = fnv1a_cp(p, n);
  const uint64_t tag = h >> 24;
  for (uint32_t q = uint32_t(h) & cm.mask, k = 0; k <= cm.mask; q = (q + 1) & cm.mask, ++k) {
    const uint64_t v = cm.slot[q];
    if (!v) break;
    if ((v >> 24) != tag) continue;
    const uint32_t idx = uint32_t(v & 0xFFFFFFu) - 1;
    const uint32_t k0 = cm.key_off[idx], kn = cm.key_off[idx + 1] - k0;
    if (kn != n) continue;
    bool eq = true;
    for (uint32_t i = 0; i < n && eq; ++i) eq = cm.keys[k0 + i] == p[i];
    if (!eq) continue;
    const uint8_t c = cm.code[idx];
    *host = c == 0xFF;
    return c;
  }
  *host = true;
  return 255;
}

// canonical refSNP number of "rs<N>" bytes (N without leading zeros, < 10^18), else 0
template <class CP>
AVDB_HD uint64_t rs_number(CP p, uint32_t n) {
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
AVDB_HD void line16(const WordAt& word_at, uint32_t mis, uint32_t len, uint32_t f,
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
AVDB_HD uint32_t digits8_value(uint64_t x, uint32_t n) {
  if (n == 0) return 0;
  uint64_t v = (x ^ 0x3030303030303030ull) << (8 * (8 - n));  // leading zero digits below
  v = (v * 10 + (v >> 8)) & 0x00FF00FF00FF00FFull;
  v = (v * 100 + (v >> 16)) & 0x0000FFFF0000FFFFull;
  v = (v * 10000 + (v >> 32)) & 0xFFFFFFFFull;
  return uint32_t(v);
}

// a decimal field of n <= 16 bytes in (x0, x1): *ok = all digits; value (64-bit)
AVDB_HD uint64_t decimal16(uint64_t x0, uint64_t x1, uint32_t n, bool* ok) {
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

// the tab-separated fields of a line of len bytes (first 8 starts; INFO ends at
// the 8th tab or the end): L.field[1..7] / L.field_end8 for the tabs present
// (the caller preset the rest), returns the field count.  SWAR over the line's
// aligned words (word_at/mis).
template <class WordAt>
AVDB_HD uint32_t fields_swar(const WordAt& word_at, uint32_t mis, uint32_t len, avdb_vcf_line& L) {
  uint32_t nf = 1;
  const uint32_t k1 = (len + mis + 7) >> 3;
  for (uint32_t k = 0; k < k1; ++k) {
    uint64_t m = zero_bytes_mask(word_at(k) ^ kTab) & kHiBits;
    if (k == 0) m &= ~low_bytes_mask(mis);
    const uint32_t hi = len + mis - 8 * k;
    if (hi < 8) m &= low_bytes_mask(hi);
    if (nf > 8) {  // past INFO: only the count matters
      nf += uint32_t(__builtin_popcountll(m));
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
  return nf;
}

// one line: s points at its first byte (LDS or global), len = bytes up to its
// newline; word_at/mis give the same bytes as aligned 8-byte words (SWAR scans);
// find_fields(len, L) fills the field table and returns the field count
// (fields_swar, or the tab bitmap of a staged window: avdb_vcf.hip).
// kDeferInfo: a line whose refSNP must come from INFO gets L.pad[0] =
// kInfoPending instead of the INFO scan (the window parse gathers those lines of a
// round and scans their INFO fields with the whole workgroup: avdb_vcf.hip)
constexpr uint8_t kInfoPending = 1;
template <bool kDeferInfo = false, class CP, class WordAt, class FindFields>
AVDB_HD void parse_line_with(const FindFields& find_fields, CP s, const WordAt& word_at, uint32_t mis,
                             uint32_t len, avdb_vcf_line& L, uint64_t& recs, uint64_t& hbytes,
                             const ChromMapView& cm, uint32_t min_fields) {
    while (len && is_ws(s[len - 1])) --len;  // str.rstrip()
    L.len = len;
    L.flags = 0;
    L.pos = 0;
    L.ext_id = 0;
    L.n_alt = 0;
    L.n_rec = 0;
    L.chrom = 255;
    L.pad[0] = L.pad[1] = L.pad[2] = 0;
    L.field[0] = 0;
    for (int k = 1; k < 8; ++k) L.field[k] = len + 1;
    L.field_end8 = len;
    if (len && s[0] == '#') L.flags |= AVDB_VCF_COMMENT;
    if (!len) L.flags |= AVDB_VCF_EMPTY;
    const uint32_t nf = find_fields(len, L);
    L.n_fields = nf;
    recs = 0;
    hbytes = 0;
    if (!(L.flags & (AVDB_VCF_COMMENT | AVDB_VCF_EMPTY))) {
      // fewer values than header fields: the reference's IndexError (vcf_parser.py:90-112)
      if (nf < 8 || nf < min_fields) L.flags |= AVDB_VCF_FEW_FIELDS;
      const uint32_t nfields = nf < 8 ? nf : 8;
      auto fend = [&](int k) -> uint32_t {  // end of field k (exclusive)
        return (k + 1 < int(nfields)) ? L.field[k + 1] - 1 : (k == 7 ? L.field_end8 : len);
      };
      if (!(L.flags & AVDB_VCF_FEW_FIELDS)) {
        // CHROM
        bool host = false;
        L.chrom = cm.slot ? chrom_map_code(cm, s, fend(0), &host) : chrom_code_of(s, fend(0), &host);
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
        // ID (its first 16 bytes in two registers: an "rs<digits>" or '.' ID, the
        // dbSNP shapes, needs no other read)
        const CP id = s + L.field[2];
        const uint32_t idn = fend(2) - L.field[2];
        uint64_t i0, i1;
        line16(word_at, mis, len, L.field[2], &i0, &i1);
        const uint32_t c0 = idn > 0 ? uint32_t(i0 & 0xFF) : 0u, c1 = idn > 1 ? uint32_t((i0 >> 8) & 0xFF) : 0u;
        const bool rs_head = idn >= 2 && c0 == 'r' && c1 == 's';
        const bool id_dot = idn == 1 && c0 == '.';
        bool has_rs = rs_head;
        if (!rs_head && !id_dot) {
          // 16 bytes at a time: digits / number-like bytes / an "rs" pair ("rs..."
          // holds a letter and '.' no digit, so neither can be number-like)
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
        if (id_dot || rs_head) L.flags |= AVDB_VCF_ID_METASEQ;
        if (has_rs) {
          L.flags |= AVDB_VCF_ID_RS;
          if (idn >= 3 && idn <= 18 && rs_head && ((i0 >> 16) & 0xFF) != '0') {
            uint64_t y0, y1;  // "rs" + up to 16 digits, SWAR
            if (idn <= 16) {  // bytes 2.. of the registers already read
              y0 = (i0 >> 16) | (i1 << 48);
              y1 = i1 >> 16;
            } else {
              line16(word_at, mis, len, L.field[2] + 2, &y0, &y1);
            }
            bool ok;
            const uint64_t v = decimal16(y0, y1, idn - 2, &ok);
            L.ext_id = ok ? v : 0ull;
          } else {
            L.ext_id = rs_number(id, idn);
          }
          if (!L.ext_id) L.flags |= AVDB_VCF_EXT_HOST;
        } else if (kDeferInfo) {
          L.pad[0] = kInfoPending;
        } else {
          // INFO: the last entry whose key is exactly "RS" (dict(...) keeps the last).
          // One pass over the INFO's words with no data-dependent branch: an entry
          // "RS" / "RS=..." is an 'R' at an entry start (the INFO start or after a
          // ';') followed by 'S', then '=', ';' or the INFO end — exact, as INFO
          // holds no tab.  The last such entry decides: "RS" bare, "RS=<v>" a value.
          const uint32_t f7 = L.field[7], e7 = fend(7);
          int64_t rs_at = -1;  // line offset of the last entry's 'R'
          bool rs_val = false;  // ... followed by '='
          if (e7 >= f7 + 2) {
            const uint32_t kend = (len + mis + 7) >> 3;
            const uint32_t ka = (f7 + mis) >> 3, kb = (e7 + mis + 7) >> 3;
            uint64_t x = word_at(ka), semi_c = 0;  // semi_c bit 7: the byte before word k is ';'
            for (uint32_t k = ka; k < kb; ++k) {
              const uint64_t nx = k + 1 < kend ? word_at(k + 1) : 0ull;
              const int32_t base = int32_t(8 * k) - int32_t(mis);  // line offset of the word's byte 0
              const uint64_t semi = bytes_eq_mask(x, ';');
              uint64_t at = (semi << 8) | semi_c;
              const int32_t js = int32_t(f7) - base, jz = int32_t(e7) - 1 - base;  // 'R' at [js, jz)
              if (js >= 0 && js < 8) at |= uint64_t(0x80) << (8 * js);
              uint64_t range = kHiBits;
              if (js > 0) range &= ~low_bytes_mask(uint32_t(js));
              if (jz < 8) range &= jz > 0 ? low_bytes_mask(uint32_t(jz)) : 0ull;
              const uint64_t v1 = (x >> 8) | (nx << 56), v2 = (x >> 16) | (nx << 48);
              const int32_t je = int32_t(e7) - 2 - base;  // 'R' two bytes before the INFO end
              const uint64_t eq = bytes_eq_mask(v2, '=');
              uint64_t tail = eq | bytes_eq_mask(v2, ';');
              if (je >= 0 && je < 8) tail |= uint64_t(0x80) << (8 * je);
              const uint64_t cand = bytes_eq_mask(x, 'R') & bytes_eq_mask(v1, 'S') & at & tail & range;
              if (cand) {
                const uint32_t j = (63u - uint32_t(__builtin_clzll(cand))) >> 3;
                rs_at = base + int32_t(j);
                rs_val = (eq >> (8 * j)) & 0x80;
              }
              semi_c = semi >> 56;
              x = nx;
            }
          }
          if (rs_at >= 0) {
            L.flags |= AVDB_VCF_INFO_RS;
            uint64_t v = 0;
            bool ok = false;
            if (rs_val) {
              // the value [rs_at + 3, next ';' or the INFO end): all digits, 1..18 of them
              const uint32_t vs = uint32_t(rs_at) + 3;
              uint64_t y0, y1;
              line16(word_at, mis, len, vs, &y0, &y1);
              const uint64_t nd0 = nondigit_mask(y0), nd1 = nondigit_mask(y1);
              const uint32_t nd = nd0 ? uint32_t(__builtin_ctzll(nd0)) >> 3
                                      : (nd1 ? 8u + (uint32_t(__builtin_ctzll(nd1)) >> 3) : 16u);
              const uint32_t vmax = e7 - vs;  // bytes to the INFO end
              if (nd < 16 || vmax <= 16) {
                const uint32_t n = nd < vmax ? nd : vmax;  // leading digits inside INFO
                // the value ends at the INFO end or at a ';' right after its digits
                const bool term = n == vmax || (n < 16 && (((n < 8 ? y0 >> (8 * n) : y1 >> (8 * (n - 8))) & 0xFF) == ';'));
                if (term && n >= 1) v = decimal16(y0, y1, n, &ok);
              } else {  // 16 digits and more: the byte loop (<= 18 digits)
                const CP inf = s + vs;
                uint32_t n = 0;
                while (n < vmax && inf[n] != ';') ++n;
                ok = n <= 18;
                for (uint32_t q = 0; ok && q < n; ++q) {
                  ok = is_digit(inf[q]);
                  v = v * 10 + (inf[q] - '0');
                }
              }
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
          commas += uint32_t(__builtin_popcountll(bytes_eq_mask(y0, ',') & m0) + __builtin_popcountll(bytes_eq_mask(y1, ',') & m1));
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

template <class CP, class WordAt>
AVDB_HD void parse_line(CP s, const WordAt& word_at, uint32_t mis, uint32_t len, avdb_vcf_line& L, uint64_t& recs,
                        uint64_t& hbytes, const ChromMapView& cm = ChromMapView{}, uint32_t min_fields = 8) {
  parse_line_with([&word_at, mis](uint32_t n, avdb_vcf_line& l) { return fields_swar(word_at, mis, n, l); }, s, word_at,
                  mis, len, L, recs, hbytes, cm, min_fields);
}

}  // namespace avdb

// the chromosome map object of the C ABI: the table on the host (K5h, the per-line
// host entry) and on the device (K0's parse kernel)
struct avdb_chrom_map {
  int device;
  std::vector<uint64_t> slot;
  std::vector<uint8_t> keys;
  std::vector<uint32_t> key_off;
  std::vector<uint8_t> code;
  void* d_mem;  // one device allocation: slot | key_off | code | keys
  avdb::ChromMapView host_view() const {
    return avdb::ChromMapView{slot.data(), keys.data(), key_off.data(), code.data(), uint32_t(slot.size() - 1)};
  }
  avdb::ChromMapView dev;
};
