// K5b kernel template (SIZE and WRITE passes are compiled in separate translation
// units, avdb_format.hip and avdb_format_write.hip, so the two build in parallel).
#pragma once

#include "avdb_fmt.hpp"

#include <string.h>



namespace avdb {

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
AVDB_HD bool plain_allele(CP s, uint32_t n) {
  return swar_find(s, n, [](uint64_t x) {
           const uint64_t lt20 = ~((x & 0x7F7F7F7F7F7F7F7Full) + 0x6060606060606060ull) & kHiBits;
           return (x & kHiBits) | lt20 | bytes_eq_mask(x, 0x7F) | bytes_eq_mask(x, '"') |
                  bytes_eq_mask(x, '\\') | bytes_eq_mask(x, '\'') | bytes_eq_mask(x, ':');
         }) == n;
}

template <class CP>
AVDB_HD bool bytes_eq(CP a, CP b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// next separator at or after i in [i, e), or e
template <class CP>
AVDB_HD uint32_t find_byte(CP s, uint32_t i, uint32_t e, uint8_t c) {
  if (i >= e) return i;
  return i + swar_find(s + i, e - i, [c](uint64_t x) { return bytes_eq_mask(x, c); });
}

// FREQ value [v0, v1) of the line: is it one the GPU renders?  Every population
// needs a ':' (pop.split(':')[1]), a JSON-plain name, and names must be unique
// (the reference's dict comprehension keeps the last value at the first
// position).
template <class CP>
AVDB_HD bool freq_plain(CP s, uint32_t v0, uint32_t v1) {
  uint32_t np = 0;
  for (uint32_t p0 = v0; p0 <= v1; ++np) {
    const uint32_t p1 = find_byte(s, p0, v1, '|');
    const uint32_t c1 = find_byte(s, p0, p1, ':');
    if (c1 == p1 || np >= kMaxPops) return false;
    // population name: printable ASCII without '"' or '\\' (SWAR)
    if (swar_find(s + p0, c1 - p0, [](uint64_t x) {
          const uint64_t lt20 = ~((x & 0x7F7F7F7F7F7F7F7Full) + 0x6060606060606060ull) & kHiBits;
          return (x & kHiBits) | lt20 | bytes_eq_mask(x, 0x7F) | bytes_eq_mask(x, '"') | bytes_eq_mask(x, '\\');
        }) != c1 - p0)
      return false;
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
AVDB_HD O freq_json(O o, CP s, uint32_t v0, uint32_t v1, uint32_t k) {
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

// oc / om: the COPY and .mapping sinks
template <bool WRITE, class OC, class OM, class CP>
AVDB_HD uint8_t format_line(const FormatArgs& A, const avdb_vcf_line& L, CP s, size_t li,
                               OC& oc, OM& om, uint32_t* n_rows, uint32_t* n_skip,
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
  // WRITE: the first record's status / bin / keep / end are loaded before the
  // ALT loop (nearly every line has one ALT), not inside it behind the LDS scans
  const uint64_t r0 = r;
  uint32_t st0 = 0, code0 = 0, end0 = 0;
  bool keep0 = true;
  if constexpr (WRITE) {
    st0 = A.status[r0];
    code0 = A.code[r0];
    end0 = A.end[r0];
    keep0 = !A.keep || A.keep[r0];
  }
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
    const bool first = WRITE && r == r0;
    const uint32_t st = first ? st0 : A.status[r];
    if (st == AVDB_STATUS_UNKNOWN_CHROM || st == AVDB_STATUS_OUT_OF_RANGE) return kLineHost;
    const uint32_t code = first ? code0 : A.code[r];
    const bool keep = first ? keep0 : (!A.keep || A.keep[r]);
    // altIndex = altAlleles.index(allele) + 1: the first equal ALT
    uint32_t k = ai + 1;
    for (uint32_t b0 = alt0, bi = 0; bi < ai; ++bi) {
      const uint32_t b1 = find_byte(s, b0, alt1, ',');
      if (b1 - b0 == al && bytes_eq(s + b0, alt, al)) { k = bi + 1; break; }
      b0 = b1 + 1;
    }
    // primary key (primary_key_generator.py:106-122)
    auto pk = [&](auto& o) {
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
      oc.append(L.n_alt > 1 ? 0x65757254ull : 0x4C4C554Eull, 4);  // "True" / "NULL"
      oc.put('#');
      oc = display_json<false>(oc, c, L.pos, first ? end0 : A.end[r], ref, rl, alt, al, posd);
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
        if (freq_json(typename OC::Counter(nullptr, 0), s, uint32_t(fq0), uint32_t(fq1), k).bad) return kLineHost;
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

// Lines of one shape in the same wave.  A wave runs the union of its lanes'
// paths: one two-ALT line makes all 64 lanes pay a second ALT iteration, one
// indel the non-SNV display branches, one host line nothing.  The tile's lines
// are ranked by shape (LDS counting sort; order inside a shape is free: every
// line writes at its own offsets) and lane t takes the t-th.
constexpr uint32_t kShapes = 6;

template <bool WRITE>
__device__ __forceinline__ uint32_t tile_order(const FormatArgs& A, size_t base, size_t last, uint32_t* s_key) {
  const uint32_t t = threadIdx.x;
  uint32_t* cnt = s_key + kBlock;
  if (t < kShapes) cnt[t] = 0;
  __syncthreads();
  const size_t lj = base + t;
  uint32_t key = kShapes - 1;  // past the end, or a line with nothing to render
  if (lj < last) {
    const avdb_vcf_line& L = A.lines[lj];
    const bool live = WRITE ? A.line_state[lj] == kLineGpu
                            : !(L.flags & (AVDB_VCF_COMMENT | kHostFlags)) && L.chrom < 25;
    if (live) {
      const uint32_t rl = L.field[4] - 1 - L.field[3], alts = L.field[5] - 1 - L.field[4];
      const bool snv = rl == 1 && alts == 2 * L.n_alt - 1;  // every ALT one base
      const uint32_t na = L.n_alt < 3 ? L.n_alt : 3;
      key = (na - 1) * 2 + (snv ? 0 : 1);
      if (key > kShapes - 2) key = kShapes - 2;
    }
  }
  const uint32_t rank = atomicAdd(&cnt[key], 1u);
  __syncthreads();
  uint32_t at = rank;
  for (uint32_t k = 0; k < key; ++k) at += cnt[k];
  s_key[at] = t;
  __syncthreads();
  return s_key[t];
}

// K5 workgroups over 256-line tiles (A/B on 8.4 M lines, load workload): the size
// pass with one workgroup per tile 1.73 -> 1.56 ms (against a 4,096-workgroup
// grid-stride), the write pass best at 8,192 (4.48 -> 4.39 ms; one per tile 4.43)
#ifndef AVDB_K5_SIZE_GRID
#define AVDB_K5_SIZE_GRID (1u << 30)
#endif
#ifndef AVDB_K5_WRITE_GRID
#define AVDB_K5_WRITE_GRID 8192
#endif
template <bool WRITE>
__global__ __launch_bounds__(kBlock, kFormatWaves) void k_vcf_format(FormatArgs A) {
  __shared__ u32x4 s_text[kStage / 16];
  __shared__ uint32_t s_key[kBlock + 8];
  const Heap h = make_heap(A.text, A.text_bytes);
  uint32_t rows = 0, skip = 0, dups = 0, hosts = 0, upds = 0;
  for (size_t base = size_t(blockIdx.x) * kBlock; base < A.n_lines; base += size_t(gridDim.x) * kBlock) {
    const size_t last = base + kBlock < A.n_lines ? base + kBlock : A.n_lines;
    const avdb_vcf_line& Z = A.lines[last - 1];
    // (the tile's text one load per trip: staging it with every load in flight, as
    // K0 does, spills this pass's registers — write 4.40 -> 4.77 ms,
    // profiles/k5_ab/r05_stage_batch_ab.log)
    const Window w = stage_window<kBlock, kStage, false>(h, A.lines[base].start, Z.start + Z.len, s_text);
    const size_t li = base + tile_order<WRITE>(A, base, last, s_key);
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

}  // namespace avdb

using namespace avdb;

static inline int fill_args(FormatArgs* A, avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                     const avdb_vcf_line* lines, const uint64_t* rec_off, const uint32_t* end,
                     const uint32_t* bin_code, const uint8_t* status, const char* digest,
                     const uint8_t* keep, const avdb_format_opts* opts) {
  if (!ctx || !lines || !rec_off || !end || !bin_code || !status || (text_bytes && !text)) {
    avdb_set_error("avdb_vcf_format: null argument");
    return AVDB_EINVAL;
  }
  if (opts && opts->struct_size != sizeof(avdb_format_opts)) {
    avdb_set_error("avdb_vcf_format: avdb_format_opts.struct_size %u, this library expects %zu (ABI %d)",
                   opts->struct_size, sizeof(avdb_format_opts), AVDB_ABI_VERSION);
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
