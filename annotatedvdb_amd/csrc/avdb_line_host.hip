// K5h avdb_vcf_line_host: ONE VCF line -> its COPY rows and .mapping line, in the
// library's host code.
//
// The reference's loader takes one line per call (Load/bin/load_vcf_file.py:112 ->
// VCFVariantLoader.parse_variant, vcf_variant_loader.py:351-391).  A GPU launch
// and a stream sync per line would cost more than the reference's whole call, so
// this entry runs the kernels' own per-line code on the host: K0's parse_line
// (avdb_vcfline.hpp), K2's infer_end + classify (avdb_internal.hpp) and K5's
// format_line (avdb_k5.hpp, SIZE pass for the GPU/host decision, then WRITE) —
// the same AVDB_HD definitions the tokenizer / formatter kernels compile, into a
// host sink.  Lines K5 would leave to the host (AVDB_LINE_HOST) are left to the
// caller here too.
#include "avdb_k5.hpp"
#include "avdb_vcfline.hpp"

#include <string.h>

#include <vector>

using namespace avdb;

namespace {

constexpr uint32_t kMaxLineRecords = 4096;

struct LineScratch {
  std::vector<uint64_t> text;   // the line, 16 bytes in, zero padded (aligned word reads)
  std::vector<uint8_t> heap;    // one record's REF + ALT (infer_end reads them as one heap)
  std::vector<uint32_t> end, code;
  std::vector<uint8_t> status;
};

thread_local LineScratch g_scratch;

}  // namespace

extern "C" int avdb_vcf_line_host(const avdb_ctx* ctx, const char* line, size_t len, const avdb_format_opts* opts,
                                  const avdb_vcf_opts* vopts, char* copy_out, size_t copy_cap, char* map_out,
                                  size_t map_cap, avdb_line_result* res) {
  if (!ctx || (!line && len) || !opts || !res) {
    avdb_set_error("avdb_vcf_line_host: null argument");
    return AVDB_EINVAL;
  }
  if (opts->struct_size != sizeof(avdb_format_opts)) {
    avdb_set_error("avdb_vcf_line_host: avdb_format_opts.struct_size %u, this library expects %zu (ABI %d)",
                   opts->struct_size, sizeof(avdb_format_opts), AVDB_ABI_VERSION);
    return AVDB_EINVAL;
  }
  if (vopts && vopts->struct_size != sizeof(avdb_vcf_opts)) {
    avdb_set_error("avdb_vcf_line_host: avdb_vcf_opts.struct_size %u, this library expects %zu",
                   vopts->struct_size, sizeof(avdb_vcf_opts));
    return AVDB_EINVAL;
  }
  if (opts->match || opts->adsp_dup) {
    avdb_set_error("avdb_vcf_line_host: --skipExisting / ADSP key matches are batch features (avdb_vcf_format_*)");
    return AVDB_EINVAL;
  }
  if (len > 0xFFFFFFF0u) {
    avdb_set_error("avdb_vcf_line_host: line too long");
    return AVDB_EINVAL;
  }
  memset(res, 0, sizeof(*res));
  LineScratch& S = g_scratch;
  const size_t words = (16 + len + 16 + 7) / 8;
  if (S.text.size() < words) S.text.resize(words);
  memset(S.text.data(), 0, words * 8);
  uint8_t* s = reinterpret_cast<uint8_t*>(S.text.data()) + 16;
  if (len) memcpy(s, line, len);
  const uint64_t* lw = reinterpret_cast<const uint64_t*>(s);
  avdb_vcf_line L;
  memset(&L, 0, sizeof(L));
  uint64_t recs = 0, hbytes = 0;
  const ChromMapView cm = vopts && vopts->chrom_map ? vopts->chrom_map->host_view() : ChromMapView{};
  parse_line(static_cast<const uint8_t*>(s), [lw](uint32_t k) { return lw[k]; }, 0u, uint32_t(len), L, recs, hbytes,
             cm, vopts ? vopts->min_fields : 0u);
  res->flags = L.flags;
  if (L.flags & AVDB_VCF_COMMENT) {
    res->state = AVDB_LINE_SKIP;
    return AVDB_OK;
  }
  if ((L.flags & kHostFlags) || L.chrom >= 25 || L.chrom >= uint32_t(ctx->tab.n) || recs > kMaxLineRecords) {
    res->state = AVDB_LINE_HOST;
    return AVDB_OK;
  }
  // K2 per record (ALT != '.', as K0's emit_line cuts them): end + bin
  const uint32_t n = uint32_t(recs);
  S.end.resize(n + 1);
  S.code.resize(n + 1);
  S.status.resize(n + 1);
  const uint32_t nfields = L.n_fields < 8 ? L.n_fields : 8;
  const uint32_t ref0 = L.field[3], rl = L.field[4] - 1 - ref0;
  const uint32_t alt0 = L.field[4], aend = 5 < nfields ? L.field[5] - 1 : L.len;
  uint32_t r = 0;
  for (uint32_t a0 = alt0; a0 <= aend && r < n;) {
    uint32_t a1 = a0;
    while (a1 < aend && s[a1] != ',') ++a1;
    const uint32_t al = a1 - a0;
    if (!(al == 1 && s[a0] == '.')) {
      if (S.heap.size() < size_t(rl) + al + 8) S.heap.resize(size_t(rl) + al + 8);
      memcpy(S.heap.data(), s + ref0, rl);
      memcpy(S.heap.data() + rl, s + a0, al);
      const Heap hp = make_heap(S.heap.data(), size_t(rl) + al);
      const bool snv = rl == 1u && al == 1u;
      uint32_t lcp;
      const uint32_t e = infer_end(hp, 0, rl, al, L.pos, snv ? 0 : heap_u64(hp, 0), snv ? 0 : heap_u64(hp, rl), &lcp);
      uint32_t cd;
      S.status[r] = uint8_t(classify(L.chrom, L.pos, e, ctx->tab.n, ctx->tab.len, &cd));
      S.end[r] = e;
      S.code[r] = cd;
      ++r;
    }
    a0 = a1 + 1;
  }
  if (r != n) {  // (parse_line and this cut agree; anything else is the caller's)
    res->state = AVDB_LINE_HOST;
    return AVDB_OK;
  }
  FormatArgs A;
  memset(&A, 0, sizeof(A));
  const uint64_t rec_off[2] = {0, n};
  A.text = s;
  A.text_bytes = len;
  A.n_lines = 1;
  A.rec_off = rec_off;
  A.end = S.end.data();
  A.code = S.code.data();
  A.status = S.status.data();
  A.max_seq_len = opts->max_seq_len;
  const char* alg = opts->alg_id ? opts->alg_id : "";
  const size_t alg_len = strlen(alg);
  if (alg_len >= AVDB_MAX_ALG_ID) {
    avdb_set_error("avdb_vcf_line_host: algorithm id longer than %d bytes", AVDB_MAX_ALG_ID - 1);
    return AVDB_EINVAL;
  }
  memcpy(A.alg, alg, alg_len);
  A.alg_len = uint32_t(alg_len);
  A.adsp_col = (opts->flags & AVDB_FORMAT_ADSP) != 0;
  // SIZE pass: every GPU/host decision, and the byte counts
  uint32_t rows = 0, skip = 0, dup = 0, upd = 0;
  HostOut oc(nullptr, 0), om(nullptr, 0);
  const uint8_t st = format_line<false>(A, L, static_cast<const uint8_t*>(s), 0, oc, om, &rows, &skip, &dup, &upd);
  res->n_rec = n;
  if (st != kLineGpu) {
    res->state = st == kLineSkip ? AVDB_LINE_SKIP : AVDB_LINE_HOST;
    return AVDB_OK;
  }
  res->state = AVDB_LINE_GPU;
  res->copy_bytes = oc.size();
  res->map_bytes = om.size();
  res->n_rows = rows;
  res->n_skip = skip;
  res->n_dup = dup;
  res->n_upd = upd;
  if (oc.size() > copy_cap || om.size() > map_cap || (oc.size() && !copy_out) || (om.size() && !map_out)) {
    avdb_set_error("avdb_vcf_line_host: output needs %u + %u bytes", oc.size(), om.size());
    return AVDB_ERANGE;
  }
  // WRITE pass
  rows = skip = dup = upd = 0;
  HostOut wc(reinterpret_cast<uint8_t*>(copy_out), 0), wm(reinterpret_cast<uint8_t*>(map_out), 0);
  format_line<true>(A, L, static_cast<const uint8_t*>(s), 0, wc, wm, &rows, &skip, &dup, &upd);
  if (wc.size() != oc.size() || wm.size() != om.size()) {
    avdb_set_error("avdb_vcf_line_host: size and write passes disagree (%u/%u, %u/%u)", wc.size(), oc.size(),
                   wm.size(), om.size());
    return AVDB_EINVAL;
  }
  return AVDB_OK;
}
