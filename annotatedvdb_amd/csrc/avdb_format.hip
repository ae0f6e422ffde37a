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
//   SIZE pass (bytes per line) -> exclusive scans (avdb_scan.hpp) -> WRITE pass, both the
//   same templated code.  One lane per line, 256 consecutive lines per workgroup
//   with their text staged in LDS (as K0); each lane writes its own contiguous
//   span of both outputs (sink and alternatives measured: see Out below).  A
//   line the GPU does not render byte-exact (non-ASCII text,
//   allele bytes that need escaping, an unmappable record (TypeError), a key the
//   reference cannot build (':' in an allele), malformed or non-canonical FREQ
//   numbers, K0 host-resolved fields) is marked HOST and gets zero bytes; the
//   host renders it between its neighbours.
// (K5a display attributes and K7 keys: avdb_keys.hip; K8: avdb_small.hip; the
// shared sink and renderers: avdb_fmt.hpp.)
#include "avdb_k5.hpp"

#include "avdb_scan.hpp"


static size_t scan_bytes(size_t n) { return (avdb::scan::workspace_bytes(n, 2) + 255) & ~size_t(255); }

extern "C" int avdb_format_workspace_size(size_t n, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  const size_t a = scan_bytes(n + 1), b = avdb::key_size_workspace(n);  // (K7's u16 sizes + scan)
  *bytes = (a > b ? a : b) + 256;
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
  const unsigned grid = stream_grid(n_lines, kBlock, AVDB_K5_SIZE_GRID);
  hipLaunchKernelGGL(k_vcf_format<false>, dim3(grid), dim3(kBlock), 0, s, A);
  AVDB_LAUNCH_CHECK("k_vcf_format<size>");
  size_t tb = scan_bytes(n_lines + 1);
  if (int e = avdb::scan::exclusive_u64_pair(copy_off, copy_off, map_off, map_off, n_lines + 1, workspace, tb, s))
    return e;
  return AVDB_OK;
}
