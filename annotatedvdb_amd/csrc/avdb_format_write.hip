// K5b WRITE pass host entry (the kernel template: avdb_k5.hpp).
#include "avdb_k5.hpp"

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
  const unsigned grid = stream_grid(n_lines, kBlock, AVDB_K5_WRITE_GRID);
  // (the write pass split into a COPY launch and a .mapping launch, each sink-free
  // of the other stream, measured slower: 5.25 vs 4.41 ms, profiles/k5_ab/r05_split_write_ab.log)
  hipLaunchKernelGGL(k_vcf_format<true>, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream), A);
  AVDB_LAUNCH_CHECK("k_vcf_format<write>");
  return AVDB_OK;
}
