// K9 — genome-piece sharding of VCF text on the device (gfx950).
//
// The reference's only parallelism is one OS process per chromosome file
// (Load/bin/load_vcf_file.py:307-313).  Here one large file is split over the
// GPUs of a node by the length-balanced piece plan (annotatedvdb_amd/shard.py:
// contigs cut at 64 Mb = L1 bin boundaries, pieces assigned by LPT): a line
// belongs to the rank owning the piece that holds its POS.  Bins and keys are
// functions of (chrom, pos, alleles) alone and equal keys share (chrom, pos), so
// no line ever needs another rank's data.
//   avdb_vcf_select_lines  one lane per K0 line: owner rank from the piece table
//                          (per-contig piece bases and piece -> rank, staged in
//                          LDS), this rank's bytes per line, hipCUB scan
//   avdb_vcf_select_copy   the selected lines (+ '\n') gathered into one text
#include "avdb_internal.hpp"

#include "avdb_scan.hpp"
#include <string.h>

namespace avdb {

constexpr int kMaxPieces = 1024;

struct ShardArgs {
  uint32_t piece_base[AVDB_MAX_CHROM];  // first piece of each contig
  uint32_t piece_count[AVDB_MAX_CHROM];
  uint8_t piece_rank[kMaxPieces];
  uint32_t cut;                         // piece width (bp)
  int32_t n_chrom;
  int32_t rank;
};

// lines the GPU cannot place (host-resolved contig or position, empty or short
// lines) go to rank 0, so every data line is processed by exactly one rank
constexpr uint32_t kUnplaced = AVDB_VCF_BAD_POS | AVDB_VCF_CHROM_HOST | AVDB_VCF_EMPTY | AVDB_VCF_FEW_FIELDS;

__global__ __launch_bounds__(kBlock) void k_vcf_select(const avdb_vcf_line* __restrict__ lines, size_t n_lines,
                                                       ShardArgs S, unsigned long long* __restrict__ sel) {
  __shared__ uint32_t s_base[AVDB_MAX_CHROM], s_cnt[AVDB_MAX_CHROM];
  __shared__ uint8_t s_rank[kMaxPieces];
  for (int t = threadIdx.x; t < kMaxPieces; t += blockDim.x) s_rank[t] = S.piece_rank[t];
  if (threadIdx.x < AVDB_MAX_CHROM) {
    s_base[threadIdx.x] = S.piece_base[threadIdx.x];
    s_cnt[threadIdx.x] = S.piece_count[threadIdx.x];
  }
  __syncthreads();
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_lines; i += size_t(gridDim.x) * blockDim.x) {
    const avdb_vcf_line L = lines[i];
    int owner;
    if (L.flags & AVDB_VCF_COMMENT) {
      owner = -1;  // no output on any rank (load_vcf_file.py:103)
    } else if ((L.flags & kUnplaced) || L.chrom >= uint32_t(S.n_chrom)) {
      owner = 0;
    } else {
      const uint32_t c = L.chrom;
      uint32_t k = L.pos ? (L.pos - 1u) / S.cut : 0u;
      if (k >= s_cnt[c]) k = s_cnt[c] - 1u;  // past the contig end: its last piece
      owner = s_rank[s_base[c] + k];
    }
    sel[i] = owner == S.rank ? uint64_t(L.len) + 1u : 0ull;
  }
}

__global__ __launch_bounds__(kBlock) void k_vcf_select_copy(const uint8_t* __restrict__ text, size_t n_lines,
                                                            const avdb_vcf_line* __restrict__ lines,
                                                            const uint64_t* __restrict__ sel_off,
                                                            uint8_t* __restrict__ out) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_lines; i += size_t(gridDim.x) * blockDim.x) {
    const uint64_t o = sel_off[i];
    if (sel_off[i + 1] == o) continue;
    const avdb_vcf_line& L = lines[i];
    const uint8_t* s = text + L.start;
    uint32_t k = 0;
    // 8 bytes at a time (unaligned global_load/store_dwordx2: gfx950 unaligned mode)
    for (; k + 8 <= L.len; k += 8)
      reinterpret_cast<U64u*>(out + o + k)->v = reinterpret_cast<const U64u*>(s + k)->v;
    for (; k < L.len; ++k) out[o + k] = s[k];
    out[o + L.len] = '\n';
  }
}

}  // namespace avdb

using namespace avdb;

extern "C" int avdb_shard_workspace_size(size_t n_lines, size_t* bytes) {
  if (!bytes) return AVDB_EINVAL;
  *bytes = (scan::workspace_bytes(n_lines + 1) + 255) & ~size_t(255);
  return AVDB_OK;
}

extern "C" int avdb_vcf_select_lines(avdb_ctx* ctx, size_t n_lines, const avdb_vcf_line* lines,
                                     const uint32_t* piece_base_host, const uint32_t* piece_count_host,
                                     const uint8_t* piece_rank_host, uint32_t n_pieces, uint32_t cut, int rank,
                                     void* workspace, size_t workspace_bytes, uint64_t* sel_off, void* stream) {
  if (!ctx || !sel_off || !piece_base_host || !piece_count_host || !piece_rank_host || (n_lines && !lines)) {
    avdb_set_error("avdb_vcf_select_lines: null argument");
    return AVDB_EINVAL;
  }
  if (n_pieces == 0 || n_pieces > uint32_t(kMaxPieces) || cut == 0) {
    avdb_set_error("avdb_vcf_select_lines: 1..%d pieces of nonzero width required", kMaxPieces);
    return AVDB_EINVAL;
  }
  ShardArgs S;
  memset(&S, 0, sizeof(S));
  for (int c = 0; c < ctx->tab.n; ++c) {
    if (piece_count_host[c] == 0 || piece_base_host[c] + piece_count_host[c] > n_pieces) {
      avdb_set_error("avdb_vcf_select_lines: contig %d has no pieces in the table", c);
      return AVDB_EINVAL;
    }
    S.piece_base[c] = piece_base_host[c];
    S.piece_count[c] = piece_count_host[c];
  }
  memcpy(S.piece_rank, piece_rank_host, n_pieces);
  S.cut = cut;
  S.n_chrom = ctx->tab.n;
  S.rank = rank;
  size_t need = 0;
  avdb_shard_workspace_size(n_lines, &need);
  if (!workspace || workspace_bytes < need) {
    avdb_set_error("avdb_vcf_select_lines: workspace of %zu bytes required", need);
    return AVDB_ERANGE;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* so = reinterpret_cast<unsigned long long*>(sel_off);
  AVDB_HIP_TRY(hipMemsetAsync(so + n_lines, 0, 8, s));
  if (n_lines == 0) return AVDB_OK;
  hipLaunchKernelGGL(k_vcf_select, dim3(stream_grid(n_lines, kBlock, 4096)), dim3(kBlock), 0, s, lines, n_lines, S,
                     so);
  AVDB_LAUNCH_CHECK("k_vcf_select");
  size_t tb = need;
  if (int e = scan::exclusive_u64(sel_off, sel_off, n_lines + 1, workspace, tb, s)) return e;
  return AVDB_OK;
}

extern "C" int avdb_vcf_select_copy(avdb_ctx* ctx, const uint8_t* text, size_t text_bytes, size_t n_lines,
                                    const avdb_vcf_line* lines, const uint64_t* sel_off, uint8_t* out,
                                    void* stream) {
  (void)text_bytes;
  if (!ctx || !sel_off || (n_lines && (!lines || !text || !out))) {
    avdb_set_error("avdb_vcf_select_copy: null argument");
    return AVDB_EINVAL;
  }
  if (n_lines == 0) return AVDB_OK;
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_vcf_select_copy, dim3(stream_grid(n_lines, kBlock, 4096)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), text, n_lines, lines, sel_off, out);
  AVDB_LAUNCH_CHECK("k_vcf_select_copy");
  return AVDB_OK;
}
