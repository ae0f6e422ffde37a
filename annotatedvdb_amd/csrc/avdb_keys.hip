// K5a avdb_display_attributes (display-attribute JSON of a record batch) and K7
// avdb_primary_keys (primary keys + ltree bin paths of a record batch) (gfx950).
#include "avdb_fmt.hpp"

#include <hipcub/hipcub.hpp>
#include <string.h>

namespace avdb {

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

}  // namespace avdb

using namespace avdb;

static size_t scan_bytes(size_t n) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, static_cast<const unsigned long long*>(nullptr),
                                         static_cast<unsigned long long*>(nullptr), n);
  return (t + 255) & ~size_t(255);
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
