// K8 avdb_small_prep: the per-record drop-in path in one launch (gfx950).
#include "avdb_fmt.hpp"

#include <string.h>

namespace avdb {

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

static int check_small_batch(const char* fn, const void* ctx, const avdb_small_batch* b) {
  if (!ctx || !b || !b->chrom || !b->pos || !b->end_out || !b->code || !b->status || !b->off_out ||
      !b->overflow || (!b->end_in && !b->ref_len)) {
    avdb_set_error("%s: null argument", fn);
    return AVDB_EINVAL;
  }
  if (b->ref_len && (!b->allele_off || !b->alt_len || !b->heap || !b->key_state || !b->disp_state)) {
    avdb_set_error("%s: alleles need allele_off, alt_len, heap, key_state and disp_state", fn);
    return AVDB_EINVAL;
  }
  if ((b->want & (AVDB_SMALL_KEY | AVDB_SMALL_DISPLAY)) && !b->ref_len) {
    avdb_set_error("%s: keys and display attributes need alleles", fn);
    return AVDB_EINVAL;
  }
  for (int k = 0; k < 3; ++k)
    if ((b->want & (1u << k)) && !b->text_out[k]) {
      avdb_set_error("%s: text stream %d requested without a buffer", fn, k);
      return AVDB_EINVAL;
    }
  if (b->n > AVDB_SMALL_MAX) {
    avdb_set_error("%s: at most %d records", fn, AVDB_SMALL_MAX);
    return AVDB_EINVAL;
  }
  return AVDB_OK;
}

extern "C" int avdb_small_prep(avdb_ctx* ctx, const avdb_small_batch* b, void* stream) {
  if (int rc = check_small_batch("avdb_small_prep", ctx, b)) return rc;
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

// ---------------------------------------------------------------------------
// K8h: the same per-record work for a call that arrives one record / one VCF
// line at a time (BinIndex.find_bin_index, VCFVariantLoader.parse_variant —
// the reference's own calling pattern, bin_index.py:59-75,
// vcf_variant_loader.py:351-391).  A GPU launch plus a stream sync costs more
// than the whole reference call (~1 us per record of arithmetic), so the
// per-call entry runs the kernels' record arithmetic (infer_end, classify,
// bin_path, display_json: the AVDB_HD definitions K2/K7/K8 compile) in the
// library's host code.  Batches go to the kernels.
// ---------------------------------------------------------------------------
namespace {

// ':' (the reference's metaseq split raises ValueError) or a non-ASCII byte
inline bool host_key_allele_ok(const uint8_t* s, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if ((s[i] & 0x80u) || s[i] == ':') return false;
  return true;
}

inline bool host_ascii(const uint8_t* s, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (s[i] & 0x80u) return false;
  return true;
}

}  // namespace

extern "C" int avdb_small_prep_host(const avdb_ctx* ctx, const avdb_small_batch* b) {
  if (int rc = check_small_batch("avdb_small_prep_host", ctx, b)) return rc;
  const uint32_t n = b->n;
  const Heap hp = make_heap(b->heap, b->heap ? b->heap_bytes : 0);
  uint32_t run[3] = {0, 0, 0};
  uint32_t ov = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t c = b->chrom[i], p = b->pos[i];
    uint32_t e, cd = AVDB_BIN_NONE, r = 0, a = 0;
    uint64_t o = 0, x = 0;
    uint8_t kst = AVDB_KEY_HOST, dst = 1;
    bool fits = true;
    if (b->ref_len) {
      o = b->allele_off[i];
      r = b->ref_len[i];
      a = b->alt_len[i];
      x = b->ext_id ? b->ext_id[i] : 0ull;
      fits = o <= b->heap_bytes && uint64_t(r) + a <= b->heap_bytes - o;
    }
    if (b->end_in) {
      e = b->end_in[i];
    } else {
      const bool snv = r == 1u && a == 1u;
      uint32_t l;
      e = infer_end(hp, o, r, a, p, snv ? 0 : heap_u64(hp, o), snv ? 0 : heap_u64(hp, o + r), &l);
    }
    const uint8_t st = uint8_t(classify(c, p, e, ctx->tab.n, ctx->tab.len, &cd));
    b->end_out[i] = e;
    b->code[i] = cd;
    b->status[i] = st;
    const uint8_t* ref = fits && b->heap ? b->heap + o : nullptr;
    if (b->ref_len) {
      const bool ascii = fits && host_ascii(ref, r + a);
      dst = fits ? (ascii ? 0 : 1) : 2;
      if (c >= 25 || (x >> 63) || !ascii) kst = AVDB_KEY_HOST;
      else if (uint64_t(r) + a > b->max_seq_len) kst = AVDB_KEY_NEED_DIGEST;
      else if (!host_key_allele_ok(ref, r + a)) kst = AVDB_KEY_HOST;
      else kst = AVDB_KEY_OK;
      b->key_state[i] = kst;
      b->disp_state[i] = dst;
    }
    for (int sidx = 0; sidx < 3; ++sidx) {
      if (!(b->want & (1u << sidx))) continue;
      uint32_t* offs = b->off_out + size_t(sidx) * (n + 1);
      offs[i] = run[sidx];
      bool emit = true;
      if (sidx == 0) emit = cd != AVDB_BIN_NONE && c < 25;
      if (sidx == 1) emit = kst == AVDB_KEY_OK;
      if (sidx == 2) emit = dst == 0;
      if (!emit) continue;
      auto render = [&](HostOut o_) -> HostOut {
        if (sidx == 0) return bin_path(o_, c, cd);
        if (sidx == 1) {
          chrom_name(o_, c);
          o_.put(':');
          o_.u32v(p);
          o_.put(':');
          o_.bytes(ref, r);
          o_.put(':');
          o_.bytes(ref + r, a);
          if (x) {
            o_.lit(":rs");
            o_.u64v(x);
          }
          return o_;
        }
        return display_json<true>(o_, c, p, e, ref, r, ref + r, a);
      };
      const uint32_t len = render(HostOut(nullptr, 0)).size();
      if (uint64_t(run[sidx]) + len > b->text_cap[sidx]) ov |= 1u << sidx;
      if (!(ov & (1u << sidx))) render(HostOut(b->text_out[sidx], run[sidx]));
      run[sidx] += len;
    }
  }
  for (int sidx = 0; sidx < 3; ++sidx)
    if (b->want & (1u << sidx)) b->off_out[size_t(sidx) * (n + 1) + n] = run[sidx];
  *b->overflow = ov;
  return AVDB_OK;
}

// K1h: one interval's smallest enclosing bin and its ltree path on the host — a
// BinIndex.find_bin_index cache miss (bin_index.py:43-56,75), the reference's
// per-call SQL round trip.  classify + bin_path are K1/K7's AVDB_HD definitions.
extern "C" int avdb_bin_path_host(const avdb_ctx* ctx, uint8_t chrom, uint32_t start, uint32_t end,
                                  uint32_t* code, uint8_t* status, char* out, size_t cap) {
  if (!ctx || !code || !status || (!out && cap)) {
    avdb_set_error("avdb_bin_path_host: null argument");
    return AVDB_EINVAL;
  }
  uint32_t cd;
  *status = uint8_t(classify(chrom, start, end, ctx->tab.n, ctx->tab.len, &cd));
  *code = cd;
  if (cd == AVDB_BIN_NONE || chrom >= 25) return 0;
  const uint32_t len = bin_path(HostOut(nullptr, 0), chrom, cd).size();
  if (len > cap) {
    avdb_set_error("avdb_bin_path_host: %u bytes needed", len);
    return AVDB_ERANGE;
  }
  bin_path(HostOut(reinterpret_cast<uint8_t*>(out), 0), chrom, cd);
  return int(len);
}

// K8a: one VariantAnnotator (variant_annotator.py:21-241) on the host — the
// drop-in class the reference constructs per alt allele (vcf_parser.py:225-231).
// infer_end (K2) and display_shape / display_allele_text / sequence_allele_text
// (K5a) are the kernels' AVDB_HD definitions; the end is returned relative to the
// position (infer_end at pos 0, as int32), so the caller's integer position is
// never narrowed.
extern "C" int avdb_annotate_host(const avdb_ctx* ctx, const uint8_t* alleles, uint32_t r, uint32_t a,
                                  uint32_t pos, int want_display, avdb_annotation* out, char* text, size_t cap) {
  if (!ctx || !out || (!alleles && uint64_t(r) + a) || (!text && cap)) {
    avdb_set_error("avdb_annotate_host: null argument");
    return AVDB_EINVAL;
  }
  const uint64_t n = uint64_t(r) + a;
  const Heap hp = make_heap(alleles, size_t(n));
  const bool snv = r == 1u && a == 1u;
  uint32_t lcp;
  const uint32_t rel = infer_end(hp, 0, r, a, 0u, snv ? 0 : heap_u64(hp, 0), snv ? 0 : heap_u64(hp, r), &lcp);
  memset(out, 0, sizeof(*out));
  out->end_rel = int32_t(rel);
  out->lcp = lcp;
  out->state = 2;
  if (!want_display) return AVDB_OK;
  // display coordinates pos, pos + 1 and the end stay in u32 (VCF positions do);
  // a non-ASCII allele is outside the byte-level contract
  if (!host_ascii(alleles, uint32_t(n)) || uint64_t(pos) + n + 2 > 0xFFFFFFFFull ||
      int64_t(pos) + int32_t(rel) < 0) {
    out->state = 1;
    return AVDB_OK;
  }
  const uint8_t* alt = alleles + r;
  const DisplayShape<const uint8_t*> d = display_shape(pos, pos + rel, alleles, r, alt, a);
  out->location_start = d.ls;
  out->location_end = d.le;
  out->variant_class = d.cls == 5 ? (d.dup ? AVDB_VC_DUPLICATION : AVDB_VC_INSERTION)
                                  : (d.cls == 6 ? AVDB_VC_DELETION : uint32_t(d.cls));
  HostOut c0(nullptr, 0), c1(nullptr, 0);
  display_allele_text<false>(c0, d, alleles, r, alt, a);
  sequence_allele_text<false>(c1, d, alleles, r, alt, a);
  out->display_bytes = c0.size();
  out->sequence_bytes = c1.size();
  if (uint64_t(c0.size()) + c1.size() > cap) {
    avdb_set_error("avdb_annotate_host: %u bytes needed", c0.size() + c1.size());
    return AVDB_ERANGE;
  }
  HostOut w0(reinterpret_cast<uint8_t*>(text), 0), w1(reinterpret_cast<uint8_t*>(text), c0.size());
  display_allele_text<false>(w0, d, alleles, r, alt, a);
  sequence_allele_text<false>(w1, d, alleles, r, alt, a);
  out->state = 0;
  return AVDB_OK;
}
