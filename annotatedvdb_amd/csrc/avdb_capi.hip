// C ABI plumbing: contexts, error reporting, and host-side formatting of the
// kernels' bin codes into the ltree text the reference returns
// (BinIndex.find_bin_index -> BinIndexRef.global_bin_path, bin_index.py:75;
// labels from generate_bin_index_references.py:54,60-61,74).
#include "avdb_internal.hpp"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

static thread_local char g_err[512] = "";

void avdb_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" int avdb_abi_version(void) { return AVDB_ABI_VERSION; }

extern "C" const char* avdb_last_error(void) { return g_err; }

extern "C" int avdb_device_count(int* n) {
  if (!n) return AVDB_EINVAL;
  int c = 0;
  AVDB_HIP_TRY(hipGetDeviceCount(&c));
  *n = c;
  return AVDB_OK;
}

extern "C" int avdb_ctx_create(int device, const uint32_t* chrom_len, int n_chrom, avdb_ctx** out) {
  if (!out || !chrom_len || n_chrom <= 0 || n_chrom > AVDB_MAX_CHROM) {
    avdb_set_error("avdb_ctx_create: need 1..%d chromosome lengths", AVDB_MAX_CHROM);
    return AVDB_EINVAL;
  }
  *out = nullptr;
  avdb_ctx* c = new (std::nothrow) avdb_ctx();
  if (!c) return AVDB_ENOMEM;
  memset(&c->tab, 0, sizeof(c->tab));
  c->device = device;
  c->d_seq_digest = nullptr;
  c->d_loc_tail = nullptr;
  c->has_digests = false;
  c->tab.n = n_chrom;
  uint32_t off = 0;
  for (int i = 0; i < n_chrom; ++i) {
    if (chrom_len[i] == 0) {
      delete c;
      avdb_set_error("avdb_ctx_create: chromosome %d has length 0", i);
      return AVDB_EINVAL;
    }
    c->tab.len[i] = chrom_len[i];
    c->tab.l8_off[i] = off;
    off += (chrom_len[i] + avdb::kL8Width - 1) / avdb::kL8Width;
  }
  c->tab.n_l8 = off;
  c->n_cu = 256;
  if (device >= 0) {
    int nd = 0;
    hipError_t e = hipGetDeviceCount(&nd);
    if (e != hipSuccess || device >= nd) {
      delete c;
      avdb_set_error("avdb_ctx_create: device %d not available (%d devices, %s)", device, nd,
                     hipGetErrorString(e));
      return AVDB_EHIP;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
      c->n_cu = cus;
  }
  // Grid knobs (the same kernels on other grids; tests/test_gpu_parity.py::
  // test_grid_knobs_parity runs each at a non-default value against the oracle).
  // K1 defaults from the on-device A/B (tools/k1_sweep.py, tools/k1_geom.py;
  // profiles/r01_k1_*.log): 512-thread workgroups x 4 per CU (32 waves, one
  // 24.7 KB LDS histogram per 8 waves), 2 lane-groups in flight, nontemporal
  // loads AND stores, grid-stride sweep (each workgroup step covers 4096
  // consecutive records, so a sorted batch still hits ~1 histogram bin per step):
  // 5.75 TB/s on C2 and 5.76 TB/s on C3 in back-to-back launches vs 5.45 / 5.33
  // for plain stores.
  c->k1_blocks_per_cu = 4;
  if (const char* s = getenv("AVDB_K1_BLOCKS_PER_CU")) {
    const int v = atoi(s);
    if (v >= 1 && v <= 64) c->k1_blocks_per_cu = v;
  }
  c->k2_blocks_per_cu = 4;
  if (const char* s = getenv("AVDB_K2_BLOCKS_PER_CU")) {
    const int v = atoi(s);
    if (v >= 1 && v <= 64) c->k2_blocks_per_cu = v;
  }
  // K4 (SHA-512, VALU-bound) persistent grid: its occupancy by default; fewer
  // workgroups leave CUs to a kernel running beside it on another stream
  c->k4_blocks_per_cu = 3;
  if (const char* s = getenv("AVDB_K4_BLOCKS_PER_CU")) {
    const int v = atoi(s);
    if (v >= 1 && v <= 3) c->k4_blocks_per_cu = v;
  }
  c->k4_grid = 0;  // avdb_ctx_set_option(AVDB_OPT_K4_GRID): workgroups, 0 = n_cu * k4_blocks_per_cu
  c->k7_grid = 0;  // avdb_ctx_set_option(AVDB_OPT_K7_GRID): workgroups, 0 = the compiled grid
  c->k7_raw_blocks = 256;
  if (const char* s = getenv("AVDB_K7_RAW_BLOCKS")) c->k7_raw_blocks = size_t(strtoull(s, nullptr, 10));
  *out = c;
  return AVDB_OK;
}

extern "C" int avdb_ctx_set_option(avdb_ctx* ctx, int option, int64_t value) {
  if (!ctx) { avdb_set_error("null context"); return AVDB_EINVAL; }
  switch (option) {
    case AVDB_OPT_K4_GRID:
      if (value < 0 || value > 65536) {
        avdb_set_error("avdb_ctx_set_option: K4 grid of %lld workgroups out of range", (long long)value);
        return AVDB_EINVAL;
      }
      ctx->k4_grid = int(value);
      return AVDB_OK;
    case AVDB_OPT_K7_GRID:
      if (value < 0 || value > (int64_t(1) << 24)) {
        avdb_set_error("avdb_ctx_set_option: K7 grid of %lld workgroups out of range", (long long)value);
        return AVDB_EINVAL;
      }
      ctx->k7_grid = int(value);
      return AVDB_OK;
    default:
      avdb_set_error("avdb_ctx_set_option: unknown option %d", option);
      return AVDB_EINVAL;
  }
}

extern "C" int avdb_ctx_destroy(avdb_ctx* ctx) {
  if (!ctx) return AVDB_OK;
  if (ctx->d_seq_digest) {
    (void)hipSetDevice(ctx->device);
    (void)hipFree(ctx->d_seq_digest);
  }
  if (ctx->d_loc_tail) {
    (void)hipSetDevice(ctx->device);
    (void)hipFree(ctx->d_loc_tail);
  }
  delete ctx;
  return AVDB_OK;
}

extern "C" int avdb_ctx_n_chrom(const avdb_ctx* ctx) { return ctx ? ctx->tab.n : AVDB_EINVAL; }

extern "C" int avdb_l8_bin_count(const avdb_ctx* ctx, uint32_t* n_bins) {
  if (!ctx || !n_bins) return AVDB_EINVAL;
  *n_bins = ctx->tab.n_l8;
  return AVDB_OK;
}

extern "C" int avdb_ctx_set_sequence_digests(avdb_ctx* ctx, const char* digests, int n_chrom) {
  if (!ctx || !digests || n_chrom != ctx->tab.n) {
    avdb_set_error("avdb_ctx_set_sequence_digests: need one 32-char digest per chromosome");
    return AVDB_EINVAL;
  }
  AVDB_HIP_TRY(hipSetDevice(ctx->device));
  if (!ctx->d_seq_digest)
    AVDB_HIP_TRY(hipMalloc(&ctx->d_seq_digest, size_t(AVDB_MAX_CHROM) * AVDB_DIGEST_CHARS));
  AVDB_HIP_TRY(hipMemcpy(ctx->d_seq_digest, digests, size_t(n_chrom) * AVDB_DIGEST_CHARS,
                         hipMemcpyHostToDevice));
  std::vector<uint64_t> tail;
  avdb::location_tail_table(digests, n_chrom, tail);
  if (!ctx->d_loc_tail)
    AVDB_HIP_TRY(hipMalloc(&ctx->d_loc_tail, size_t(AVDB_MAX_CHROM) * 19 * 16 * sizeof(uint64_t)));
  AVDB_HIP_TRY(hipMemcpy(ctx->d_loc_tail, tail.data(), tail.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  ctx->has_digests = true;
  return AVDB_OK;
}

// ---- formatting ----------------------------------------------------------
static const char* const kChromNames[25] = {"1",  "2",  "3",  "4",  "5",  "6",  "7",
                                            "8",  "9",  "10", "11", "12", "13", "14",
                                            "15", "16", "17", "18", "19", "20", "21",
                                            "22", "X",  "Y",  "M"};

static inline int put_uint(char* p, uint32_t v) {
  char t[10];
  int k = 0;
  do { t[k++] = char('0' + v % 10); v /= 10; } while (v);
  for (int i = 0; i < k; ++i) p[i] = t[k - 1 - i];
  return k;
}

// Writes the path into p (caller guarantees AVDB_MAX_PATH bytes); returns length.
static int format_path(int n_chrom, uint8_t chrom, uint32_t code, char* p) {
  if (code == AVDB_BIN_NONE || chrom >= n_chrom) return -1;
  int k = 0;
  p[k++] = 'c'; p[k++] = 'h'; p[k++] = 'r';
  if (chrom < 25) {
    for (const char* s = kChromNames[chrom]; *s; ++s) p[k++] = *s;
  } else {
    k += put_uint(p + k, chrom);  // contigs beyond the human 25: numeric label
  }
  const uint32_t level = code >> 28, g = code & 0x0FFFFFFFu;
  if (level > 13) return -1;
  for (uint32_t l = 1; l <= level; ++l) {
    const uint32_t gl = g >> (level - l);
    const uint32_t b = l == 1 ? gl + 1 : (gl & 1u) + 1;
    p[k++] = '.'; p[k++] = 'L';
    k += put_uint(p + k, l);
    p[k++] = '.'; p[k++] = 'B';
    k += put_uint(p + k, b);
  }
  return k;
}

extern "C" int avdb_format_bin_path(const avdb_ctx* ctx, uint8_t chrom, uint32_t code, char* out,
                                    size_t cap) {
  if (!ctx || !out) return AVDB_EINVAL;
  char buf[AVDB_MAX_PATH];
  const int k = format_path(ctx->tab.n, chrom, code, buf);
  if (k < 0) { avdb_set_error("unmappable bin code"); return AVDB_EINVAL; }
  if (size_t(k) > cap) return AVDB_ERANGE;
  memcpy(out, buf, size_t(k));
  if (size_t(k) < cap) out[k] = '\0';
  return k;
}

extern "C" int avdb_format_bin_paths(const avdb_ctx* ctx, const uint8_t* chrom, const uint32_t* code,
                                     size_t n, char* out, size_t cap, uint64_t* out_off) {
  if (!ctx || (n && (!chrom || !code || !out_off))) return AVDB_EINVAL;
  size_t pos = 0;
  char buf[AVDB_MAX_PATH];
  for (size_t i = 0; i < n; ++i) {
    out_off[i] = pos;
    int k = format_path(ctx->tab.n, chrom[i], code[i], buf);
    if (k < 0) k = 0;  // unmappable -> empty string; caller checks status
    if (pos + size_t(k) > cap) { avdb_set_error("avdb_format_bin_paths: output too small"); return AVDB_ERANGE; }
    memcpy(out + pos, buf, size_t(k));
    pos += size_t(k);
  }
  out_off[n] = pos;
  return AVDB_OK;
}

extern "C" int avdb_host_alloc(size_t bytes, void** ptr) {
  if (!ptr || bytes == 0) {
    avdb_set_error("avdb_host_alloc: null pointer or zero size");
    return AVDB_EINVAL;
  }
  *ptr = nullptr;
  AVDB_HIP_TRY(hipHostMalloc(ptr, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  return AVDB_OK;
}

extern "C" int avdb_host_free(void* ptr) {
  if (ptr) AVDB_HIP_TRY(hipHostFree(ptr));
  return AVDB_OK;
}
